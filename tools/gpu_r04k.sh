#!/bin/bash
# round 4: the capture-safe (linear) split step: parity, capture probes, then the captured
# split step timed against the one-stream pass. Stops at the first failure or crash.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04/k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 300 --timeout-method thread > $O/pytest_split.log 2>&1 || { tail -30 $O/pytest_split.log; exit 1; }
tail -1 $O/pytest_split.log
MODES="linear linstep" CAPTURE_TAG=_linear bash tools/gpu_capture_bisect.sh || exit 1
GTF_SPLIT_GRAPH=1 GTF_SPLIT_LINEAR=1 timeout -k 10 180 python3 -X faulthandler -u tools/split_time.py 20 3 > $O/split_graph_linear.log 2>&1 || { tail -20 $O/split_graph_linear.log; exit 1; }
grep '^{' $O/split_graph_linear.log
echo r04k-done
