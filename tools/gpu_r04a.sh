#!/bin/bash
# round 4: parity of the live-coordinate / static-class node kernel, then per-kernel rocprofv3
# durations with the graph-static classes on and off (GTF_NO_CLASSES=1), two alternating rounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c4_digest.py tests/test_gpu_fullsize.py tests/test_dropin.py tests/test_gpu_synthetic.py tests/test_gpu_layouts.py tests/test_gpu_edges.py tests/test_gpu_comm_native.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/gpu_abv.sh r04/a/abv 2 libgtf.so libgtf_early.so libgtf_lean.so libgtf_w5.so || exit 1
# the split step captured as hipGraphs: once, its own time limit
(GTF_SPLIT_GRAPH=1 timeout -k 10 180 python3 -u tools/split_time.py 5 1 > $OUT/split_graph.log 2>&1; echo "split_graph rc=$?" >> $OUT/split_graph.log)
tail -5 $OUT/split_graph.log
echo r04a-done
