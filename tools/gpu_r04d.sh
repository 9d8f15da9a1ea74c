#!/bin/bash
# round 4: the whole GPU suite (world-8 shard tests included), then the capture bisection
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/d
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "suite rc=$?"; tail -3 $OUT/pytest_gpu.log; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20
bash tools/gpu_capture_bisect.sh
echo r04d-done
