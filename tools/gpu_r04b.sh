#!/bin/bash
# round 4: the whole GPU suite (world-8 shard tests included), then the PMC traffic passes of
# the default bench and the SQ instruction mix of the pass kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/gpu_profile.sh gpurun_out/r04/b/prof --steps 20 --warmup 3 --no-c5 --no-dropin || exit 1
python3 tools/pmc_summary.py $OUT/prof profiles/r01_pmc/calib $OUT/prof/pmc_c4.json c4 > $OUT/prof/pmc.txt || exit 1
cat $OUT/prof/pmc.txt | tail -8
bash tools/gpu_sqmix.sh r04/b/sqmix || exit 1
echo r04b-done
