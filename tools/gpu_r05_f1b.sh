#!/bin/bash
# round 5: the fused phase 1b with the scan's operands handed to the extrapolation (only the
# slot's own fields loaded again): the world-8 sharded tests (both phase-1b forms) and the
# rank-0 phase times with each form
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r05/f1b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_c4.py tests/test_gpu_comm_native.py -m gpu -v --timeout 500 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; grep -E "^FAILED|^ERROR" $OUT/pytest.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/shard_pass_time.py 1 2 4 8 --json > $OUT/two_launch.log 2>&1 || { tail -20 $OUT/two_launch.log; exit 1; }
grep "^N=" $OUT/two_launch.log | cut -c1-160
GTF_SHARD_FUSED_1B=1 timeout -k 10 300 python -u tools/shard_pass_time.py 1 2 4 8 --json > $OUT/fused.log 2>&1 || { tail -20 $OUT/fused.log; exit 1; }
grep "^N=" $OUT/fused.log | cut -c1-160
echo f1b-done
