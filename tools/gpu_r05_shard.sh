#!/bin/bash
# round 5: the sharded pass in phases (halo exchange beside phase 1a) -- the sharded GPU
# tests (gloo ranks sharing the GPU, the native RCCL world of one), then rank 0's share of
# the C4 pass at N = 1, 2, 4, 8 with its three phases timed alone.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/${TAG:-shard}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard_c4.py tests/test_shard.py tests/test_gpu_comm_native.py tests/test_gpu_shard_tags.py tests/test_gpu_split.py -m gpu -v --timeout 420 --timeout-method thread > $OUT/pytest_shard.log 2>&1
rc=$?
echo "shard tests rc=$rc"; tail -2 $OUT/pytest_shard.log; grep -E "^FAILED|^ERROR" $OUT/pytest_shard.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/shard_pass_time.py 1 2 4 8 --json > $OUT/shard_pass_time.log 2>&1 || { tail -20 $OUT/shard_pass_time.log; exit 1; }
grep "^N=" $OUT/shard_pass_time.log
echo shard-done
