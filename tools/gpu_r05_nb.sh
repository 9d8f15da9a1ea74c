#!/bin/bash
# round 5: the node kernels in 128- / 64-thread blocks (GTF_NODE_BLOCK; LDS 15.6 / 8.2 KB per
# block, still 5 waves per SIMD) against 256: a block's slots free only when its slowest
# wave ends; then the decision-sensitive tests on both
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NO_TESTS=1 bash tools/gpu_ab_env.sh r05/nb 2 b256=libgtf.so b128=libgtf_nb128.so b64=libgtf_nb64.so || exit 1
OUT=$R/gpurun_out/r05/nb
for v in libgtf_nb128.so libgtf_nb64.so; do
  GTF_LIB=$R/gnn-track-finding_amd/gtf/$v timeout -k 10 400 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $OUT/$v.tests.log 2>&1
  echo "$v tests rc=$?: $(tail -1 $OUT/$v.tests.log)"
done
echo nb-done
