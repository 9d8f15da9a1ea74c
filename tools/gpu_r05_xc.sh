#!/bin/bash
# round 5: the node kernel's blocks in runs of 2 / 4 / 8 consecutive work blocks per XCD
# (GTF_NODE_XCD_CHUNK, node_block_map) against dispatch order; then the decision-sensitive
# tests on the variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NO_TESTS=1 bash tools/gpu_ab_env.sh r05/xc 2 c1=libgtf.so c2=libgtf_xc2.so c4=libgtf_xc4.so c8=libgtf_xc8.so || exit 1
OUT=$R/gpurun_out/r05/xc
for v in libgtf_xc2.so libgtf_xc4.so libgtf_xc8.so; do
  GTF_LIB=$R/gnn-track-finding_amd/gtf/$v timeout -k 10 400 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $OUT/$v.tests.log 2>&1
  echo "$v tests rc=$?: $(tail -1 $OUT/$v.tests.log)"
done
echo xc-done
