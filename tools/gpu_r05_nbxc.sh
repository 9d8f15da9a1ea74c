#!/bin/bash
# round 5: smaller node-kernel blocks with the same XCD locality (128 threads in runs of 8,
# 64 threads in runs of 16) against 256 threads in runs of 4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NO_TESTS=1 bash tools/gpu_ab_env.sh r05/nbxc 2 b256c4=libgtf.so b128c8=libgtf_b128c8.so b64c16=libgtf_b64c16.so || exit 1
for v in libgtf_b128c8.so libgtf_b64c16.so; do
  GTF_LIB=$R/gnn-track-finding_amd/gtf/$v timeout -k 10 400 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05/nbxc/$v.tests.log 2>&1
  echo "$v tests rc=$?: $(tail -1 gpurun_out/r05/nbxc/$v.tests.log)"
done
echo nbxc-done
