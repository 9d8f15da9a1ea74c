#!/bin/bash
# round 5: k_extrapolate as load / compute / store (default), two slots per thread with their
# arithmetic interleaved (p2: 162 VGPRs, 3 waves; p2w4: 4 waves, 42 VGPRs spilled), against
# the previous single-body form (head)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NO_TESTS=1 bash tools/gpu_ab_env.sh r05/pair 2 head=libgtf_head.so m=libgtf.so p2=libgtf_p2.so p2w4=libgtf_p2w4.so || exit 1
for v in libgtf.so libgtf_p2.so; do
  GTF_LIB=$R/gnn-track-finding_amd/gtf/$v timeout -k 10 400 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_synthetic.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05/pair/$v.tests.log 2>&1
  echo "$v tests rc=$?: $(tail -1 gpurun_out/r05/pair/$v.tests.log)"
done
echo pair-done
