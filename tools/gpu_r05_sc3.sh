#!/bin/bash
# round 5: three out-edge chunks per round of loads in the chunked sender scan (77 VGPRs, 6
# waves per SIMD) against two (67 VGPRs, 7 waves)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NO_TESTS=1 bash tools/gpu_ab_env.sh r05/sc3 3 c2=libgtf.so c3=libgtf_sc3.so || exit 1
GTF_LIB=$R/gnn-track-finding_amd/gtf/libgtf_sc3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05/sc3/sc3.tests.log 2>&1
echo "sc3 tests rc=$?: $(tail -1 gpurun_out/r05/sc3/sc3.tests.log)"
echo sc3-done
