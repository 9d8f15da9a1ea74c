#!/bin/bash
# round 5: k_extrapolate's predicated gathers, the sender's unchanged-carry store skipped and
# two out-edge chunks per round of loads in the chunked sender scan (default build m5)
# against the same without the chunks (c1), the previous form (np), the reciprocal-product
# quotients (xf) and the recomputed block inverses (i2); the decision-sensitive tests on m5
# and xf; then the sharded tests and rank-0 phase times with the fused phase 1b
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NO_TESTS=1 bash tools/gpu_ab_env.sh r05/ab2 2 m5=libgtf.so tp0=libgtf.so,GTF_TAG_POLL=0 c1=libgtf_c1.so np=libgtf_np.so xf=libgtf_xf.so i2=libgtf_i2.so || exit 1
OUT=$R/gpurun_out/r05/ab2
for v in libgtf.so libgtf_xf.so; do
  GTF_LIB=$R/gnn-track-finding_amd/gtf/$v timeout -k 10 400 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_synthetic.py tests/test_gpu_layouts.py tests/test_gpu_devmem.py -x -q --timeout 200 --timeout-method thread > $OUT/$v.tests.log 2>&1
  rc=$?
  echo "$v tests rc=$rc: $(tail -1 $OUT/$v.tests.log)"
  [ $rc -ne 0 ] && [ $v = libgtf.so ] && exit 1
done
# (the sharded tests and phase times: tools/gpu_r05_shard.sh, a call of its own)
echo ab2-done
