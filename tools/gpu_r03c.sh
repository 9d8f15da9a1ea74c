#!/bin/bash
# round 3: tiled parabolic-KL layout (parity test + cold A/B against the ordered layout),
# per-kernel A/B of the out-order sender scan under rocprofv3. Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for t in 0 8748 4096 16384; do
    GTF_KL_TILE=$t timeout -k 10 120 python tools/pkl_time.py 48 >> $O/kl_ab.jsonl || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  GTF_NO_OUTIDX=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/outidx$v -o run --output-format csv -- python3 $R/tools/pass_loop.py 100 > $R/$O/outidx$v.log 2>&1 || exit 1
done
echo r03c-done
