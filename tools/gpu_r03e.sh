#!/bin/bash
# round 3: the LDS-window KL kernel (tiled layout): parity tests, cold A/B against the ordered
# layout, HBM counters. Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py tests/test_gpu_layouts.py tests/test_gpu_diagnostics.py tests/test_shard.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for t in 0 256 128; do
    GTF_KL_TILE=$t timeout -k 10 120 python tools/pkl_time.py 48 >> $O/kl_ab.jsonl || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for t in 0 256; do
  GTF_KL_TILE=$t timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$O/kl$t/fetch -o run --output-format csv -- python3 $R/tools/pkl_time.py 24 > $R/$O/kl$t.fetch.log 2>&1 || exit 1
  GTF_KL_TILE=$t timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$O/kl$t/write -o run --output-format csv -- python3 $R/tools/pkl_time.py 24 > $R/$O/kl$t.write.log 2>&1 || exit 1
done
echo r03e-done
