#!/bin/bash
# round 4: config 5's hybrid tiled layout (bucket 0 in LDS-window tiles, one load round;
# buckets 1..3 by list in the same launch): parity, cold A/B against the ordered layout and
# two build variants, HBM counters. Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04/h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py tests/test_gpu_batches.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=$R/gnn-track-finding_amd/gtf
for i in 1 2; do
  for t in 0 256 128; do
    GTF_KL_TILE=$t timeout -k 10 120 python tools/pkl_time.py 48 >> $O/kl_ab.jsonl || exit 1
  done
  GTF_KL_TILE_B1=0 GTF_KL_TILE=256 timeout -k 10 120 python tools/pkl_time.py 48 >> $O/kl_ab.jsonl || exit 1
  for v in klw4 klw768; do
    GTF_LIB=$L/libgtf_$v.so GTF_KL_TILE=256 timeout -k 10 120 python tools/pkl_time.py 48 >> $O/kl_ab.jsonl || exit 1
  done
done
cat $O/kl_ab.jsonl
cd /tmp && export TMPDIR=/tmp
for t in 0 256; do
  GTF_KL_TILE=$t timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/$O/kl$t/stats -o run --output-format csv -- python3 $R/tools/pkl_time.py 48 > $R/$O/kl$t.stats.log 2>&1 || exit 1
  GTF_KL_TILE=$t timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$O/kl$t/fetch -o run --output-format csv -- python3 $R/tools/pkl_time.py 24 > $R/$O/kl$t.fetch.log 2>&1 || exit 1
  GTF_KL_TILE=$t timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$O/kl$t/write -o run --output-format csv -- python3 $R/tools/pkl_time.py 24 > $R/$O/kl$t.write.log 2>&1 || exit 1
done
echo r04h-done
