#!/bin/bash
# round 4: config 5 block order inside the one launch (GTF_KL_ORDER 1: bucket 0 first, 2:
# the other buckets spread among bucket 0's), cold, against the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04/n4
mkdir -p $O
L=$R/gnn-track-finding_amd/gtf
for v in mix50 mix75; do
  GTF_LIB=$L/libgtf_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for i in 1 2 3; do
  for v in libgtf libgtf_ord0 libgtf_mix50 libgtf_mix75; do
    GTF_LIB=$L/$v.so timeout -k 10 120 python tools/pkl_time.py 48 >> $O/kl_ab.jsonl || exit 1
  done
done
cat $O/kl_ab.jsonl
echo r04n-done
