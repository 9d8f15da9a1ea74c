#!/bin/bash
# round 4: config 5 ordered layout with degree runs (buckets 1 / 2 by arithmetic): parity, cold
# A/B against the round-3 ordered form and the 4-lane bucket 1, each bucket alone
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04/j2
mkdir -p $O
L=$R/gnn-track-finding_amd/gtf
timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py tests/test_gpu_batches.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for keep in 0 1 2 12 123; do
  GTF_KL_KEEP=$keep timeout -k 10 120 python tools/pkl_time.py 48 | sed "s/^{/{\"keep\": \"$keep\", \"runs\": 1, /" >> $O/kl_ab.jsonl || exit 1
  GTF_KL_DEG_RUNS=0 GTF_KL_KEEP=$keep timeout -k 10 120 python tools/pkl_time.py 48 | sed "s/^{/{\"keep\": \"$keep\", \"runs\": 0, /" >> $O/kl_ab.jsonl || exit 1
done
cat $O/kl_ab.jsonl
echo r04j-done
