#!/bin/bash
# config 5: bucket 0 in its own launch on a side stream (GTF_KL_SPLIT=1) vs one launch,
# parity first, then cold timings alternating (b0 kernel at 8 waves, and 6 / 10 builds)
set -o pipefail
O=gpurun_out/kl_split
mkdir -p $O
GTF_KL_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py tests/test_gpu_batches.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  GTF_KL_SPLIT=0 timeout -k 10 120 python tools/pkl_time.py 48 --f32 | sed 's/^/{"split":0,"w":8,"r":/; s/$/}/' >> $O/ab.jsonl || exit 1
  GTF_KL_SPLIT=1 timeout -k 10 120 python tools/pkl_time.py 48 --f32 | sed 's/^/{"split":1,"w":8,"r":/; s/$/}/' >> $O/ab.jsonl || exit 1
  for w in 6 10; do
    GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_b0w$w.so GTF_KL_SPLIT=1 timeout -k 10 120 python tools/pkl_time.py 48 --f32 | sed "s/^/{\"split\":1,\"w\":$w,\"r\":/; s/\$/}/" >> $O/ab.jsonl || exit 1
  done
done
cat $O/ab.jsonl
