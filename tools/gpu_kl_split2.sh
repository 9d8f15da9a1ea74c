#!/bin/bash
# config 5 cold: bucket 0 in its own launch before the others, same stream (GTF_KL_SPLIT builds)
set -o pipefail
O=gpurun_out/kl_split2
mkdir -p $O
for i in 1 2; do
  for v in default 6 8 10; do
    if [ $v = default ]; then unset GTF_LIB; else export GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_split$v.so; fi
    timeout -k 10 120 python tools/pkl_time.py 48 --f32 | sed "s/^/{\"v\":\"$v\",\"r\":/; s/\$/}/" >> $O/ab.jsonl || exit 1
  done
done
cat $O/ab.jsonl
