#!/bin/bash
# config 5 cold: non-temporal stores / loads of the once-touched streams (GTF_KL_NT builds)
set -o pipefail
O=gpurun_out/kl_nt
mkdir -p $O
for i in 1 2; do
  for nt in 0 1 3 7; do
    if [ $nt = 0 ]; then unset GTF_LIB; else export GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_nt$nt.so; fi
    timeout -k 10 120 python tools/pkl_time.py 48 --f32 | sed "s/^/{\"nt\":$nt,\"r\":/; s/\$/}/" >> $O/ab.jsonl || exit 1
  done
done
cat $O/ab.jsonl
