#!/bin/bash
# config-5 KL kernel: this build against the round-2 kernel source (gtf/ab/libgtf_r02kl.so),
# hot (one batch relaunched) and cold (8 batches rotated), alternating
set -o pipefail
O=gpurun_out/kl_ab
mkdir -p $O
for i in 1 2; do
  for lib in default gnn-track-finding_amd/gtf/ab/libgtf_r02kl.so; do
    if [ $lib = default ]; then unset GTF_LIB; else export GTF_LIB=$PWD/$lib; fi
    timeout -k 10 120 python tools/pkl_time.py 48 --hot >> $O/ab.jsonl || exit 1
    timeout -k 10 120 python tools/pkl_time.py 48 >> $O/ab.jsonl || exit 1
  done
done
cat $O/ab.jsonl
