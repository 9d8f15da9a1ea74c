#!/bin/bash
# config 5 cold: block size / waves per SIMD builds of k_parabolic_kl (GTF_KL_BLOCK, GTF_KL_WAVES)
set -o pipefail
O=gpurun_out/kl_sweep
mkdir -p $O
for i in 1 2; do
  for v in default 256_5 64_4 64_6 128_5; do
    if [ $v = default ]; then unset GTF_LIB; else export GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_kl_$v.so; fi
    timeout -k 10 120 python tools/pkl_time.py 48 --f32 | sed "s/^/{\"v\":\"$v\",\"r\":/; s/\$/}/" >> $O/ab.jsonl || exit 1
  done
done
cat $O/ab.jsonl
