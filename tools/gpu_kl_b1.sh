#!/bin/bash
# config 5 cold: the 3..4-edge bucket on 4-lane groups (GTF_KL_B1_LANES=1: 70 VGPRs, 6 / 7
# waves per SIMD) vs one thread per node (96 VGPRs, 5 waves)
set -o pipefail
O=gpurun_out/kl_b1
mkdir -p $O
GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_b1l_w7.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py -q -k "not ordered_layout_equals_lists" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in default 6 7; do
    if [ $v = default ]; then unset GTF_LIB; else export GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_b1l_w$v.so; fi
    timeout -k 10 120 python tools/pkl_time.py 48 --f32 | sed "s/^/{\"v\":\"$v\",\"r\":/; s/\$/}/" >> $O/ab.jsonl || exit 1
  done
done
cat $O/ab.jsonl
