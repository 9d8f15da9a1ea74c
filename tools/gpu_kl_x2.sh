#!/bin/bash
# config 5: two bucket-0 nodes per thread (GTF_KL_B0X2 build): parity, then cold A/B
set -o pipefail
O=gpurun_out/kl_x2
mkdir -p $O
GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_x2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py tests/test_gpu_batches.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  unset GTF_LIB; timeout -k 10 120 python tools/pkl_time.py 48 --f32 | sed 's/^/{"v":"default","r":/; s/$/}/' >> $O/ab.jsonl || exit 1
  GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_x2.so timeout -k 10 120 python tools/pkl_time.py 48 --f32 | sed 's/^/{"v":"x2","r":/; s/$/}/' >> $O/ab.jsonl || exit 1
done
cat $O/ab.jsonl
