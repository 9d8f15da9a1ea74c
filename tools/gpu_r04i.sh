#!/bin/bash
# round 4: config 5 ordered layout, cold -- build variants (NPT_ORD 2 / 3, waves 4 / 6, 128-thread
# blocks), the bucket-0 launch alone, and bucket 0 without its dependent round (diagnostics)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04/i
mkdir -p $O
L=$R/gnn-track-finding_amd/gtf
timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in npt2 npt3 rcp rcpnpt2; do
  GTF_LIB=$L/libgtf_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for i in 1; do
  for v in libgtf libgtf_npt2 libgtf_npt3 libgtf_rcp libgtf_rcpnpt2 libgtf_klwv6 libgtf_klwv4 libgtf_klb128; do
    GTF_LIB=$L/$v.so timeout -k 10 120 python tools/pkl_time.py 48 >> $O/kl_ab.jsonl || exit 1
  done
  for keep in 0 123; do
    GTF_KL_KEEP=$keep timeout -k 10 120 python tools/pkl_time.py 48 | sed "s/^{/{\"keep\": \"$keep\", /" >> $O/kl_ab.jsonl || exit 1
    GTF_LIB=$L/libgtf_nodep.so GTF_KL_KEEP=$keep timeout -k 10 120 python tools/pkl_time.py 48 | sed "s/^{/{\"keep\": \"$keep\", /" >> $O/kl_ab.jsonl || exit 1
  done
done
cat $O/kl_ab.jsonl
PROG="tools/pkl_time.py 24" bash tools/gpu_sqmix.sh r04/i/sq_pkl || exit 1
echo r04i-done
