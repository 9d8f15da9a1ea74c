#!/bin/bash
# round 4: config 5 with bucket 0 in its own launch (8 / 10 waves per SIMD), the fused node
# kernel's early-stage builds, then the linear split step captured as hipGraphs (last: a
# capture crash ends the call). Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04/l
mkdir -p $O
L=$R/gnn-track-finding_amd/gtf
for v in splitb0 splitb0w10; do
  GTF_LIB=$L/libgtf_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for i in 1 2; do
  for v in libgtf libgtf_splitb0 libgtf_splitb0w10; do
    GTF_LIB=$L/$v.so timeout -k 10 120 python tools/pkl_time.py 48 >> $O/kl_ab.jsonl || exit 1
  done
done
cat $O/kl_ab.jsonl
bash tools/gpu_abv.sh r04/l/abv 2 libgtf.so libgtf_es1.so libgtf_es2.so || exit 1
GTF_SPLIT_GRAPH=1 GTF_SPLIT_LINEAR=1 timeout -k 10 180 python3 -X faulthandler -u tools/split_time.py 20 3 > $O/split_graph_linear.log 2>&1 || { tail -20 $O/split_graph_linear.log; exit 1; }
grep '^{' $O/split_graph_linear.log
echo r04l-done
