#!/bin/bash
# round 4: config 5 with the 3..4-edge bucket on 4-lane groups (LDS-staged, 70 VGPRs) so the
# launch fits 6 / 7 waves per SIMD without spills, cold, against the default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04/p
mkdir -p $O
L=$R/gnn-track-finding_amd/gtf
for v in b1l7 b1l6; do
  GTF_LIB=$L/libgtf_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parabolic.py tests/test_gpu_batches.py -x -q -k "not ordered_layout_equals_lists" --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for i in 1 2 3; do
  for v in libgtf libgtf_b1l5 libgtf_b1l6 libgtf_b1l7; do
    GTF_LIB=$L/$v.so timeout -k 10 120 python tools/pkl_time.py 48 >> $O/kl_ab.jsonl || exit 1
  done
done
python3 -c "
import json, collections
d = collections.defaultdict(list)
for l in open('$O/kl_ab.jsonl'):
    r = json.loads(l); d[r['lib'].split('/')[-1]].append(round(r['f64_ms'] * 1e3, 2))
print(dict(d))"
echo r04p-done
