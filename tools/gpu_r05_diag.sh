#!/bin/bash
# round 5: per-op wave timing of the node kernel with stamps inside the clustering (the
# GTF_OP_TIMING build), then the sharded C4 test at world 8 with both phase-1b forms
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r05/diag
mkdir -p $OUT
GTF_LIB=$R/gnn-track-finding_amd/gtf/libgtf_optime.so GTF_OPT_FLUSH=1 timeout -k 10 300 python -u tools/op_timing.py $OUT/op_timing.json > $OUT/op_timing.log 2>&1 || { tail -20 $OUT/op_timing.log; exit 1; }
python3 - <<PY
import json
d=json.load(open('$OUT/op_timing.json'))
print('span', round(d['kernel_span_us'],1), 'waves', d['waves'])
for G,v in d['by_G'].items():
    ph=v['phases_mean']; cs=v.get('cluster_split',{})
    print(G, 'waves', v['waves'], 'life', round(v['lifetime_mean']), 'load', round(ph.get('00_load',0)), 'cluster', round([x for k,x in ph.items() if 'cluster' in k][0]), {k: round(x) for k,x in cs.items()})
PY
timeout -k 10 600 python -u -m pytest "tests/test_gpu_shard_c4.py" -k "8" -v --timeout 500 --timeout-method thread > $OUT/shard8.log 2>&1
rc=$?; tail -3 $OUT/shard8.log; [ $rc -ne 0 ] && exit $rc
echo diag-done
