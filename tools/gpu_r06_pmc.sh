#!/bin/bash
# round 6, second closing call: the HBM counters of C4 and C3 (separate FETCH_SIZE /
# WRITE_SIZE passes, corrected by the committed calibration), the SQ instruction mix of the
# C4 pass, then the N > 1 bench path rehearsed with 4 gloo ranks sharing the one GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NAME=r06/${TAG:-final}
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
if [ -z "$NO_PMC" ]; then
  bash tools/gpu_profile.sh gpurun_out/$NAME/c4 --no-c5 --no-c3 --no-dropin --steps 20 --warmup 3 > /dev/null || { echo "c4 pmc failed"; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/$NAME/c4 profiles/r01_pmc/calib gpurun_out/$NAME/c4/pmc_c4.json c4 | tail -8 || exit 1
  bash tools/gpu_profile.sh gpurun_out/$NAME/c3 --workload c3 --no-c5 --no-dropin --steps 10 --warmup 2 > /dev/null || { echo "c3 pmc failed"; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/$NAME/c3 profiles/r01_pmc/calib gpurun_out/$NAME/c3/pmc_c3.json c3 | tail -8 || exit 1
  bash tools/gpu_sqmix.sh $NAME/sqmix > /dev/null 2>&1 || { echo "sqmix failed"; exit 1; }
  grep -A22 "k_node_multi<11" $OUT/sqmix/sqmix.txt | head -24
fi
if [ -z "$NO_GLOO" ]; then
  timeout -k 10 600 python -u bench.py --gpus 4 --backend gloo --steps 10 --warmup 2 --no-cpu --no-dropin > $OUT/bench_gpus4_gloo_one_gpu.json 2> $OUT/bench_gpus4_gloo.err || { tail -20 $OUT/bench_gpus4_gloo.err; exit 1; }
  python3 - <<PY
import json
d=json.loads(open('$OUT/bench_gpus4_gloo_one_gpu.json').read().strip().splitlines()[-1])
s=d.get('sharded_single_event') or {}
print('n_gpus', d['n_gpus'], 'ms', s.get('ms_per_step'), 'phase', s.get('rank0_phase_ms'), 'a2a', s.get('alltoall_ms'), 'speedup', s.get('speedup_vs_one_gpu'))
PY
fi
echo r06-pmc-done
