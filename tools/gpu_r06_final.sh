#!/bin/bash
# round 6 closing run on the shipped build: the GPU suite, smoke(), the default bench line,
# the same command under rocprofv3 --kernel-trace --stats (+ the per-(kernel, grid) split
# of its C4 / C3 launches), the HBM counters of C4 and C3 (separate FETCH_SIZE / WRITE_SIZE
# passes, corrected by the committed calibration) and the SQ instruction mix of the C4 pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NAME=r06/${TAG:-final}
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
if [ -z "$NO_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "suite rc=$rc"; tail -1 $OUT/pytest_gpu.log; grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 - <<PY
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('c4', round(d['ms_per_step'],5), round(d['value']/1e9,3), d['kernel_ms'], round(d['roofline']['frac'],4))
c3=d.get('c3_fused_batch') or {}
print('c3', c3.get('ms_per_step'), c3.get('kernel_ms'), (c3.get('roofline') or {}).get('frac'))
c5=d.get('c5_parabolic_kl') or {}
print('c5', c5.get('f64',{}).get('kernel_ms'), c5.get('f64',{}).get('roofline',{}).get('frac'))
a16=(d.get('other_path_stages') or {}).get('a16_tag_propagation',{})
print('a16', {k:a16.get(k) for k in ('stage_wall_ms','prepare_call_ms','sweep_call_ms','sweeps','flips','stage_over_kernels')})
a16c3=c3.get('a16_tag_propagation') or {}
print('a16 c3', {k:a16c3.get(k) for k in ('stage_wall_ms','sweep_call_ms','sweeps','flips','frac_of_peak','stage_sweep')})
print('a16 c4 stage_sweep', a16.get('stage_sweep'))
print('cpu', d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline',{}).get('seconds'))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py > $OUT/bench_under_rocprof.json 2> $OUT/bench_under_rocprof.err || { tail -20 $OUT/bench_under_rocprof.err; exit 1; }
cd $R
python3 tools/kstats.py $OUT/prof final
python3 tools/kstats_by_grid.py $OUT/prof $OUT/kernel_stats_by_grid.csv --match=k_sender,k_extrapolate,k_node,k_tag,k_count,k_parabolic > $OUT/kstats_by_grid.txt; head -16 $OUT/kstats_by_grid.txt
python3 tools/kstats_c5.py $OUT/prof $OUT/bench_under_rocprof.json $OUT/kstats_c5_cold_hot.json
if [ -z "$NO_PMC" ]; then
  bash tools/gpu_profile.sh gpurun_out/$NAME/c4 --no-c5 --no-c3 --no-dropin --steps 20 --warmup 3 > /dev/null || { echo "c4 pmc failed"; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/$NAME/c4 profiles/r01_pmc/calib gpurun_out/$NAME/c4/pmc_c4.json c4 | tail -8 || exit 1
  bash tools/gpu_profile.sh gpurun_out/$NAME/c3 --workload c3 --no-c5 --no-dropin --steps 10 --warmup 2 > /dev/null || { echo "c3 pmc failed"; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/$NAME/c3 profiles/r01_pmc/calib gpurun_out/$NAME/c3/pmc_c3.json c3 | tail -8 || exit 1
  bash tools/gpu_sqmix.sh $NAME/sqmix > /dev/null 2>&1 || { echo "sqmix failed"; exit 1; }
  grep -A14 k_node $OUT/sqmix/sqmix.txt | head -16
fi
echo r06-final-done
