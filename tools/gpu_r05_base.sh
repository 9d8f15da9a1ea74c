#!/bin/bash
# round 5 base run: the GPU suite, smoke(), the default bench line (C4 headline + C3 section +
# C5 + whole-event CPU baseline) and the same command under rocprofv3 --kernel-trace --stats,
# with the per-(kernel, grid) summary that separates the C4 launches from the C3 ones.
# Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/${TAG:-base}
mkdir -p $OUT
if [ -z "$NO_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "suite rc=$rc"; tail -2 $OUT/pytest_gpu.log; grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 - <<PY
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('c4', d['ms_per_step'], d['value']/1e9, d['kernel_ms'], round(d['roofline']['frac'],4))
c3=d.get('c3_fused_batch') or {}
print('c3', c3.get('ms_per_step'), c3.get('kernel_ms'), (c3.get('roofline') or {}).get('frac'))
c5=d.get('c5_parabolic_kl') or {}
print('c5', c5.get('f64',{}).get('kernel_ms'), c5.get('f64',{}).get('roofline',{}).get('frac'))
a16=(d.get('other_path_stages') or {}).get('a16_tag_propagation',{})
print('a16', {k:a16.get(k) for k in ('stage_wall_ms','prepare_call_ms','sweep_call_ms','sweeps','flips','stage_over_kernels')})
print('cpu', d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline',{}).get('seconds'))
PY
if [ -z "$NO_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py ${BENCH_ARGS} > $OUT/bench_under_rocprof.json 2> $OUT/bench_under_rocprof.err || { tail -20 $OUT/bench_under_rocprof.err; exit 1; }
  cd $R
  python3 tools/kstats.py $OUT/prof base
  python3 tools/kstats_by_grid.py $OUT/prof $OUT/kernel_stats_by_grid.csv --match=k_sender,k_extrapolate,k_node,k_tag,k_count,k_parabolic
fi
echo r05-done
