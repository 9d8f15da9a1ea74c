#!/bin/bash
# round 4 closing run on the shipped build: the whole GPU suite, smoke(), the default bench
# line, and the same bench command under rocprofv3 --kernel-trace --stats (the kernel
# summary the line's roofline is checked against). Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/${CLOSE_TAG:-closing}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -2 $OUT/pytest_gpu.log; grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value']/1e9, d['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic'], d['c5_parabolic_kl']['f64']['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py > $OUT/bench_under_rocprof.json 2> $OUT/bench_under_rocprof.err || { tail -20 $OUT/bench_under_rocprof.err; exit 1; }
python3 $R/tools/kstats.py $OUT/prof closing
cd $R
if [ -n "$WITH_C3" ]; then   # configs[2]: 64 fused events, the size SURVEY 8(d) quotes roofline fractions on
  timeout -k 10 600 python -u bench.py --workload c3 --no-cpu --no-c5 --no-dropin --steps 20 --warmup 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -20 $OUT/bench_c3.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_c3.json').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['value']/1e9, d['kernel_ms'], d['roofline']['frac'], d.get('pass_roofline', {}).get('frac'))"
  bash tools/gpu_profile.sh gpurun_out/r04/${CLOSE_TAG:-closing}/c3 --workload c3 --no-c5 --no-dropin --steps 10 --warmup 2 || exit 1
  python tools/pmc_summary.py gpurun_out/r04/${CLOSE_TAG:-closing}/c3 profiles/r01_pmc/calib gpurun_out/r04/${CLOSE_TAG:-closing}/c3/pmc_c3.json c3 > /dev/null || exit 1
fi
echo r04close-done
