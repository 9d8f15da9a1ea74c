#!/bin/bash
# round 4 closing run on the shipped build: the whole GPU suite, smoke(), the default bench
# line, and the same bench command under rocprofv3 --kernel-trace --stats (the kernel
# summary the line's roofline is checked against). Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/closing
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
echo r04close-done
