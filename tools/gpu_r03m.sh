#!/bin/bash
# round 3 closing evidence on the shipped libgtf.so: GPU suite, smoke(), default bench
# line, rocprofv3 kernel stats of the C4 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench-done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --no-dropin --steps 20 --warmup 3 > $O/prof_bench.json 2> $O/prof_bench.err) || { tail -20 $O/prof_bench.err; exit 1; }
python3 $R/tools/kstats.py $O/prof libgtf.so
echo r03m-done
