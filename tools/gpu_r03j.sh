#!/bin/bash
# round 3 final evidence: GPU suite, smoke(), default bench line, rocprofv3 kernel stats and
# calibrated HBM counters of the C4 pass and of the cold config-5 rotation, SQ instruction
# mix. Stops at the first failure.
set -o pipefail
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench-done
bash tools/gpu_profile.sh $O/c4 --steps 20 --warmup 3 --no-c5 --no-dropin || exit 1
python tools/pmc_summary.py $O/c4 profiles/r01_pmc/calib $O/c4/pmc_c4.json c4 > /dev/null || exit 1
bash tools/gpu_profile_py.sh $O/c5 tools/pkl_time.py 48 || exit 1
python tools/pmc_summary.py $O/c5 profiles/r01_pmc/calib $O/c5/pmc_c5.json c5 ordered 0 > /dev/null || exit 1
bash tools/gpu_sqmix.sh r03j/sqmix || exit 1
echo r03j-done
