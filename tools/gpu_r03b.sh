#!/bin/bash
# round 3: GPU suite (incl. the 800' real-data parity and the sharded C4 test), then the
# rocprofv3 kernel trace of the default bench, PMC passes of the C4 pass and of the cold
# config-5 rotation, one bench line, . Stops at the first failing GPU step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/gpu_profile.sh $O/c4 --steps 20 --warmup 3 --no-c5 --no-dropin || exit 1
python tools/pmc_summary.py $O/c4 profiles/r01_pmc/calib $O/c4/pmc_c4.json c4 > /dev/null || exit 1
bash tools/gpu_profile_py.sh $O/c5 tools/pkl_time.py 48 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
echo r03b-bench-done
for i in 1 2; do
  GTF_NO_OUTIDX=1 timeout -k 10 120 python tools/pass_loop.py 150 >> $O/ab_outidx.jsonl || exit 1
  timeout -k 10 120 python tools/pass_loop.py 150 >> $O/ab_outidx.jsonl || exit 1
done
