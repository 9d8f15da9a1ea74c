#!/bin/bash
# round 5: the driver's own commands on the final build -- smoke(), then the bench line as the
# driver runs it (--gpus 1 --steps 20 --warmup 5), wall-timed
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r05/drv
mkdir -p $OUT
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
t0=$(date +%s.%N)
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
t1=$(date +%s.%N)
echo "bench wall $(python3 -c "print(round($t1-$t0,1))") s"
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('invalid'))"
echo drv-done
