#!/bin/bash
# GPU box: per-kernel rocprofv3 durations of the default bench under alternative bench.py
# arguments (each argument set quoted), two alternating rounds.
# usage: tools/gpu_ab_args.sh OUT "args1" "args2" ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  i=0
  for a in "$@"; do
    i=$((i+1))
    (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/v$i.$r -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --no-dropin --steps 30 --warmup 3 $a > $OUT/v$i.$r.json 2> $OUT/v$i.$r.err)
    python3 $R/tools/kstats.py $OUT/v$i.$r "[$a]"
  done
done
echo ab-args-done
