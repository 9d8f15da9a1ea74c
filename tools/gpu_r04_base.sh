#!/bin/bash
# round 4 baseline on this round's box: per-kernel rocprofv3 durations of the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/base
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --no-dropin --steps 30 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err) || exit 1
python3 $R/tools/kstats.py $OUT/prof base
timeout -k 10 200 python3 -u bench.py --no-cpu --steps 20 --warmup 3 > $OUT/bench_full.json 2> $OUT/bench_full.err
echo base-done
