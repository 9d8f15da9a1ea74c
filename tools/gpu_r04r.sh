#!/bin/bash
# round 4 final pairing: the default bench line and the rocprofv3 --kernel-trace --stats
# summary of the same command; then the opt-in C3 section once
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/final_pair
mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value']/1e9, d['kernel_ms'], d['roofline']['frac'], d['c5_parabolic_kl']['f64']['roofline']['frac'], d.get('c3_fused_batch'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py > $OUT/bench_under_rocprof.json 2> $OUT/bench_under_rocprof.err || { tail -20 $OUT/bench_under_rocprof.err; exit 1; }
python3 $R/tools/kstats.py $OUT/prof final
cd $R
timeout -k 10 600 python -u bench.py --c3 --no-cpu --no-dropin --no-c5 > $OUT/bench_c3_section.json 2> $OUT/bench_c3_section.err || { tail -20 $OUT/bench_c3_section.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_c3_section.json').read().strip().splitlines()[-1]); c=d['c3_fused_batch']; print('c3', c['ms_per_step'], c['edges_per_s']/1e9, c['roofline']['frac'])"
echo r04r-done
