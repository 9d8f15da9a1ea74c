#!/bin/bash
# round 6 A/B on one box: C4 (rocprofv3 kernel durations, alternating rounds) and C3
# (bench --workload c3, HIP events) for libgtf variants NAME=lib.so[,VAR=val...], then the
# parity tests on every variant but the first (the first is the shipped baseline).
# usage: tools/gpu_r06_ab.sh OUT ROUNDS NAME=lib[,VAR=val]...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUTN=$1; OUT=$R/gpurun_out/$1; shift
ROUNDS=$1; shift
mkdir -p $OUT
NO_TESTS=1 bash tools/gpu_ab_env.sh $OUTN $ROUNDS "$@" || exit 1
run_env() {
  local spec=$1 rest=${1#*=}
  local lib=${rest%%,*} vars=""
  [[ "$rest" == *,* ]] && vars=$(echo ${rest#*,} | tr ',' ' ')
  echo "GTF_LIB=$R/gnn-track-finding_amd/gtf/$lib $vars"
}
if [ -z "$NO_C3" ]; then
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name=${spec%%=*}
    env $(run_env $spec) timeout -k 10 300 python3 bench.py --workload c3 --no-cpu --no-c5 --no-dropin --no-c3 --steps 20 --warmup 3 > $OUT/$name.c3.$r.json 2> $OUT/$name.c3.$r.err || { echo "FAIL c3 $name"; tail -5 $OUT/$name.c3.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('   c3', sys.argv[2], 'ms/step', round(d['ms_per_step'],5), {k[:12]: round(v*1e3,1) for k,v in d['kernel_ms'].items()}, 'frac', round(d['roofline']['frac'],4))" $OUT/$name.c3.$r.json $name
  done
done
fi
first=1
[ -n "$NO_TESTS" ] && set --
for spec in "$@"; do
  name=${spec%%=*}
  if [ $first = 1 ]; then first=0; continue; fi
  env $(run_env $spec) timeout -k 10 600 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_real800.py tests/test_gpu_batches.py tests/test_gpu_synthetic.py -x -q --timeout 300 --timeout-method thread > $OUT/$name.tests.log 2>&1
  echo "$name tests: $(tail -1 $OUT/$name.tests.log)"
  grep -E "^FAILED|^ERROR" $OUT/$name.tests.log | head -5
done
echo r06-ab-done
