#!/bin/bash
# GPU box: per-kernel rocprofv3 durations of the C4 bench (no CPU / C3 / C5 / drop-in
# sections) for several (libgtf build, environment) variants, alternating rounds, then the
# C4 digest and parity tests on every variant. A variant is NAME=lib.so[,VAR=val...]
# (lib under gnn-track-finding_amd/gtf/).
# usage: tools/gpu_ab_env.sh OUT ROUNDS NAME=lib[,VAR=val]... 
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
ROUNDS=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
run_env() {   # variant spec -> "env A=B C=D"
  local spec=$1 name=${1%%=*} rest=${1#*=}
  local lib=${rest%%,*} vars=""
  [[ "$rest" == *,* ]] && vars=$(echo ${rest#*,} | tr ',' ' ')
  echo "GTF_LIB=$R/gnn-track-finding_amd/gtf/$lib $vars"
}
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name=${spec%%=*}
    (cd /tmp && env $(run_env $spec) timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/$name.$r -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --no-dropin --no-c3 --steps 30 --warmup 3 > $OUT/$name.$r.json 2> $OUT/$name.$r.err) || { echo "FAIL $name"; tail -5 $OUT/$name.$r.err; exit 1; }
    python3 $R/tools/kstats.py $OUT/$name.$r $name
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('   ', sys.argv[2], 'ms/step', round(d['ms_per_step'],5), {k[:12]: round(v*1e3,1) for k,v in d['kernel_ms'].items()})" $OUT/$name.$r.json $name
  done
done
if [ -z "$NO_TESTS" ]; then
  for spec in "$@"; do
    name=${spec%%=*}
    env $(run_env $spec) timeout -k 10 400 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $OUT/$name.tests.log 2>&1
    echo "$name tests: $(tail -1 $OUT/$name.tests.log)"
  done
fi
echo ab-env-done
