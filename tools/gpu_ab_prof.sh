#!/bin/bash
# GPU box: per-kernel rocprofv3 durations of the default bench for several libgtf builds
# (names under gnn-track-finding_amd/gtf/), two alternating rounds, then the C4 digest and
# parity tests on each non-default build.
# usage: tools/gpu_ab_prof.sh OUT lib1.so lib2.so ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for lib in "$@"; do
    (cd /tmp && GTF_LIB=$R/gnn-track-finding_amd/gtf/$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/$lib.$r -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --no-dropin --steps 30 --warmup 3 > $OUT/$lib.$r.json 2> $OUT/$lib.$r.err)
    python3 $R/tools/kstats.py $OUT/$lib.$r $lib
  done
done
for lib in "$@"; do
  if [[ "$lib" != *base* ]]; then
    GTF_LIB=$R/gnn-track-finding_amd/gtf/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $OUT/$lib.tests.log 2>&1
    tail -1 $OUT/$lib.tests.log
  fi
done
echo ab-prof-done
