#!/bin/bash
# GPU box: per-kernel rocprofv3 durations of the default bench for several library builds,
# alternating rounds, then the C4 digest + parity tests on every non-base build.
# usage: tools/gpu_abv.sh OUT ROUNDS lib1.so lib2.so ...   (names under gnn-track-finding_amd/gtf/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
ROUNDS=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for lib in "$@"; do
  if [[ "$lib" != libgtf.so ]]; then
    GTF_LIB=$R/gnn-track-finding_amd/gtf/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $OUT/$lib.tests.log 2>&1
    rc=$?
    echo "$lib tests: $(tail -1 $OUT/$lib.tests.log)"
    [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  fi
done
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    (cd /tmp && GTF_LIB=$R/gnn-track-finding_amd/gtf/$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/$lib.$r -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --no-dropin --steps 30 --warmup 3 > $OUT/$lib.$r.json 2> $OUT/$lib.$r.err) || exit 1
    python3 $R/tools/kstats.py $OUT/$lib.$r $lib
  done
done
echo abv-done
