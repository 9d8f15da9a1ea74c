#!/bin/bash
# Profile bench.py on the GPU box: kernel trace/stats, then HBM counters in their
# own passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
# usage: tools/gpu_profile.sh OUTDIR [bench args...]
set -e
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/$OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu "$@" > $R/$OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$OUT/fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu "$@" > $R/$OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$OUT/write -o run --output-format csv -- python3 $R/bench.py --no-cpu "$@" > $R/$OUT/write.log 2>&1
echo profile-done
