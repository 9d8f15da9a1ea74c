#!/bin/bash
# Kernel trace + HBM counters (separate FETCH_SIZE / WRITE_SIZE passes) of any python
# script on the GPU box: tools/gpu_profile_py.sh OUTDIR script.py [args...]
set -e
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/$OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/trace -o run --output-format csv -- python3 $R/"$@" > $R/$OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$OUT/fetch -o run --output-format csv -- python3 $R/"$@" > $R/$OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$OUT/write -o run --output-format csv -- python3 $R/"$@" > $R/$OUT/write.log 2>&1
echo profile-done
