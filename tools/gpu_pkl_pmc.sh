#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes of the config-5 parabolic KL alone (tools/pkl_time.py).
# usage: tools/gpu_pkl_pmc.sh OUTDIR
set -e
OUT=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/$OUT
cd /tmp
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$OUT/fetch -o run --output-format csv -- python3 $R/tools/pkl_time.py 20 > $R/$OUT/fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$OUT/write -o run --output-format csv -- python3 $R/tools/pkl_time.py 20 > $R/$OUT/write.log 2>&1
echo pkl-pmc-done
