#!/bin/bash
# Config-5 parabolic KL alone under rocprofv3: kernel stats, then FETCH_SIZE and
# WRITE_SIZE passes and one SQ pass (each its own run).
# usage: tools/gpu_pkl_prof.sh OUTDIR
set -e
OUT=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/$OUT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/trace -o run --output-format csv -- python3 $R/tools/pkl_time.py 20 > $R/$OUT/trace.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$OUT/fetch -o run --output-format csv -- python3 $R/tools/pkl_time.py 20 > $R/$OUT/fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$OUT/write -o run --output-format csv -- python3 $R/tools/pkl_time.py 20 > $R/$OUT/write.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-trace -d $R/$OUT/sq -o run --output-format csv -- python3 $R/tools/pkl_time.py 20 > $R/$OUT/sq.log 2>&1
echo pkl-profile-done
