#!/bin/bash
# VALU instruction mix and issue / wait split of the pass kernels (C4, tools/pass_loop.py):
# three passes of <= 8 SQ counters each. usage: [PROG="tools/pkl_time.py 24"] tools/gpu_sqmix.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT --kernel-trace -d $OUT/sq1 -o run --output-format csv -- python3 $R/${PROG:-tools/pass_loop.py 20} > $OUT/sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace -d $OUT/sq2 -o run --output-format csv -- python3 $R/${PROG:-tools/pass_loop.py 20} > $OUT/sq2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS --kernel-trace -d $OUT/sq3 -o run --output-format csv -- python3 $R/${PROG:-tools/pass_loop.py 20} > $OUT/sq3.log 2>&1
python3 $R/tools/sq_summary.py $OUT $OUT/sqmix.json > $OUT/sqmix.txt
echo sqmix-done
