#!/bin/bash
# SQ counter passes (issue vs latency) of bench.py's kernels: two passes of <= 8 SQ counters.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d $OUT/sq1 -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --steps 10 --warmup 2 "$@" > $OUT/sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM --kernel-trace -d $OUT/sq2 -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --steps 10 --warmup 2 "$@" > $OUT/sq2.log 2>&1
echo sq-done
