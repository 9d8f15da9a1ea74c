#!/bin/bash
# GPU box: one SQ counter pass (+ kernel trace) of the default bench for several libgtf
# builds (diagnostics builds of tools/ablate_build.sh): where the node kernel's VALU
# instructions and wave cycles go. usage: tools/gpu_ablate_sq.sh OUT lib1.so lib2.so ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for lib in "$@"; do
  (cd /tmp && GTF_LIB=$R/gnn-track-finding_amd/gtf/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-trace -d $OUT/$lib/sq1 -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --no-dropin --steps 10 --warmup 2 > $OUT/$lib.log 2>&1) || echo "($lib: exit $?)"
  echo "== $lib"
  python3 $R/tools/sq_summary.py $OUT/$lib | grep -A9 k_node_multi | grep -E "k_node|VALU|WAVE_CYCLES|WAIT_ANY"
done
echo ablate-sq-done
