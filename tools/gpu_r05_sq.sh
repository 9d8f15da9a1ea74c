#!/bin/bash
# round 5: where the fused node kernel's VALU instructions go -- one SQ pass per
# diagnostics build (op-sequence prefixes GTF_SEQ_VARIANT 1 / 3 / 4, clustering ablations
# GTF_ABLATE 1 / 2 / 3) beside the default, then the three-pass instruction mix of the
# default build (the bench line's valu_roofline source).
# usage: tools/gpu_r05_sq.sh OUT lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=$1; shift
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
export TMPDIR=/tmp
for lib in "$@"; do
  (cd /tmp && GTF_LIB=$R/gnn-track-finding_amd/gtf/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-trace -d $OUT/$lib/sq1 -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-c5 --no-c3 --no-dropin --steps 10 --warmup 2 > $OUT/$lib.log 2>&1) || { echo "($lib: exit $?)"; exit 1; }
  echo "== $lib"
  python3 $R/tools/sq_summary.py $OUT/$lib | grep -A9 k_node_multi | grep -E "k_node|VALU|WAVE_CYCLES|WAIT_ANY"
done
if [ -z "$NO_MIX" ]; then
  bash $R/tools/gpu_sqmix.sh $NAME/sqmix > /dev/null 2>&1 || { echo "sqmix failed"; exit 1; }
  head -80 $OUT/sqmix/sqmix.txt
fi
echo r05-sq-done
