#!/bin/bash
# round 6: the <= 2-slot / 3..4-slot receivers' node-kernel time alone, per libgtf variant,
# C3 and C4, then the SQ counters of the <= 2-slot-only C3 launch per variant
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r06/${TAG:-b}
mkdir -p $OUT
for wl in c3 c4; do
  for mode in g2 g34 all; do
    for lib in "$@"; do
      GTF_LIB=$R/gnn-track-finding_amd/gtf/$lib timeout -k 10 200 python3 tools/node_bucket_time.py $wl $mode 12 >> $OUT/times.jsonl 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
      tail -1 $OUT/times.jsonl
    done
  done
done
if [ -n "$SQ" ]; then
for lib in "$@"; do
  GTF_LIB=$R/gnn-track-finding_amd/gtf/$lib PROG="tools/node_bucket_time.py c3 g2 6" bash tools/gpu_sqmix.sh r06/${TAG:-b}/sq_${lib%.so} > /dev/null || exit 1
  echo "== $lib"; grep -i "k_node_multi" -A3 $OUT/sq_${lib%.so}/sqmix.txt | head -12
done
fi
