#!/bin/bash
# round 6: tag propagation's sweep kernel, scheduled vs thread-per-node, on C4 and C3
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r06/${TAG:-tag}
mkdir -p $OUT
for wl in c4 c3; do
  timeout -k 10 300 python3 tools/tag_sweep_time.py $wl 50 >> $OUT/tag_sweep.jsonl 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  tail -1 $OUT/tag_sweep.jsonl
done
