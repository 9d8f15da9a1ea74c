#!/bin/bash
# round 6: the C4 tag stage, current build against gtf/ab/libgtf_old.so (the first compact-list
# sweep), stage wall time and a kernel trace of each
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r06/${TAG:-tagc4}
mkdir -p $OUT
export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export GTF_LIB=$R/gnn-track-finding_amd/gtf/ab/libgtf_old.so; else unset GTF_LIB; fi
  timeout -k 10 200 python3 tools/tag_stage_time.py c4 20 1,0 >> $OUT/stage_$v.jsonl 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  tail -1 $OUT/stage_$v.jsonl
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 tools/tag_stage_time.py c4 20 1 > $OUT/prof_$v.log 2>&1 || { tail -5 $OUT/prof_$v.log; exit 1; }
  f=$(find $OUT/prof_$v -name "*kernel_stats.csv" -print -quit); grep -E "k_tag" "$f" | cut -d, -f1,2,4,6,7 | sed 's/(gtf_graph[^"]*//;s/(long[^"]*//;s/(int[^"]*//'
done
