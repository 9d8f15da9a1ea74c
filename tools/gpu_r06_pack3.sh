#!/bin/bash
# round 6: rocprofv3 kernel stats of the C3 tag stage, packed vs unpacked kept lists
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r06/pack
mkdir -p $O
for m in pack nopack; do
  if [ $m = pack ]; then export GTF_TAG_PACK=1; else export GTF_TAG_PACK=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run -- python3 -u tools/tag_sweep_marginal.py c3 1 "$m=" > $O/prof_$m.log 2>&1 || { tail -20 $O/prof_$m.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; grep -i "tag" $f | cut -d, -f1-8; done
