#!/bin/bash
# round 6: the C3 tag prepare's forms, kernel times (rocprofv3 --stats) and stage A/B
set -o pipefail
O=gpurun_out/r06/prep
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tag_propagate_stop_rule or saturated or beyond_int32" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python -u tools/tag_sweep_marginal.py c3 3 "wavepack=GTF_TAG_AHEAD:0+GTF_TAG_PREP_COOP:0" "blockpack=GTF_TAG_AHEAD:0+GTF_TAG_PREP_COOP:0+GTF_TAG_PACK:2" "coopprep=GTF_TAG_AHEAD:0" > $O/c3.jsonl 2>&1 || { tail -20 $O/c3.jsonl; exit 1; }
tail -1 $O/c3.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export GTF_TAG_AHEAD=0
for m in wave block coop; do
  export GTF_TAG_PREP_COOP=0 GTF_TAG_PACK=1
  [ $m = block ] && export GTF_TAG_PACK=2
  [ $m = coop ] && export GTF_TAG_PREP_COOP=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python3 -u tools/tag_sweep_marginal.py c3 1 "$m=" > $O/prof_$m.log 2>&1 || { tail -20 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name "*kernel_stats.csv" | head -1); echo "== $m"; grep -i "tag_prep\|tag_sweep_coop" $f | cut -d, -f1-8
done
