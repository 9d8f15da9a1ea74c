#!/bin/bash
# round 6: gtf_tag_propagate with the next batch enqueued ahead of the host's read (GTF_TAG_AHEAD)
# and the wave-cooperative prepare (GTF_TAG_PREP_COOP) -- tag tests (every form and read-back
# mode), then the C3 / C4 stage A/B from descending tags; rocprof of the C3 prepare kernels
set -o pipefail
O=gpurun_out/r06/ahead
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_shard_tags.py -k "tag" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/tag_sweep_marginal.py c3 3 "both=" "noahead=GTF_TAG_AHEAD:0" "threadprep=GTF_TAG_PREP_COOP:0" "neither=GTF_TAG_AHEAD:0+GTF_TAG_PREP_COOP:0" > $O/c3.jsonl 2>&1 || { tail -20 $O/c3.jsonl; exit 1; }
tail -1 $O/c3.jsonl
timeout -k 10 400 python -u tools/tag_sweep_marginal.py c4 3 "ahead=" "noahead=GTF_TAG_AHEAD:0" > $O/c4.jsonl 2>&1 || { tail -20 $O/c4.jsonl; exit 1; }
tail -1 $O/c4.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for m in coop thread; do
  if [ $m = coop ]; then export GTF_TAG_PREP_COOP=1; else export GTF_TAG_PREP_COOP=0; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run -- python3 -u tools/tag_sweep_marginal.py c3 1 "$m=" > $O/prof_$m.log 2>&1 || { tail -20 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name "*kernel_stats.csv" | head -1); echo "== $m"; grep -i "tag_prep\|tag_sweep_coop" $f | cut -d, -f1-8
done
