#!/bin/bash
# drop-in stage timing (bench.dropin_stage_wall), twice
set -o pipefail
O=gpurun_out/dropin_ab3
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python -u -c "
import json, sys, os
sys.path[:0] = ['.', 'gnn-track-finding_amd']
import bench
from gtf.params import Params
print(json.dumps(bench.dropin_stage_wall(Params(), reps=5)))
" >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
cat $O/ab.jsonl
