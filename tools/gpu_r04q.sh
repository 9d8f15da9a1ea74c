#!/bin/bash
# round 4: the default bench line with its C3 section, timed end to end
set -o pipefail
O=gpurun_out/r04/q
mkdir -p $O
s=$(date +%s)
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['value']/1e9, d['roofline']['frac'])
print(json.dumps(d['c3_fused_batch'])[:900])"
echo r04q-done
