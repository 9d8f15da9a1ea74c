#!/bin/bash
# round 4: the N > 1 bench path rehearsed with 8 ranks on the one GPU over gloo (final build)
set -o pipefail
O=gpurun_out/r04/t
mkdir -p $O
timeout -k 10 900 python -u bench.py --gpus 8 --backend gloo --steps 10 --warmup 2 --no-c5 > $O/bench_gpus8_gloo.json 2> $O/bench_gpus8_gloo.err || { tail -20 $O/bench_gpus8_gloo.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_gpus8_gloo.json').read().strip().splitlines()[-1])
print(d['n_gpus'], d['value']/1e9, d['ms_per_step'], d.get('rccl_world_size'), d['config'].get('parallelism'), d.get('invalid'))
print(json.dumps(d.get('event_replicas'))[:300])"
echo r04t-done
