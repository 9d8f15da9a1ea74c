#!/bin/bash
# round 5: rehearsal of the N > 1 bench line (two gloo ranks sharing the box's GPU; the driver
# runs RCCL ranks on separate GPUs), then the full GPU suite on the shipped build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r05/n2
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu --no-dropin > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || { tail -30 $OUT/bench_n2_gloo.err; exit 1; }
python3 - <<PY
import json
d=json.loads(open('$OUT/bench_n2_gloo.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','ms_per_step','n_gpus','scaling')}, d['config'].get('parallelism'))
s=d.get('sharded_single_event') or {}
print('sharded', {k: s.get(k) for k in ('ms_per_step','step_form','ms_per_step_overlapped','ms_per_step_sequential','pass_ms_no_exchange','device_error_flags')})
print('replicas', d.get('event_replicas',{}).get('value'), 'c5_sharded', (d.get('c5_event_sharded') or {}).get('value'))
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu.log; grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head; [ $rc -ne 0 ] && exit $rc
echo n2-done
