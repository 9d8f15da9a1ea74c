#!/bin/bash
# round 5: the tag stage with its final copy enqueued ahead of the host's stop decision: the
# tag tests, then the bench line's a16 section
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r05/tag
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard_tags.py tests/test_gpu_devmem.py tests/test_gpu_layouts.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_tag.log 2>&1
rc=$?; tail -1 $OUT/pytest_tag.log; grep -E "^FAILED|^ERROR" $OUT/pytest_tag.log | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --no-cpu --no-dropin --no-c3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 - <<PY
import json
d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
a=(d.get('other_path_stages') or {}).get('a16_tag_propagation',{})
print('a16', {k:a.get(k) for k in ('stage_wall_ms','prepare_call_ms','sweep_call_ms','sweeps','flips','stage_over_kernels')})
print('c4', d['ms_per_step'], d['kernel_ms'])
PY
echo tag-done
