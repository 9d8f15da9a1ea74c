#!/bin/bash
# round 4 final build: the whole GPU suite, smoke(), the default bench line; then the
# hipGraph capture probes (torch-only repro, linear exchange) last -- a crash ends the call
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "suite rc=$?"; tail -2 $OUT/pytest_gpu.log; grep -E "^FAILED|^ERROR" $OUT/pytest_gpu.log | head
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value']/1e9, d['kernel_ms'], d['roofline']['frac'], d['c5_parabolic_kl']['f64']['roofline']['frac'], d['other_path_stages']['a16_tag_propagation'])"
MODES="torchx linear" bash tools/gpu_capture_bisect.sh
echo r04f-done
