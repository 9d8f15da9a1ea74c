#!/bin/bash
# GPU box: parity suite, then a short bench of the default build and (A/B) of an
# alternative build given as $1 (a .so under gnn-track-finding_amd/gtf/).
set -e
mkdir -p gpurun_out/chk
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/chk/gpu_tests.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu --no-c5 --no-dropin --steps 30 --warmup 3 > gpurun_out/chk/bench.log 2>&1
if [ -n "$1" ]; then
  GTF_LIB=$PWD/gnn-track-finding_amd/gtf/$1 timeout -k 10 200 python -u bench.py --no-cpu --no-c5 --steps 30 --warmup 3 > gpurun_out/chk/bench_alt.log 2>&1
fi
echo check-done
