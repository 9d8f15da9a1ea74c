#!/bin/bash
# GPU box: the whole -m gpu suite, then the default bench line (CPU baselines, drop-in
# stage wall time and config 5 included) into gpurun_out/full/.
set -e
mkdir -p gpurun_out/full
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/full/gpu_tests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/full/bench.log 2>&1
echo full-done
