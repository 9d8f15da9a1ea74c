#!/bin/bash
# GPU box: A/B of builds under rocprofv3 (tools/gpu_ab_prof.sh), the staged-input test,
# SQ counters of the default build and one default bench line.
set -e
OUT=$1; shift
bash tools/gpu_ab_prof.sh $OUT "$@"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$OUT/fullsize.log 2>&1
tail -1 gpurun_out/$OUT/fullsize.log
bash tools/gpu_sq.sh $OUT/sq --no-dropin
timeout -k 10 300 python -u bench.py --no-cpu --no-dropin > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err
echo round2-done
