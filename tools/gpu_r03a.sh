#!/bin/bash
# round 3: full-size sharded C4 test, bench --gpus 2 (gloo rehearsal, self-spawned ranks), bench N=1
set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shard_c4.py > gpurun_out/r03a/shard_c4.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 2 > gpurun_out/r03a/bench_g2.json 2> gpurun_out/r03a/bench_g2.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-dropin > gpurun_out/r03a/bench_g1.json 2> gpurun_out/r03a/bench_g1.err
