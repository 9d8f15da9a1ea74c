#!/bin/bash
# GPU box: the sharding tests, then a rehearsal of bench.py's N > 1 path with two ranks on
# the one GPU over gloo (RCCL needs one GPU per rank; the driver runs N = 2..8 itself).
set -e
mkdir -p gpurun_out/shard
timeout -k 10 300 python -u -m pytest tests/test_shard.py -v --timeout 200 --timeout-method thread > gpurun_out/shard/tests.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 10 --warmup 2 --backend gloo > gpurun_out/shard/bench2.log 2>&1
echo shard-done
