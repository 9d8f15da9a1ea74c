#!/bin/bash
# rehearsal of the driver's N > 1 launch forms on the one-GPU box (gloo; ranks share the
# GPU, so the times are not scaling figures): torchrun with 2 ranks, then the
# self-spawning form with 8 ranks.
set -o pipefail
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_shard_tags.py -x -v --timeout 150 --timeout-method thread > $O/pytest_tags.log 2>&1 || { tail -30 $O/pytest_tags.log; exit 1; }
tail -1 $O/pytest_tags.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --backend gloo --no-cpu --no-dropin --no-c5 --steps 10 --warmup 2 > $O/bench_torchrun2_gloo.json 2> $O/bench_torchrun2_gloo.err || { tail -30 $O/bench_torchrun2_gloo.err; exit 1; }
echo torchrun2-done
timeout -k 10 600 python -u bench.py --gpus 8 --backend gloo --no-cpu --no-dropin --steps 10 --warmup 2 > $O/bench_gpus8_gloo.json 2> $O/bench_gpus8_gloo.err || { tail -30 $O/bench_gpus8_gloo.err; exit 1; }
echo r03l-done
