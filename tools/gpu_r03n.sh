#!/bin/bash
# the tag-propagation tests (one-call C-ABI stage, sharded sweeps)
set -o pipefail
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard_tags.py tests/test_gpu_layouts.py -x -v --timeout 150 --timeout-method thread > $O/pytest_tags.log 2>&1 || { tail -40 $O/pytest_tags.log; exit 1; }
tail -1 $O/pytest_tags.log
