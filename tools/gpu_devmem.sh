#!/bin/bash
# lean (torch-free) drop-in path: parity tests, then the cold-start breakdown
set -o pipefail
O=gpurun_out/devmem
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_devmem.py tests/test_dropin.py tests/test_extract.py tests/test_pipeline.py > $O/pytest.log 2>&1 &&
timeout -k 10 500 python -u tools/cold_start.py $O/cold.json > $O/cold.log 2>&1
