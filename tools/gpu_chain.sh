#!/bin/bash
# the run script's chain of drop-in CLIs (tests/test_pipeline.py) + event conversion, then its timing
set -o pipefail
O=gpurun_out/chain
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_pipeline.py tests/test_event_conversion.py tests/test_dropin.py tests/test_gpu_tse.py tests/test_gpu_devmem.py \
  > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/run_script_time.py $O/run_script_time.json > $O/run_script_time.log 2>&1
