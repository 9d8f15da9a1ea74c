#!/bin/bash
# the whole GPU suite, then smoke()
set -o pipefail
O=gpurun_out/suite
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/ \
  > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
