#!/bin/bash
# drop-in CLI cold-start breakdown (tools/cold_start.py)
set -o pipefail
O=gpurun_out/cold
mkdir -p $O
timeout -k 10 500 python -u tools/cold_start.py $O/cold.json > $O/cold.log 2>&1
