#!/bin/bash
# GPU box: kernel trace + FETCH/WRITE passes of bench.py (tools/gpu_profile.sh) into
# gpurun_out/$1, the PMC summary against the committed calibration, then the default
# bench line (CPU baseline and config 5 included).
set -e
OUT=gpurun_out/$1
bash tools/gpu_profile.sh $OUT --steps 20 --warmup 3 --no-c5
python tools/pmc_summary.py $OUT profiles/r01_pmc/calib $OUT/pmc_c4.json c4 > /dev/null
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1
echo round-profile-done
