#!/bin/bash
# round 6: tag propagation over compact kept lists with int32 tags vs the keep-mask sweeps:
# the tag GPU tests, the stage wall time on C4 / C3, and a kernel trace of the C3 stage
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r06/${TAG:-tagcsr}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k tag tests/test_gpu_layouts.py tests/test_gpu_shard_tags.py tests/test_gpu_devmem.py \
  tests/test_gpu_comm_native.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for wl in c4 c3; do
  timeout -k 10 300 python3 tools/tag_stage_time.py $wl 20 >> $OUT/stage.jsonl 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
  tail -1 $OUT/stage.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/tag_stage_time.py c3 5 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" -print -quit); cp "$f" $OUT/c3_kernel_stats.csv; head -12 $OUT/c3_kernel_stats.csv
