#!/bin/bash
# round 4: where the node kernel's time goes now -- per-op wave timing (diagnostics builds
# GTF_OP_TIMING=1) of the default and the 5-wave node kernel, and the SQ instruction mix /
# wait split of both; then the split-step hipGraph capture with Python's fault handler
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/c
mkdir -p $OUT
GTF_LIB=$R/gnn-track-finding_amd/gtf/libgtf_optime.so timeout -k 10 200 python -u tools/op_timing.py $OUT/op_timing.json > $OUT/op_timing.log 2>&1 || { tail -20 $OUT/op_timing.log; exit 1; }
GTF_OPT_FLUSH=1 GTF_LIB=$R/gnn-track-finding_amd/gtf/libgtf_optime_w5.so timeout -k 10 200 python -u tools/op_timing.py $OUT/op_timing_w5.json > $OUT/op_timing_w5.log 2>&1 || { tail -20 $OUT/op_timing_w5.log; exit 1; }
echo optime-done
GTF_LIB=$R/gnn-track-finding_amd/gtf/libgtf.so bash tools/gpu_sqmix.sh r04/c/sq_base || exit 1
GTF_LIB=$R/gnn-track-finding_amd/gtf/libgtf_w5.so bash tools/gpu_sqmix.sh r04/c/sq_w5 || exit 1
(GTF_SPLIT_GRAPH=1 timeout -k 10 180 python3 -X faulthandler -u tools/split_time.py 5 1 > $OUT/split_graph.log 2>&1; echo "split_graph rc=$?" >> $OUT/split_graph.log)
tail -30 $OUT/split_graph.log
echo r04c-done
