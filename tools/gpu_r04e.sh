#!/bin/bash
# round 4: the sharded tag tests after the prepare fix, the native-comm tests, then the capture
# probe modes "exchange" / "step" and the split pass replayed as hipGraphs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_tags.py tests/test_gpu_comm_native.py -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests rc=$?"; tail -3 $OUT/pytest.log
timeout -k 10 120 python3 -X faulthandler -u tools/capture_probe.py exchange > $OUT/capture_exchange.log 2>&1
rc=$?; echo "exchange rc=$rc"; tail -2 $OUT/capture_exchange.log
[ $rc -ne 0 ] && exit 0
(GTF_SPLIT_GRAPH=1 timeout -k 10 180 python3 -X faulthandler -u tools/split_time.py 20 3 > $OUT/split_graph.log 2>&1; echo "split_graph rc=$?" >> $OUT/split_graph.log)
tail -4 $OUT/split_graph.log
echo r04e-done
