#!/bin/bash
# hipGraph capture of the split pass, bisected: the modes of tools/capture_probe.py in order,
# stopping at the first that fails with exit status 3 (a crash ends the call's GPU work)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04/capture${CAPTURE_TAG:-}
mkdir -p $OUT
for m in ${MODES:-one shard halo fork exchange step}; do
  timeout -k 10 120 python3 -X faulthandler -u tools/capture_probe.py $m > $OUT/$m.log 2>&1
  rc=$?
  echo "$m rc=$rc"; tail -3 $OUT/$m.log
  [ $rc -ne 0 ] && { grep -A12 "Fatal Python error" $OUT/$m.log; exit 3; }
done
echo capture-bisect-done
