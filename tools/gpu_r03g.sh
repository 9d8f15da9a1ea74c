#!/bin/bash
# round 3: the device event build against the host build, and the drop-in stage timing
# with the runner's imports before the fork. Stops at the first failure.
set -o pipefail
O=gpurun_out/r03g2
mkdir -p $O
true
tail -3 $O/pytest.log
timeout -k 10 200 python -u -c "
import json, sys, os
sys.path[:0] = ['.', 'gnn-track-finding_amd']
import bench
from gtf.params import Params
print(json.dumps(bench.dropin_stage_wall(Params(), reps=5)))
" > $O/dropin.json 2> $O/dropin.err || { tail -20 $O/dropin.err; exit 1; }
cat $O/dropin.json
echo r03g-done
