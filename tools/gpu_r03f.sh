#!/bin/bash
# round 3: default bench line (drop-in runner with the GC off in its workers), the sharded
# per-rank pass at N = 1..8 with and without widened lane groups, and the kernel trace of
# rank 0's pass at N = 8. Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench-done
timeout -k 10 200 python -u tools/shard_pass_time.py > $O/shard_pass_time.txt 2>&1 || exit 1
GTF_SHARD_WIDEN=1 timeout -k 10 200 python -u tools/shard_pass_time.py > $O/shard_pass_time_widen1.txt 2>&1 || exit 1
cat $O/shard_pass_time*.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/shard8 -o run --output-format csv -- python3 $R/tools/shard_pass_time.py 8 > $R/$O/shard8.log 2>&1 || exit 1
echo r03f-done
