#!/bin/bash
# round 6 baseline on the round-5 build: the fused pass's node kernel per lane-group bucket
# (tools/pass_buckets.py) on C4 and C3, to size the small-node buckets' share of the launch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r06/${TAG:-base}
mkdir -p $OUT
timeout -k 10 300 python -u tools/pass_buckets.py c4 > $OUT/buckets_c4.json 2> $OUT/buckets_c4.err || { tail -20 $OUT/buckets_c4.err; exit 1; }
cat $OUT/buckets_c4.json
timeout -k 10 400 python -u tools/pass_buckets.py c3 > $OUT/buckets_c3.json 2> $OUT/buckets_c3.err || { tail -20 $OUT/buckets_c3.err; exit 1; }
cat $OUT/buckets_c3.json
