#!/bin/bash
# round 5: the staged-inverse A/B (NOINV 3 vs 2) and the SQ breakdown of the node kernel in one call
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NO_TESTS= bash tools/gpu_ab_env.sh r05/inv 2 m5=libgtf.so i2=libgtf_i2.so || exit 1
bash tools/gpu_r05_sq.sh r05/sq libgtf.so libgtf_s1.so libgtf_s3.so libgtf_s4.so libgtf_a1.so libgtf_a2.so libgtf_a3.so || exit 1
echo combo-done
