#!/bin/bash
# round 5, third closing run on the shipped build (node kernel blocks in runs of 4 per XCD):
# the sharded tests and rank-0 phase times, then the closing sequence (TAG final3)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=shard3 bash tools/gpu_r05_shard.sh || exit 1
TAG=final3 bash tools/gpu_r05_final.sh || exit 1
echo close3-done
