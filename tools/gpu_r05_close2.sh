#!/bin/bash
# round 5, second closing run: the sharded tests and rank-0 phase times (fused phase 1b), then
# the closing sequence of tools/gpu_r05_final.sh on the shipped build (TAG final2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=shard2 bash tools/gpu_r05_shard.sh || exit 1
TAG=final2 bash tools/gpu_r05_final.sh || exit 1
echo close2-done
