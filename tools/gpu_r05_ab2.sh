#!/bin/bash
# round 5: k_extrapolate's predicated gathers + the sender's unchanged-carry store skipped
# (default build) against the previous form (np), the reciprocal-product quotients (xf) and
# the recomputed block inverses (i2); then the sharded tests and rank-0 phase times with the
# fused phase 1b
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_ab_env.sh r05/ab2 2 m5=libgtf.so np=libgtf_np.so xf=libgtf_xf.so i2=libgtf_i2.so || exit 1
TAG=shard2 bash tools/gpu_r05_shard.sh || exit 1
echo ab2-done
