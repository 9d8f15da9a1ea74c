#!/bin/bash
# round 5, fifth closing run on the shipped build (the first sweep counting the processed nodes; the fused phase 1b with
# the scan operands handed over): the closing sequence (TAG final5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=final5 bash tools/gpu_r05_final.sh || exit 1
echo close5-done
