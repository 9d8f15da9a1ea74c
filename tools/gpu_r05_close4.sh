#!/bin/bash
# round 5, fourth closing run on the shipped build (tag stage's final copy queued ahead of
# the host's stop decision): the closing sequence (TAG final4)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=final4 bash tools/gpu_r05_final.sh || exit 1
echo close4-done
