#!/bin/bash
# round 5: the fused phase 1b (sharded tests + rank-0 phase times), then the extrapolation's
# reciprocal-product quotients (GTF_EXTRAP_FAST build) A/B with the decision-sensitive tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=shard2 bash tools/gpu_r05_shard.sh || exit 1
bash tools/gpu_ab_env.sh r05/xf 2 m5=libgtf.so xf=libgtf_xf.so || exit 1
GTF_LIB=$R/gnn-track-finding_amd/gtf/libgtf_xf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_synthetic.py tests/test_gpu_real800.py tests/test_gpu_batches.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05/xf/xf_more_tests.log 2>&1
echo "xf more tests rc=$?: $(tail -1 gpurun_out/r05/xf/xf_more_tests.log)"
echo next-done
