#!/bin/bash
# round 5: block -> work maps of the extrapolation and the sender scan (gtf::block_map:
# 0 one range per XCD = the default, 1 dispatch order, C runs of C blocks per XCD)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NO_TESTS=1 bash tools/gpu_ab_env.sh r05/maps 2 base=libgtf.so e1=libgtf_e1.so e4=libgtf_e4.so e16=libgtf_e16.so s1=libgtf_s1.so s4=libgtf_s4.so || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05/maps/base.tests.log 2>&1
echo "base tests rc=$?: $(tail -1 gpurun_out/r05/maps/base.tests.log)"
echo maps-done
