#!/bin/bash
# round 4: the sender scan's 16-lane bucket from gtf_graph.out_lanes (GTF_SEND_LANES16):
# parity of the new default, then per-kernel A/B against the build without it
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04/o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_shard.py tests/test_gpu_shard_tags.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_abv.sh r04/o/abv 3 libgtf.so libgtf_nol16.so || exit 1
echo r04o-done
