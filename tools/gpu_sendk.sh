#!/bin/bash
# sender scan: arguments through the laundered kernarg pointer with <= 72 SGPRs (8 blocks per
# CU, default build) vs by-value structs (~106 SGPRs: 6 blocks per CU), alternating, then
# kernel stats of both
set -o pipefail
O=gpurun_out/sendk
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c4_digest.py tests/test_shard.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  unset GTF_LIB; timeout -k 10 120 python tools/pass_loop.py 150 >> $O/ab.jsonl || exit 1
  GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_sk0.so timeout -k 10 120 python tools/pass_loop.py 150 | sed 's/^{/{"lib":"sk0",/' >> $O/ab.jsonl || exit 1
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/$O/new -o run --output-format csv -- python3 $R/tools/pass_loop.py 100 > $R/$O/new.log 2>&1 || exit 1
GTF_LIB=$R/gnn-track-finding_amd/gtf/ab/libgtf_sk0.so timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/$O/old -o run --output-format csv -- python3 $R/tools/pass_loop.py 100 > $R/$O/old.log 2>&1 || exit 1
cat $R/$O/ab.jsonl
