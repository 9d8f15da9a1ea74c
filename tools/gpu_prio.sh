#!/bin/bash
# node kernel: slot loads issued at raised wave priority (GTF_PRIO=1 build) vs default
set -o pipefail
O=gpurun_out/prio
mkdir -p $O
for i in 1 2 3; do
  unset GTF_LIB; timeout -k 10 120 python tools/pass_loop.py 150 >> $O/ab.jsonl || exit 1
  GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_prio1.so timeout -k 10 120 python tools/pass_loop.py 150 | sed 's/^{/{"lib":"prio1",/' >> $O/ab.jsonl || exit 1
done
cat $O/ab.jsonl
