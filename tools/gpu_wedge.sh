#!/bin/bash
# one-GPU pass with the event in azimuthal wedges (8 = one per XCD, 16, 32) before the tiles
set -o pipefail
O=gpurun_out/wedge
mkdir -p $O
for i in 1 2; do
  for w in 0 8 16 32; do
    GTF_WEDGES=$w timeout -k 10 150 python tools/pass_loop.py 150 >> $O/ab.jsonl || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for w in 0 8; do
  GTF_WEDGES=$w timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/$O/prof$w -o run --output-format csv -- python3 $R/tools/pass_loop.py 100 > $R/$O/prof$w.log 2>&1 || exit 1
done
cat $R/$O/ab.jsonl
