#!/bin/bash
# Diagnostics builds of libgtf with parts of the fused node kernel compiled out
# (GTF_ABLATE in csrc/gtf_node_group.h): 1 = no clustering, 2 = staging + pairwise
# distances only, 3 = no greedy KL loop, 4 = loads and stores of every field with no
# op, 6 = every op but no slot stores except the activation; GTF_SEQ_VARIANT=1..4 in
# csrc/gtf_pass.hip runs a prefix of the op sequence. Extra -D flags for experiment
# builds: tools/ablate_build.sh NAME -DFLAG=1 ... builds libgtf_NAME.so. Time them with
# tools/ab.sh.
set -e
cd "$(dirname "$0")/../gnn-track-finding_amd/csrc"
SRC="gtf_pass.hip gtf_tags.hip gtf_kl.hip gtf_tse.hip gtf_shard.hip gtf_extract.hip gtf_a15.hip gtf_build.cpp gtf_build_dev.hip gtf_mem.hip"
CXX="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -shared"
if [ -n "$1" ]; then
  name=$1; shift
  $CXX "$@" -o ../gtf/libgtf_$name.so $SRC
  exit 0
fi
for a in 1 2 3 6; do   # (4: loads + stores of every field -- faulted on a drop-in graph, not built)
  $CXX -DGTF_ABLATE=$a -o ../gtf/libgtf_ablate$a.so $SRC &
done
for v in 1 2 3 4; do
  $CXX -DGTF_SEQ_VARIANT=$v -o ../gtf/libgtf_seq$v.so $SRC &
done
wait
