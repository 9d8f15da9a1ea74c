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
# one variant: the library's Makefile with its own object directory and output name
build() {
  name=$1; shift
  make -s -j8 OUT=../gtf/libgtf_$name.so OBJDIR=../../build/obj_$name EXTRA="$*"
}
if [ -n "$1" ]; then
  build "$@"
  exit 0
fi
for a in 1 2 3 6; do   # (4: loads + stores of every field -- faulted on a drop-in graph, not built)
  build ablate$a -DGTF_ABLATE=$a
done
for v in 1 2 3 4; do
  build seq$v -DGTF_SEQ_VARIANT=$v
done
