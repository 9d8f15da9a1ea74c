#!/bin/bash
# Diagnostics builds of libgtf with parts of the fused node kernel compiled out
# (GTF_ABLATE in csrc/gtf_node_group.h): 1 = no clustering, 2 = staging + pairwise
# distances only, 3 = no greedy KL loop, 4 = loads and stores of every field with no
# op, 6 = every op but no slot stores except the activation; GTF_SEQ_VARIANT=1..4 in
# csrc/gtf_pass.hip runs a prefix of the op sequence. Time them with tools/ab.sh.
set -e
cd "$(dirname "$0")/../gnn-track-finding_amd/csrc"
for a in 1 2 3 4 6; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DGTF_ABLATE=$a -shared \
    -o ../gtf/libgtf_ablate$a.so gtf_pass.hip gtf_tags.hip gtf_kl.hip gtf_tse.hip gtf_shard.hip gtf_extract.hip gtf_build.cpp
done
