#!/bin/bash
# Diagnostics builds of libgtf with parts of the clustering kernel compiled out
# (GTF_ABLATE in csrc/gtf_node_group.h): 1 = no clustering, 2 = staging + pairwise
# distances only, 3 = no greedy KL loop. Time one with GTF_LIB=<path> python bench.py.
set -e
cd "$(dirname "$0")/../gnn-track-finding_amd/csrc"
for a in 1 2 3; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DGTF_ABLATE=$a -shared \
    -o ../gtf/libgtf_ablate$a.so gtf_pass.hip gtf_tags.hip gtf_kl.hip gtf_tse.hip gtf_shard.hip gtf_extract.hip gtf_build.cpp
done
