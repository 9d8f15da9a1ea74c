#!/bin/bash
# A/B of config-5 gtf_parabolic_kl builds on one box: tools/gpu_kl_ab.sh LIB... (file
# names under gnn-track-finding_amd/gtf; "libgtf.so" is the default build), two rounds.
set -e
for r in 1 2; do
  for lib in "$@"; do
    GTF_LIB=$PWD/gnn-track-finding_amd/gtf/$lib timeout -k 10 200 python -u tools/pkl_time.py 50 2>/dev/null | sed "s/^/$lib r$r /" | cut -c1-200
  done
done
