#!/bin/bash
# GPU box: A/B of alternative libgtf builds on the default bench (no CPU / config-5
# sections), two alternating rounds; each line goes to gpurun_out/ab/<lib>.<round>.json.
# usage: tools/ab.sh libgtf.so libgtf_base.so ...   (names under gnn-track-finding_amd/gtf/)
set -e
mkdir -p gpurun_out/ab
for r in 1 2; do
  for lib in "$@"; do
    GTF_LIB=$PWD/gnn-track-finding_amd/gtf/$lib timeout -k 10 120 python -u bench.py --no-cpu --no-c5 --no-dropin --steps 50 --warmup 5 \
      > gpurun_out/ab/$lib.$r.json 2> gpurun_out/ab/$lib.$r.err
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['kernel_ms'])" gpurun_out/ab/$lib.$r.json $lib
  done
done
echo ab-done
