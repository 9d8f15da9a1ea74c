#!/bin/bash
# round 6: the sweep's existing knobs on the block-packed kept lists (C3)
set -o pipefail
O=gpurun_out/r06/pack
mkdir -p $O
timeout -k 10 600 python -u tools/tag_sweep_marginal.py c3 3 "pack=" "n4r4=GTF_TAG_NPT:4+GTF_TAG_R:4" "n2r4=GTF_TAG_R:4" "n1=GTF_TAG_NPT:1" "nopack=GTF_TAG_PACK:0" > $O/c3_knobs.jsonl 2>&1 || { tail -20 $O/c3_knobs.jsonl; exit 1; }
tail -1 $O/c3_knobs.jsonl
