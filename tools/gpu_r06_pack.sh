#!/bin/bash
# round 6: the block-packed kept lists of the compact-list tag prepare (GTF_TAG_PACK) -- tag tests,
# then the C3 sweep A/B (marginal per-sweep time of the product call) and the C4 stage
set -o pipefail
O=gpurun_out/r06/pack
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tag" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u tools/tag_sweep_marginal.py c3 3 "pack=" "nopack=GTF_TAG_PACK:0" > $O/c3.jsonl 2>&1 || { tail -20 $O/c3.jsonl; exit 1; }
tail -1 $O/c3.jsonl
