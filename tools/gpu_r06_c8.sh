#!/bin/bash
# round 6: count bytes + wave prefix offsets in the C3 tag sweep (GTF_TAG_C8) -- tag tests, then A/B
set -o pipefail
O=gpurun_out/r06/c8
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tag" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python -u tools/tag_sweep_marginal.py c3 3 "c8=" "word=GTF_TAG_C8:0" "nopack=GTF_TAG_PACK:0" > $O/c3.jsonl 2>&1 || { tail -20 $O/c3.jsonl; exit 1; }
tail -1 $O/c3.jsonl
