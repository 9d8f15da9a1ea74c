#!/bin/bash
# round 6: the wave-cooperative tag sweep on block-packed lists (GTF_TAG_COOP) -- tag tests, then C3 A/B
set -o pipefail
O=gpurun_out/r06/coop
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "tag" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u tools/tag_sweep_marginal.py c3 3 "coop2=" "coop1=GTF_TAG_COOP:1" "coop4=GTF_TAG_COOP:4" "lanes=GTF_TAG_COOP:0" > $O/c3.jsonl 2>&1 || { tail -20 $O/c3.jsonl; exit 1; }
tail -1 $O/c3.jsonl
