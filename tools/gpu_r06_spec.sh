#!/bin/bash
# round 6: one sweep enqueued behind each batch's report (GTF_TAG_SPEC) -- tag tests (every form and
# read-back mode, C3 size included), then the C3 / C4 stage A/B from descending tags
set -o pipefail
O=gpurun_out/r06/spec
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_shard_tags.py tests/test_gpu_fullsize.py -k "tag" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/tag_sweep_marginal.py c3 3 "spec=" "nospec=GTF_TAG_SPEC:0" > $O/c3.jsonl 2>&1 || { tail -20 $O/c3.jsonl; exit 1; }
tail -1 $O/c3.jsonl
timeout -k 10 400 python -u tools/tag_sweep_marginal.py c4 3 "spec=" "nospec=GTF_TAG_SPEC:0" > $O/c4.jsonl 2>&1 || { tail -20 $O/c4.jsonl; exit 1; }
tail -1 $O/c4.jsonl
