#!/bin/bash
# round 6: C4's tag stage on the packed lists + cooperative sweep vs its default (lane-group prepare, csr1 sweep)
set -o pipefail
O=gpurun_out/r06/coop
mkdir -p $O
timeout -k 10 600 python -u tools/tag_sweep_marginal.py c4 3 "def=" "coop2=GTF_TAG_PREP_NPT:1+GTF_TAG_NPT:2" "coop1=GTF_TAG_PREP_NPT:1+GTF_TAG_NPT:2+GTF_TAG_COOP:1" "p1csr1=GTF_TAG_PREP_NPT:1" > $O/c4.jsonl 2>&1 || { tail -20 $O/c4.jsonl; exit 1; }
tail -1 $O/c4.jsonl
