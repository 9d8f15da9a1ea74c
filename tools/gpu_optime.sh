#!/bin/bash
set -o pipefail
O=gpurun_out/optime
mkdir -p $O
GTF_LIB=$PWD/gnn-track-finding_amd/gtf/ab/libgtf_optime.so timeout -k 10 200 python -u tools/op_timing.py $O/op_timing.json > $O/op_timing.log 2>&1 || { tail -20 $O/op_timing.log; exit 1; }
echo done
