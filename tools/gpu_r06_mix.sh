#!/bin/bash
# round 6: the node kernel's 3..4-slot and <= 2-slot buckets interleaved block by block
# (GTF_NODE_MIX=1, libgtf_mix.so) against bucket after bucket (libgtf.so): parity tests on the
# mixed build, then alternating C4 and C3 bench lines (kernel times between HIP events)
set -o pipefail
O=gpurun_out/r06/mix
mkdir -p $O
L=gnn-track-finding_amd/gtf
GTF_LIB=$L/libgtf_mix.so timeout -k 10 500 python -u -m pytest tests/test_gpu_c4_digest.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_real800.py tests/test_gpu_batches.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in base mix; do
    lib=$L/libgtf.so; [ $v = mix ] && lib=$L/libgtf_mix.so
    GTF_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --no-c5 --no-dropin --no-c3 --steps 30 --warmup 3 > $O/c4_$v.$r.json 2> $O/c4_$v.$r.err || { tail -5 $O/c4_$v.$r.err; exit 1; }
    GTF_LIB=$lib timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --no-c5 --no-dropin --steps 10 --warmup 2 > $O/c3_$v.$r.json 2> $O/c3_$v.$r.err || { tail -5 $O/c3_$v.$r.err; exit 1; }
    python3 -c "
import json,sys
for w in ('c4','c3'):
    d=json.loads(open('$O/%s_$v.$r.json'%w).read().strip().splitlines()[-1])
    print(w, '$v', $r, round(d['ms_per_step'],5), {k[:13]: round(v*1e3,1) for k,v in d['kernel_ms'].items()})
"
  done
done
