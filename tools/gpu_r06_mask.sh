#!/bin/bash
# round 6: the packed prepare keeping the kept bits between its count and write passes
# (GTF_TAG_PACK_MASK, libgtf.so) against re-gathering the radii (libgtf_nomask.so): tag tests,
# C3 stage A/B, rocprof of the prepare kernel for both builds
set -o pipefail
O=gpurun_out/r06/mask
mkdir -p $O
L=gnn-track-finding_amd/gtf
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "tag" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in mask nomask; do
    lib=$L/libgtf.so; [ $v = nomask ] && lib=$L/libgtf_nomask.so
    GTF_LIB=$lib timeout -k 10 300 python -u tools/tag_sweep_marginal.py c3 2 "$v=" > $O/c3_$v.$r.jsonl 2>&1 || { tail -20 $O/c3_$v.$r.jsonl; exit 1; }
    tail -1 $O/c3_$v.$r.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=list(d['modes'].values())[0]; print('$v', $r, 'stage', round(m['stage_ms_median'],4), 'sweep', round(m['sweep_us_median'],2), m['equal'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in mask nomask; do
  export GTF_LIB=$L/libgtf.so; [ $v = nomask ] && export GTF_LIB=$L/libgtf_nomask.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 -u tools/tag_sweep_marginal.py c3 1 "$v=" > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1); echo "== $v"; grep -i "tag_prep" $f | cut -d, -f1-4
done
