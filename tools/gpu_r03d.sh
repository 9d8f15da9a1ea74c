#!/bin/bash
# round 3: instruction mix of the pass kernels, and counters of the cold config-5 KL kernel
# in the ordered and tiled layouts. Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r03d
mkdir -p $O
bash tools/gpu_sqmix.sh r03d/sqmix || exit 1
cd /tmp && export TMPDIR=/tmp
for t in 0 8748; do
  GTF_KL_TILE=$t timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$O/kl$t/fetch -o run --output-format csv -- python3 $R/tools/pkl_time.py 24 > $R/$O/kl$t.fetch.log 2>&1 || exit 1
  GTF_KL_TILE=$t timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-trace -d $R/$O/kl$t/sq -o run --output-format csv -- python3 $R/tools/pkl_time.py 24 > $R/$O/kl$t.sq.log 2>&1 || exit 1
  GTF_KL_TILE=$t timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace -d $R/$O/kl$t/tcc -o run --output-format csv -- python3 $R/tools/pkl_time.py 24 > $R/$O/kl$t.tcc.log 2>&1 || exit 1
done
echo r03d-done
