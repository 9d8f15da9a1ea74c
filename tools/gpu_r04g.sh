#!/bin/bash
# round 4 final evidence: rocprofv3 kernel stats and calibrated HBM counters of the C4 pass and
# of the cold config-5 rotation, the SQ instruction mix, the per-op wave timing of the final
# node kernel (GTF_OP_TIMING build), and the N > 1 bench path rehearsed with 4 ranks on the
# one GPU over gloo. Stops at the first failure.
set -o pipefail
O=gpurun_out/r04/g
mkdir -p $O
bash tools/gpu_profile.sh $O/c4 --steps 20 --warmup 3 --no-c5 --no-dropin || exit 1
python tools/pmc_summary.py $O/c4 profiles/r01_pmc/calib $O/c4/pmc_c4.json c4 > $O/c4/pmc.txt || exit 1
bash tools/gpu_profile_py.sh $O/c5 tools/pkl_time.py 48 || exit 1
python tools/pmc_summary.py $O/c5 profiles/r01_pmc/calib $O/c5/pmc_c5.json c5 ordered 0 > $O/c5/pmc.txt || exit 1
bash tools/gpu_sqmix.sh r04/g/sqmix || exit 1
GTF_OPT_FLUSH=1 GTF_LIB=$PWD/gnn-track-finding_amd/gtf/libgtf_optime.so timeout -k 10 200 python -u tools/op_timing.py $O/op_timing.json > $O/op_timing.log 2>&1 || { tail -20 $O/op_timing.log; exit 1; }
timeout -k 10 500 python -u bench.py --gpus 4 --backend gloo --steps 10 --warmup 2 --no-c5 > $O/bench_gpus4_gloo.json 2> $O/bench_gpus4_gloo.err || { tail -20 $O/bench_gpus4_gloo.err; exit 1; }
echo r04g-done
