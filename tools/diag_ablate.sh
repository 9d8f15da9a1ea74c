set -e
mkdir -p gpurun_out/diag
timeout -k 10 200 python -u tools/node_buckets.py c4 > gpurun_out/diag/buckets.log 2>&1
for a in "" 1 2 3; do
  if [ -n "$a" ]; then export GTF_LIB=$PWD/gnn-track-finding_amd/gtf/libgtf_ablate$a.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu --no-c5 --steps 30 --warmup 3 > gpurun_out/diag/bench_ab$a.log 2>&1
done
echo diag-done
