#!/bin/bash
# round 3 re-entry check of the current tree: the sharded tag tests first, then the GPU
# suite, smoke(), the default bench line, and the 2-rank gloo rehearsal of the N > 1 bench.
set -o pipefail
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_tags.py -x -v --timeout 200 --timeout-method thread > $O/pytest_tags.log 2>&1 || { tail -40 $O/pytest_tags.log; exit 1; }
tail -2 $O/pytest_tags.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench-done
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --no-cpu --no-dropin --steps 20 --warmup 3 > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err || { tail -20 $O/bench_gpus2_gloo.err; exit 1; }
echo r03k-done
