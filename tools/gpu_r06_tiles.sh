#!/bin/bash
# round 6: the tiled layout's tile size (nodes per tile) on C4 and C3, bench kernels only
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r06/${TAG:-tiles}
mkdir -p $OUT
for T in 4096 1024 2048 8192 16384 65536 4096; do
  timeout -k 10 240 python3 bench.py --no-cpu --no-c5 --no-dropin --tile $T > $OUT/bench_$T.json 2> $OUT/err_$T.log || { tail -5 $OUT/err_$T.log; exit 1; }
  python3 - <<PY
import json
d = json.loads(open("$OUT/bench_$T.json").read().strip().splitlines()[-1])
c3 = d.get("c3_fused_batch") or {}
print("tile", $T, "c4", round(d["ms_per_step"], 5), {k[:12]: round(v * 1e3, 1) for k, v in d["kernel_ms"].items()},
      "c3", round(c3.get("ms_per_step", 0), 4), {k[:12]: round(v * 1e3, 1) for k, v in (c3.get("kernel_ms") or {}).items()})
PY
done
