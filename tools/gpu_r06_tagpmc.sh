#!/bin/bash
# round 6: HBM counters (FETCH_SIZE / WRITE_SIZE passes, tools/pmc_summary.py's calibration) of
# the tag stage's kernels on C3, compact-list form only (tools/tag_stage_time.py mode "1")
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/r06/${TAG:-tagpmc}
mkdir -p $OUT
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  d=$(echo $c | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $OUT/$d -o run --output-format csv -- python3 $R/tools/tag_stage_time.py c3 3 ${MODES:-1} > $OUT/$d.log 2>&1 || { tail -5 $OUT/$d.log; exit 1; }
done
python3 - <<PY
import csv, collections, json, numpy as np
def load(p, ctr=None):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        if ctr and r["Counter_Name"] != ctr:
            continue
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        n = n[:n.find("(")] if "(" in n else n
        agg[n.strip()].append(float(r["Counter_Value"]))
    return {k: (float(np.median(v)), len(v)) for k, v in agg.items()}
cal = "$R/profiles/r01_pmc/calib"
cf, cw = load(cal + "/fetch/run_counter_collection.csv"), load(cal + "/write/run_counter_collection.csv")
rf, wf = (1 << 30) / (cf["rd8"][0] * 1024), (1 << 30) / (cw["wr8"][0] * 1024)
f, w = load("$OUT/fetch_size/run_counter_collection.csv"), load("$OUT/write_size/run_counter_collection.csv")
h, m = load("$OUT/tcc_hit_sum/run_counter_collection.csv", "TCC_HIT_sum"), load("$OUT/tcc_hit_sum/run_counter_collection.csv", "TCC_MISS_sum")
res = {}
for k in f:
    if "tag" in k:
        res[k] = {"launches": f[k][1], "fetch_MB": f[k][0] * 1024 * rf / 1e6, "write_MB": w.get(k, (0,))[0] * 1024 * wf / 1e6,
                  "tcc_hit": h.get(k, (None,))[0], "tcc_miss": m.get(k, (None,))[0]}
json.dump(res, open("$OUT/tag_pmc_c3.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
