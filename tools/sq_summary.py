"""Per-kernel SQ counter sums (mean over dispatches) from tools/gpu_sq.sh output.

    python tools/sq_summary.py SQDIR [OUT.json]
"""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(d + "/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if not any(s in n for s in ("k_sender", "k_extrapolate", "k_node", "k_parabolic")):
            continue
        n = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(n, r["Counter_Name"])].add((f, r["Dispatch_Id"]))   # ids restart in every pass
out = {}
for n, cs in acc.items():
    out[n] = {c: v / max(len(disp[(n, c)]), 1) for c, v in sorted(cs.items())}
for n, cs in out.items():
    w = cs.get("SQ_WAVES", 1)
    print(n)
    for c, v in cs.items():
        print("   %-22s %14.0f  per wave %9.1f" % (c, v, v / w))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
