"""Print the average duration (us) of the pass kernels from a rocprofv3 --stats directory."""
import csv
import glob
import sys

d, name = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0]))) if f else []
out = []
for r in rows:
    n = r["Name"]
    if any(s in n for s in ("k_sender", "k_extrapolate", "k_node", "k_rec")):
        out.append("%s %.1f us x%s" % (n.split("(")[0][-60:], float(r["AverageNs"]) / 1e3, r["Calls"]))
print(name, " | ".join(out))
