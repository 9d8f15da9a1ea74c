"""Per-kernel launch statistics from a rocprofv3 --kernel-trace directory, grouped by
(kernel, grid size): the bench command launches the pass kernels on the C4 event and on
the C3 batch, whose grids differ, so each workload's average duration can be read apart
from the other's (rocprofv3 --stats averages every launch of a kernel name together).

    python tools/kstats_by_grid.py <rocprof dir> [out.csv] [--match substr,substr,...]
"""
import csv
import glob
import sys
from collections import defaultdict


def load(d):
    f = sorted(glob.glob(d + "/**/*kernel_trace.csv", recursive=True))
    if not f:
        raise SystemExit("no kernel_trace.csv under %s" % d)
    rows = []
    for p in f:
        rows += list(csv.DictReader(open(p)))
    return rows


def group(rows, match=None):
    g = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if match and not any(m in name for m in match):
            continue
        grid = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
        g[(name, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = []
    for (name, grid), ts in g.items():
        ts.sort()
        out.append({"Name": name, "GridSize": grid, "Calls": len(ts), "AverageNs": sum(ts) / len(ts),
                    "MedianNs": ts[len(ts) // 2], "MinNs": ts[0], "MaxNs": ts[-1], "TotalNs": sum(ts)})
    out.sort(key=lambda x: -x["TotalNs"])
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    for a in sys.argv[1:]:
        if a.startswith("--match="):
            match = a.split("=", 1)[1].split(",")
    st = group(load(args[0]), match)
    if len(args) > 1:
        with open(args[1], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(st[0].keys()))
            w.writeheader()
            w.writerows(st)
    for r in st[:40]:
        print("%-70s grid %9d  x%-4d avg %9.2f us  med %9.2f us" % (r["Name"][:70], r["GridSize"], r["Calls"],
                                                                   r["AverageNs"] / 1e3, r["MedianNs"] / 1e3))


if __name__ == "__main__":
    main()
