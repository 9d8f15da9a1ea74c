"""Config 5's k_parabolic_kl launches of a rocprofv3 --kernel-trace run of bench.py, split
into the warm-up, the cold rotation (the roofline figure of the bench line) and the hot
relaunches of one batch, by their order in the trace and the launch_sequence the bench
line records per dtype (rocprofv3 --stats averages all of them together).

    python tools/kstats_c5.py <rocprof dir> <bench json line file> [out.json]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kstats_by_grid import load  # noqa: E402


def main():
    d, bj = sys.argv[1], sys.argv[2]
    line = json.loads(open(bj).read().strip().splitlines()[-1])
    c5 = line["c5_parabolic_kl"]
    rows = [r for r in load(d) if "k_parabolic_kl" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = {}
    i = 0
    # the bench runs f64 then f32, each: warm-up, cold rotation, hot relaunches
    for dt in ("f64", "f32"):
        if dt not in c5:
            continue
        seq = c5[dt]["launch_sequence"]
        res = {}
        for part in ("warmup", "cold", "hot"):
            n = int(seq[part])
            ts = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[i:i + n]]
            i += n
            if ts:
                ts.sort()
                res[part] = {"launches": len(ts), "average_ns": sum(ts) / len(ts), "median_ns": ts[len(ts) // 2],
                             "min_ns": ts[0], "max_ns": ts[-1]}
        nb = c5[dt]["roofline"]["algorithmic_bytes_per_launch"]
        if "cold" in res:
            res["cold_frac_of_peak_rocprof"] = nb / (res["cold"]["average_ns"] * 1e-9) / 8e12
        res["bench_line_cold_kernel_ms"] = c5[dt]["kernel_ms"]
        out[dt] = res
    if i != len(rows):
        out["note"] = "%d k_parabolic_kl launches in the trace, %d accounted for" % (len(rows), i)
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
