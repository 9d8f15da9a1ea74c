"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/<round>_pmc/.

    python tools/pmc_summary.py PROFDIR CALIBDIR OUT.json [workload [layout [tile]]]

PROFDIR holds fetch/ and write/ counter passes of bench.py (tools/gpu_profile.sh);
CALIBDIR the same two passes of tools/calib_fetch (kernels that stream exactly
1 GiB with 1-, 8- and 16-byte lanes and write 1 GiB with 8-byte lanes). The
read factor applied to FETCH_SIZE is the measured bytes/FETCH ratio of the
8-byte-lane stream (this repository's kernels load 1-8 bytes per lane); the
MI355X guide's x2 for 16-byte streams is reported beside it for reference.
"""
import csv
import collections
import json
import sys

import numpy as np

NAMES = {
    "k_sender": "k_sender",
    "k_sender_sched": "k_sender",
    "k_sender_sched<false>": "k_sender",
    "k_extrapolate": "k_extrapolate",
    "k_node_multi<1, 3, 4, 3, 4, 5, 6, 2, 3, 4>": "k_node_multi<reweight,update>",
    "k_node_multi<10, 5, 8, 3>": "k_node_multi<cluster> (KL-distance kernel)",
    "k_node_multi<1, 3, 4, 3, 4, 5, 6, 2, 3, 4, 10, 5, 8, 3>": "k_node_multi<update+cluster> (KL-distance kernel)",
    "k_node_multi<11, 1, 3, 4, 3, 4, 5, 6, 2, 3, 4, 10, 5, 8, 3>": "k_node_multi<update+cluster> (KL-distance kernel)",
    "k_node_multi<11, 1, 3, 4, 3, 4, 5, 6, 2, 3, 4, 12, 10, 5, 8, 3>": "k_node_multi<update+cluster> (KL-distance kernel)",
    "k_parabolic_kl<double, false>": "k_parabolic_kl (fp64)",
    "k_parabolic_kl<float, false>": "k_parabolic_kl (fp32)",
    "k_parabolic_kl_win<double, false>": "k_parabolic_kl_win (fp64, tiled layout)",
}


def load(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        n = n[:n.find("(")] if "(" in n else n
        agg[n.strip()].append(float(r["Counter_Value"]))
    return {k: float(np.median(v)) for k, v in agg.items()}


def main():
    prof, calib, out = sys.argv[1:4]
    workload = sys.argv[4] if len(sys.argv) > 4 else "c4"
    layout = sys.argv[5] if len(sys.argv) > 5 else "tiled"
    tile = int(sys.argv[6]) if len(sys.argv) > 6 else 4096
    cf, cw = load(calib + "/fetch/run_counter_collection.csv"), load(calib + "/write/run_counter_collection.csv")
    gib = float(1 << 30)
    read_factor = {k: gib / (cf[k] * 1024) for k in ("rd1", "rd8", "rd16") if k in cf}
    write_factor = gib / (cw["wr8"] * 1024)
    f, w = load(prof + "/fetch/run_counter_collection.csv"), load(prof + "/write/run_counter_collection.csv")
    rf = read_factor["rd8"]
    ks = {}
    for raw, name in NAMES.items():
        if raw in f:
            ks[name] = {"FETCH_SIZE_KiB": f[raw], "WRITE_SIZE_KiB": w.get(raw, 0.0),
                        "hbm_bytes_per_launch": f[raw] * 1024 * rf + w.get(raw, 0.0) * 1024 * write_factor}
    if "k_sender" in ks and "k_extrapolate" in ks:
        ks["k_sender+k_extrapolate"] = {"hbm_bytes_per_launch": ks["k_sender"]["hbm_bytes_per_launch"] +
                                        ks["k_extrapolate"]["hbm_bytes_per_launch"]}
    # the event the counters were taken on: bench.py's own line in the trace pass
    edges = nodes = None
    try:
        for ln in open(prof + "/trace.log"):
            if ln.startswith("{"):
                c = json.loads(ln)["config"]
                edges, nodes = c.get("directed_edges_per_gpu"), c.get("nodes_per_gpu")
    except (OSError, ValueError, KeyError):
        pass
    res = {"workload": workload, "layout": layout, "tile": tile, "edges": edges, "nodes": nodes, "read_factor_applied": rf, "write_factor_applied": write_factor,
           "calibration_bytes_per_FETCH_KiB": {k: v for k, v in read_factor.items()},
           "note": "FETCH_SIZE/WRITE_SIZE in KiB per launch (median over launches); hbm bytes = "
                   "FETCH*1024*read_factor + WRITE*1024*write_factor, factors measured by tools/calib_fetch",
           "kernels": ks}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
