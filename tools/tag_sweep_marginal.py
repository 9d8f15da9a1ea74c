"""A/B of gtf_tag_propagate's sweep forms on C3 / C4 after one pass: per mode (an environment
set), the stage wall time from descending tags (median of K calls, the bench's setting) and the
marginal per-sweep time of the product call between 8 and 264 forced sweeps (flip threshold -1,
the bench line's `stage_sweep`), modes alternated over R rounds; every mode's tags and flips
compared word for word with the first mode's.
usage: python tools/tag_sweep_marginal.py c3|c4 R name=K1:V1+K2:V2 name2=...   ("name=" : defaults)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-track-finding_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gtf import synth  # noqa: E402
from gtf.device import DeviceGraph  # noqa: E402
from gtf.params import Params  # noqa: E402

KEYS = ("GTF_TAG_CSR", "GTF_TAG_KWORD", "GTF_TAG_NPT", "GTF_TAG_PREP_NPT", "GTF_TAG_R", "GTF_TAG_BATCH0",
        "GTF_TAG_PACK", "GTF_TAG_COOP", "GTF_TAG_AHEAD", "GTF_TAG_POLL", "GTF_TAG_PREP_COOP", "GTF_TAG_SPEC")


def parse(arg):
    name, _, rest = arg.partition("=")
    env = {}
    for kv in filter(None, rest.split("+")):
        k, _, v = kv.partition(":")
        env[k] = v
    return name, env


def main():
    wl, R = sys.argv[1], int(sys.argv[2])
    modes = [parse(a) for a in sys.argv[3:]]
    g = synth.workload(wl, seed=0)
    d = DeviceGraph(g, layout="tiled")
    d.full_pass(Params())
    rad = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(g.node["xyzr"][:, 3]))).to(d.device)
    t = np.arange(g.n_nodes, dtype=np.int64)[::-1].copy()
    t_init = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(t))).to(d.device)
    ta = torch.empty_like(t_init)
    nbytes = 4 * g.n_edges + 8 * g.n_nodes

    def wall(reps, **kw):
        ts = []
        for _ in range(reps + 1):
            ta.copy_(t_init)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fl = d.tag_propagation_dev(ta, rad, **kw)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts[1:])), fl

    res = {name: {"stage_ms": [], "sweep_us": []} for name, _ in modes}
    ref = None
    for rnd in range(R):
        for name, env in modes:
            for k in KEYS:
                os.environ[k] = env.get(k, "")
            st, fl = wall(10)
            out = (list(fl), ta.clone())
            if ref is None:
                ref = out
            res[name]["equal"] = res[name].get("equal", True) and out[0] == ref[0] and bool(torch.equal(out[1], ref[1]))
            w8, _ = wall(5, threshold=-1.0, max_sweeps=8)
            w264, _ = wall(5, threshold=-1.0, max_sweeps=264)
            sw = (w264 - w8) / 256 * 1e6
            res[name]["stage_ms"].append(st * 1e3)
            res[name]["sweep_us"].append(sw)
            print(json.dumps({"round": rnd, "mode": name, "stage_ms": st * 1e3, "sweep_us": sw,
                              "frac_of_peak": nbytes / (sw * 1e-6) / 8e12, "sweeps": len(fl)}), flush=True)
    for name, r in res.items():
        r["sweep_us_median"] = float(np.median(r["sweep_us"]))
        r["stage_ms_median"] = float(np.median(r["stage_ms"]))
        r["frac_of_peak"] = nbytes / (r["sweep_us_median"] * 1e-6) / 8e12
    print(json.dumps({"workload": wl, "nodes": g.n_nodes, "edges": g.n_edges, "B_tag": nbytes, "modes": res}))


if __name__ == "__main__":
    main()
