"""Per-stage device timing on the benchmark workload (diagnostics, not the bench).

Times (HIP events, median of R repeats) each piece of the pass separately:
message passing (scan + extrapolate), and node-op sequences / single ops on the
post-extrapolation state, restoring the inputs before every repeat.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gtf import synth  # noqa: E402
from gtf.device import DeviceGraph  # noqa: E402
from gtf.params import Params  # noqa: E402


def timeit(d, snap, fn, R=20):
    ts = []
    for _ in range(R):
        d.restore(snap)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c4"
    sched = (sys.argv[2] != "nosched") if len(sys.argv) > 2 else True
    p = Params()
    g = synth.workload(wl)
    d = DeviceGraph(g, schedule=sched)
    snap0 = d.snapshot()
    out = {"workload": wl, "edges": g.n_edges, "nodes": g.n_nodes, "n_g": d.n_g}
    out["full_pass"] = timeit(d, snap0, lambda: d.full_pass(p))
    out["message_passing"] = timeit(d, snap0, lambda: d.message_passing(p))
    d.restore(snap0)
    d.message_passing(p)
    snap1 = d.snapshot()
    seqs = {
        "extrap_ops": ["priors_uts", "reweight_uts", "priors_uts", "reweight_uts", "degree"],
        "update_ops": ["prune", "priors_tse", "priors_uts", "reweight_uts"],
        "cluster_ops": ["cluster_uts", "degree", "mw_uts", "priors_uts"],
        "priors_uts": ["priors_uts"],
        "reweight_uts": ["reweight_uts"],
        "degree": ["degree"],
        "cluster_uts": ["cluster_uts"],
        "all_node_ops": ["ranks", "priors_uts", "reweight_uts", "priors_uts", "reweight_uts", "degree", "prune",
                         "priors_tse", "priors_uts", "reweight_uts", "cluster_uts", "degree", "mw_uts", "priors_uts"],
    }
    for name, ops in seqs.items():
        out[name] = timeit(d, snap1, lambda ops=ops: d.node_ops(ops, p, p.cluster_chi2, p.cluster_kl))
    out["restore_only"] = timeit(d, snap0, lambda: None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
