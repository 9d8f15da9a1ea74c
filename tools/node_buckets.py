"""Time the clustering node kernel per lane-group bucket on C4 (diagnostics): the
pass up to clustering runs once, then gtf_cluster is timed with one bucket's count
kept and the others zeroed (nodes beyond 64 slots are always run)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-track-finding_amd")]

import torch  # noqa: E402

from gtf import synth, _native as nat  # noqa: E402
from gtf.device import DeviceGraph  # noqa: E402
from gtf.params import Params  # noqa: E402


def main():
    p = Params()
    g = synth.workload(sys.argv[1] if len(sys.argv) > 1 else "c4")
    d = DeviceGraph(g)
    d.message_passing(p)
    d.node_ops(["priors_uts", "reweight_uts", "priors_uts", "reweight_uts", "degree", "prune", "priors_tse",
                "priors_uts", "reweight_uts"], p)
    snap = d.snapshot()
    full = list(d.n_g)
    res = {"n_g": full, "n_big": d.n_big}
    cp = d.cparams(p)
    for name, keep in (("all", (0, 1, 2, 3, 4)), ("g4", (0,)), ("g8", (1,)), ("g16", (2,)), ("g32", (3,)),
                       ("g64", (4,)), ("none", ())):
        cg = nat.GtfGraph()
        ctypes.memmove(ctypes.byref(cg), ctypes.byref(d.cg), ctypes.sizeof(cg))
        cg.n_g4, cg.n_g8, cg.n_g16, cg.n_g32, cg.n_g64 = [full[i] if i in keep else 0 for i in range(5)]
        ts = []
        for r in range(12):
            d.restore(snap)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            nat.check(d.lib.gtf_cluster(ctypes.byref(cg), ctypes.byref(d.cn), ctypes.byref(d.cuts),
                                        ctypes.byref(d.ce), 1, p.cluster_chi2, p.cluster_kl, ctypes.byref(cp),
                                        d.ptr("ws"), d.stream))
            b.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(a.elapsed_time(b))
        res[name] = sorted(ts)[len(ts) // 2]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
