"""Time the fused pass's node kernel per lane-group bucket on C4 (diagnostics): the
whole pass runs with one bucket's node count kept and the others zeroed (nodes beyond
64 slots always run), node-kernel time from the pass's own HIP events."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-track-finding_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gtf import synth, _native as nat  # noqa: E402
from gtf.device import DeviceGraph  # noqa: E402
from gtf.params import Params  # noqa: E402


def main():
    p = Params()
    g = synth.workload(sys.argv[1] if len(sys.argv) > 1 else "c4")
    d = DeviceGraph(g)
    snap = d.snapshot(DeviceGraph.PASS_INPUTS)
    full = list(d.n_g)
    deg = np.diff(g.slot_ptr)
    res = {"n_g": full, "n_big": d.n_big, "slots_per_bucket": [int(deg[(deg >= lo) & (deg <= hi)].sum())
                                                               for lo, hi in ((0, 4), (5, 8), (9, 16), (17, 32), (33, 64))]}
    cp = d.cparams(p)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    for e in evs:
        e.record()
    h = (ctypes.c_void_p * 5)(*[e.cuda_event for e in evs])
    for name, keep in (("all", (0, 1, 2, 3, 4)), ("g4", (0,)), ("g8", (1,)), ("g16", (2,)), ("g32", (3,)),
                       ("g64", (4,)), ("none", ())):
        cg = nat.GtfGraph()
        ctypes.memmove(ctypes.byref(cg), ctypes.byref(d.cg), ctypes.sizeof(cg))
        cg.n_g4, cg.n_g8, cg.n_g16, cg.n_g32, cg.n_g64 = [full[i] if i in keep else 0 for i in range(5)]
        if len(keep) == 1:   # the bucket's own list at the front of the schedule view, no big nodes
            off = sum(full[:keep[0]])
            cg.sched = ctypes.c_void_p(d.t["sched"].data_ptr() + 4 * off)
            cg.sched_seg = ctypes.c_void_p(d.t["sched_seg"].data_ptr() + 8 * off)
            cg.n_big = 0
        ts = []
        for r in range(12):
            d.restore(snap)
            nat.check(d.lib.gtf_pass_ev(ctypes.byref(cg), ctypes.byref(d.cn), ctypes.byref(d.ctse),
                                        ctypes.byref(d.cuts), ctypes.byref(d.ce), ctypes.byref(cp), d.ptr("ws"),
                                        d.stream, h))
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(evs[2].elapsed_time(evs[3]))
        res[name] = sorted(ts)[len(ts) // 2]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
