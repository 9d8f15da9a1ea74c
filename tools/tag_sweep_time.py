"""Tag propagation's sweep kernel on C3 / C4 after one pass (diagnostics): the scheduled form
(lane groups over the sender schedule, k_tag_sweep_sched) against one thread per node
(k_tag_sweep: a graph view without out_sched), K calls back to back between two events.
usage: python tools/tag_sweep_time.py c3|c4 [K]"""
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
    wl = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    g = synth.workload(wl, seed=0)
    d = DeviceGraph(g, layout="tiled")
    d.full_pass(Params())
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rad = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(g.node["xyzr"][:, 3]))).to(d.device)
    ta = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(np.arange(g.n_nodes, dtype=np.int64)[::-1].copy()))).to(d.device)
    tb = torch.empty_like(ta)
    keep = torch.zeros(max(g.n_edges, 1), dtype=torch.uint8, device=d.device)
    proc = torch.zeros(max(g.n_nodes, 1), dtype=torch.uint8, device=d.device)
    cnt = torch.zeros(2, dtype=torch.int32, device=d.device)
    nosched = nat.GtfGraph()
    ctypes.memmove(ctypes.byref(nosched), ctypes.byref(d.cg), ctypes.sizeof(nosched))
    nosched.out_sched = ctypes.c_void_p(0)
    nosched.out_lanes = ctypes.c_void_p(0)
    nosched.n_o4 = nosched.n_o8 = nosched.n_o16 = 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {"workload": wl, "nodes": g.n_nodes, "edges": g.n_edges}
    for name, cg in (("sched", d.cg), ("thread_per_node", nosched)):
        nat.check(d.lib.gtf_tag_prepare(ctypes.byref(cg), vp(rad), vp(keep), vp(proc), vp(cnt), d.stream))
        torch.cuda.synchronize()
        e0.record()
        for i in range(K):
            nat.check(d.lib.gtf_tag_prepare(ctypes.byref(cg), vp(rad), vp(keep), vp(proc), vp(cnt), d.stream))
        e1.record()
        torch.cuda.synchronize()
        prep = e0.elapsed_time(e1) / K
        outs = []
        for rep in range(2):
            e0.record()
            for i in range(K):
                nat.check(d.lib.gtf_tag_sweep(ctypes.byref(cg), vp(keep), vp(proc), vp(ta if i % 2 == 0 else tb),
                                              vp(tb if i % 2 == 0 else ta), vp(cnt[1:2]), d.stream))
            e1.record()
            torch.cuda.synchronize()
            outs.append(e0.elapsed_time(e1) / K)
        res[name] = {"prepare_ms": prep, "sweep_ms": min(outs)}
    nb = 4 * g.n_edges + 8 * g.n_nodes
    for name in ("sched", "thread_per_node"):
        res[name]["sweep_frac_of_peak"] = nb / (res[name]["sweep_ms"] * 1e-3) / 8e12
    print(json.dumps(res))


if __name__ == "__main__":
    main()
