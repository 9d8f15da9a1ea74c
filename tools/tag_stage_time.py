"""Tag propagation's whole stage (one gtf_tag_propagate call, device-resident tags / radius)
on C4 / C3 after one pass, over the compact kept lists with int32 tags (GTF_TAG_CSR=1; csr1 one
packed word per node at the defaults; csr1r4: four kept indices per node in the sweep's second
round (GTF_TAG_R), csr1n1 / csr1n2: one / two nodes per sweep thread (GTF_TAG_NPT), csr1p1 / csr1gp: the one-node-
per-thread / lane-group prepare (GTF_TAG_PREP_NPT), csr1b2: a first batch of 2 sweeps (GTF_TAG_BATCH0)) against the keep-mask sweeps
(GTF_TAG_CSR=0), both initial tag orders; wall time median of K calls,
and the tags / flips of the two forms compared word for word (diagnostics).
usage: python tools/tag_stage_time.py c3|c4 [K [mode,mode...]]"""
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


def main():
    wl = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    only = sys.argv[3].split(",") if len(sys.argv) > 3 else None   # a subset of the modes
    g = synth.workload(wl, seed=0)
    d = DeviceGraph(g, layout="tiled")
    d.full_pass(Params())
    rad = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(g.node["xyzr"][:, 3]))).to(d.device)
    res = {"workload": wl, "nodes": g.n_nodes, "edges": g.n_edges}
    for order in ("ascending", "descending"):
        t = np.arange(g.n_nodes, dtype=np.int64)
        if order == "descending":
            t = t[::-1].copy()
        t_init = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(t))).to(d.device)
        outs = {}
        modes = (("1", {}), ("1r4", {"GTF_TAG_R": "4"}), ("1n1", {"GTF_TAG_NPT": "1"}), ("1n2", {"GTF_TAG_NPT": "2"}),
                 ("1p1", {"GTF_TAG_PREP_NPT": "1"}), ("1gp", {"GTF_TAG_PREP_NPT": "0"}), ("1b2", {"GTF_TAG_BATCH0": "2"}), ("0", {"GTF_TAG_CSR": "0"}))
        keys = ("GTF_TAG_CSR", "GTF_TAG_KWORD", "GTF_TAG_NPT", "GTF_TAG_PREP_NPT", "GTF_TAG_R", "GTF_TAG_BATCH0")
        for csr, env in modes:
            if only and csr not in only:
                continue
            for key in keys:
                os.environ[key] = env.get(key, "")
            ta = torch.empty_like(t_init)
            ts = []
            for _ in range(K + 1):
                ta.copy_(t_init)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                flips = d.tag_propagation_dev(ta, rad)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            outs[csr] = (flips, ta.clone())
            res["%s_csr%s_ms" % (order, csr)] = float(np.median(ts[1:])) * 1e3
        res["%s_sweeps" % order] = len(next(iter(outs.values()))[0])
        if only:
            continue
        res["%s_equal" % order] = all(outs[m][0] == outs["0"][0] and bool(torch.equal(outs[m][1], outs["0"][1]))
                                      for m, _ in modes[:-1])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
