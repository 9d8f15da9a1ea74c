"""Tag propagation's whole stage (one gtf_tag_propagate call, device-resident tags / radius)
on C4 / C3 after one pass, over the compact kept lists with int32 tags (GTF_TAG_CSR=1) against
the keep-mask sweeps (GTF_TAG_CSR=0), both initial tag orders; wall time median of K calls,
and the tags / flips of the two forms compared word for word (diagnostics).
usage: python tools/tag_stage_time.py c3|c4 [K]"""
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
        for csr in ("1", "0"):
            os.environ["GTF_TAG_CSR"] = csr
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
        res["%s_sweeps" % order] = len(outs["1"][0])
        res["%s_equal" % order] = outs["1"][0] == outs["0"][0] and bool(torch.equal(outs["1"][1], outs["0"][1]))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
