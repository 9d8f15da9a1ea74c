"""Time each degree bucket of gtf_parabolic_kl alone on config 5 (diagnostics)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-track-finding_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gtf import io, parabolic  # noqa: E402


def main():
    kat = os.path.join(ROOT, "tests", "golden", "kat134")
    g = io.load_event(os.path.join(kat, "event_1_filtered_graph_"), 7, 7)
    truth = io.read_truth(os.path.join(kat, "truth_vol7.csv"), g.node["node_id"])
    ptr, src = parabolic.in_edge_csr(g)
    ptr, src, gnn, tr = parabolic.batch(ptr, src, g.node["gnn"], truth, 256)
    k = parabolic.ParabolicKL(ptr, src, gnn, tr, "cuda:0")
    out = k.alloc("f64", emp="var")
    full = [k._g.count[i] for i in range(4)]
    res = {"counts": full}
    for name, keep in (("all", (0, 1, 2, 3)), ("b0", (0,)), ("b1", (1,)), ("b2", (2,)), ("b3", (3,))):
        for i in range(4):
            k._g.count[i] = full[i] if i in keep else 0
        for _ in range(3):
            k.run(out, "f64")
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(40):           # back to back: device time per launch
            k.run(out, "f64")
        b.record()
        torch.cuda.synchronize()
        res[name] = a.elapsed_time(b) / 40
    print(json.dumps(res))


if __name__ == "__main__":
    main()
