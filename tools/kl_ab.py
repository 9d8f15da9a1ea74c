"""GPU box: config-5 gtf_parabolic_kl time, list layout vs ordered layout (fp64 and fp32)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd")]
import torch  # noqa: E402
from gtf import io, parabolic, roofline as rf  # noqa: E402

kat = os.path.join(ROOT, "tests", "golden", "kat134")
g = io.load_event(os.path.join(kat, "event_1_filtered_graph_"), 7, 7)
truth = io.read_truth(os.path.join(kat, "truth_vol7.csv"), g.node["node_id"])
ptr, src = parabolic.in_edge_csr(g)
ptr, src, gnn, tr = parabolic.batch(ptr, src, g.node["gnn"], truth, 256)
for rnd in range(2):
    for ordered in (False, True):
        k = parabolic.ParabolicKL(ptr, src, gnn, tr, "cuda", ordered=ordered)
        for dt in ("f64", "f32"):
            out = k.alloc(dt, emp="var")
            for _ in range(5):
                k.run(out, dt)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            for _ in range(50):
                k.run(out, dt)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / 50
            nb = rf.parabolic_kl_bytes(k.n_nodes, k.n_listed, k.n_slots, k.n_pairs, dt)
            print("ordered=%d %s %.1f us  frac %.3f" % (ordered, dt, ms * 1e3, nb / (ms * 1e-3) / 8e12), flush=True)
