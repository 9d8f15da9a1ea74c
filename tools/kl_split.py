"""GPU box: config-5 gtf_parabolic_kl (ordered layout) time by bucket -- the launch with
only one in-degree bucket's count left (the others set to 0), fp64."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd")]
import torch  # noqa: E402
from gtf import io, parabolic  # noqa: E402

kat = os.path.join(ROOT, "tests", "golden", "kat134")
g = io.load_event(os.path.join(kat, "event_1_filtered_graph_"), 7, 7)
truth = io.read_truth(os.path.join(kat, "truth_vol7.csv"), g.node["node_id"])
ptr, src = parabolic.in_edge_csr(g)
ptr, src, gnn, tr = parabolic.batch(ptr, src, g.node["gnn"], truth, 256)
k = parabolic.ParabolicKL(ptr, src, gnn, tr, "cuda", ordered=True)
full = list(k._g.count)
print("bucket counts", full, "pairs", k.n_pairs)
out = k.alloc("f64", emp="var")


def timeit():
    for _ in range(5):
        k.run(out, "f64")
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(50):
        k.run(out, "f64")
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / 50 * 1e3


print("all buckets %.1f us" % timeit())
for keep in range(4):
    for i in range(4):
        k._g.count[i] = full[i] if i == keep else 0
    print("bucket %d only (%d nodes): %.1f us" % (keep, full[keep], timeit()))
for i in range(4):
    k._g.count[i] = full[i]
