"""C4 passes back to back (tiled layout, staged inputs) for a profiler: python tools/pass_loop.py [passes]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd")]
import torch  # noqa: E402
from gtf import synth  # noqa: E402
from gtf.device import DeviceGraph  # noqa: E402
from gtf.params import Params  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
g = synth.workload("c4", seed=0)
d = DeviceGraph(g, "cuda:0", layout="tiled")
snap = d.snapshot(DeviceGraph.PASS_INPUTS)
d.stage_inputs(min(K, 50))
d.fill_inputs(snap)
p = Params()
for i in range(K):
    d.use_inputs(i % min(K, 50))
    d.full_pass(p)
torch.cuda.synchronize()
print("passes", K, "flags", d.errors())
