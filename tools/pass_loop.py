"""C4 passes back to back (tiled layout, staged inputs): device time per pass between two
events, for A/B of builds / env switches and for profilers.
    python tools/pass_loop.py [passes]"""
import json
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
W = int(os.environ.get("GTF_WEDGES", "0"))   # diagnostics: azimuthal wedges (one per XCD) before the tiles
if W > 1:
    from gtf.shard import shard_layout
    gd, _, _, _ = shard_layout(g, W, int(os.environ.get("GTF_WEDGE_TILE", "4096")))
    d = DeviceGraph(gd, "cuda:0", layout="natural")
else:
    d = DeviceGraph(g, "cuda:0", layout="tiled")
snap = d.snapshot(DeviceGraph.PASS_INPUTS)
S = min(K, 50)
d.stage_inputs(S)
d.fill_inputs(snap)
p = Params()
for i in range(5):
    d.use_inputs(i)
    d.full_pass(p)
d.fill_inputs(snap)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
times = []
for r in range(max(1, K // S)):
    d.fill_inputs(snap)
    torch.cuda.synchronize()
    a.record()
    for i in range(S):
        d.use_inputs(i)
        d.full_pass(p)
    b.record()
    torch.cuda.synchronize()
    times.append(a.elapsed_time(b) / S)
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("GTF_")}, "passes": S * len(times),
                  "ms_per_pass": times, "flags": d.errors()}))
