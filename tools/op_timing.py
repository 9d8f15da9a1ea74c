"""Per-op wave timing of the fused node kernel (diagnostics build GTF_OP_TIMING=1):

    GTF_LIB=gnn-track-finding_amd/gtf/ab/libgtf_optime.so python tools/op_timing.py [out.json]

Runs the C4 pass (tiled layout), reads back lane 0's shader-clock stamps of every
wavefront of the node kernel (start, after the slot loads, after each of the 15 ops,
after the stores) and prints, per lane-group size G, the mean cycles of each phase, the
wave lifetime, and the dispatch timeline (when waves start and end relative to the first
one)."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd")]
import torch  # noqa: E402
from gtf import synth, _native as nat  # noqa: E402
from gtf.device import DeviceGraph  # noqa: E402
from gtf.params import Params  # noqa: E402

OPS = ["fresh", "ranks", "priors_uts", "reweight", "priors_uts", "reweight", "degree", "prune", "priors_tse",
       "priors_uts", "reweight", "cluster_uts", "degree", "mw_uts", "priors_uts"]
if os.environ.get("GTF_OPT_FLUSH", "0") == "1":   # a GTF_EARLY_STORE build: OP_FLUSH before the clustering
    OPS.insert(OPS.index("cluster_uts"), "flush")
NP = len(OPS) + 3   # start, after the loads, after each op, after the stores
W = 65536

L = nat.lib()
L.gtf_op_timing.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
L.gtf_op_timing.restype = ctypes.c_int
g = synth.workload(os.environ.get("GTF_OPT_WL", "c4"), seed=0)
d = DeviceGraph(g, "cuda:0", layout="tiled")
snap = d.snapshot(DeviceGraph.PASS_INPUTS)
p = Params()
for _ in range(3):
    d.restore(snap)
    d.full_pass(p)
d.restore(snap)
torch.cuda.synchronize()
assert L.gtf_op_timing(None, 0, 1) == 0
d.full_pass(p)
torch.cuda.synchronize()
buf = np.zeros(W * 24, np.uint64)
assert L.gtf_op_timing(ctypes.c_void_p(buf.ctypes.data), buf.size, 0) == 0
rows = buf.reshape(W, 24).astype(np.int64)
rows = rows[rows[:, 23] > 0]
t0 = rows[:, 20].min()   # real-time clock (100 MHz), aligned across XCDs
RT = 100.0               # ticks per microsecond
out = {"waves": int(rows.shape[0]), "kernel_span_us": float((rows[:, 21].max() - t0) / RT), "by_G": {}}
for G in sorted(set(rows[:, 23].tolist()), reverse=True):
    r = rows[rows[:, 23] == G]
    ph = np.diff(r[:, :NP], axis=1)   # load, the ops, store
    names = ["%02d_%s" % (i, n) for i, n in enumerate(["load"] + OPS + ["store"])]
    out["by_G"][int(G)] = {"waves": int(r.shape[0]),
                           "lifetime_mean": float((r[:, NP - 1] - r[:, 0]).mean()),
                           "lifetime_p90": float(np.percentile(r[:, NP - 1] - r[:, 0], 90)),
                           "lifetime_us_mean": float((r[:, 21] - r[:, 20]).mean() / RT),
                           "start_first_us": float((r[:, 20].min() - t0) / RT),
                           "start_last_us": float((r[:, 20].max() - t0) / RT),
                           "end_last_us": float((r[:, 21].max() - t0) / RT),
                           "phases_mean": {n: float(v) for n, v in zip(names, ph.mean(axis=0))},
                           "phases_p90": {n: float(v) for n, v in zip(names, np.percentile(ph, 90, axis=0))}}
# inside the clustering (words 22 / 19: the states staged, the pair loop done), waves whose
# first lane group clustered
ic = OPS.index("cluster_uts") + 1   # row index of the stamp before the clustering op
for G in sorted(set(rows[:, 23].tolist()), reverse=True):
    r = rows[(rows[:, 23] == G) & (rows[:, 22] > 0) & (rows[:, 19] > 0)]
    if r.shape[0] == 0:
        continue
    out["by_G"][int(G)]["cluster_split"] = {
        "waves": int(r.shape[0]),
        "stage_mean": float((r[:, 22] - r[:, ic]).mean()),
        "pairs_mean": float((r[:, 19] - r[:, 22]).mean()),
        "merge_store_mean": float((r[:, ic + 1] - r[:, 19]).mean()),
        "rest_of_wave_mean": float(((r[:, NP - 1] - r[:, 0]) - (r[:, ic + 1] - r[:, ic])).mean())}
# dispatch timeline: waves resident over time (16 bins)
span = rows[:, 21].max() - t0
edges = np.linspace(0, span, 33)
res = [int(((rows[:, 20] - t0 <= e) & (rows[:, 21] - t0 > e)).sum()) for e in edges[:-1]]
out["resident_waves_at_us"] = {"%.1f" % (e / RT): n for e, n in zip(edges[:-1], res)}
s = json.dumps(out, indent=1)
print(s)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(s)
