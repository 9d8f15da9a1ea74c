"""GPU box (GTF_SHARD_WIDEN=k: the widened lane-group schedule): one rank's share of the edge-sharded C4 pass at N = 1, 2, 4, 8 on one GPU
(rank 0's wedge; no exchange; argv: the world sizes, default 1 2 4 8): device time per pass (events around K back-to-back
passes) and host time per pass_() call -- the compute side of the N > 1 bench step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd")]
import torch  # noqa: E402
from gtf import synth  # noqa: E402
from gtf.device import DeviceGraph  # noqa: E402
from gtf.params import Params  # noqa: E402
from gtf.shard import ShardedDeviceGraph  # noqa: E402

g = synth.workload("c4", seed=0)
p = Params()
K = 50
worlds = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
for world in worlds:
    sd = ShardedDeviceGraph(g, 0, world, "cuda:0", backend="gloo")
    snap = sd.d.snapshot(DeviceGraph.PASS_INPUTS)
    sd.d.stage_inputs(K)
    sd.d.fill_inputs(snap)
    for i in range(3):
        sd.d.use_inputs(i)
        sd.pass_(p)
    sd.d.fill_inputs(snap)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for i in range(K):
        sd.d.use_inputs(i)
        sd.pass_(p)
    b.record()
    host = (time.perf_counter() - t0) / K
    torch.cuda.synchronize()
    print("N=%d rank0 slots %d: device %.1f us/pass, host %.1f us/call, halo %d B/pass" %
          (world, int(sd.plan.slot_hi[0] - sd.plan.slot_lo[0]), a.elapsed_time(b) / K * 1e3, host * 1e6,
           sd.halo_bytes), flush=True)
