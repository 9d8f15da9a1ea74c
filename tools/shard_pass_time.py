"""GPU box: one rank's share of the edge-sharded C4 pass at N = 1, 2, 4, 8 on one GPU (rank
0's wedge; no exchange; argv: the world sizes, default 1 2 4 8): device time per pass
(events around K back-to-back passes) and host time per pass_() call -- the compute side
of the N > 1 bench step -- and the same pass in its three phases (gtf_shard.phases,
ShardedDeviceGraph.step): phase 1a (the interior senders and the slots they send to: the
part the halo exchange of the previous pass runs beside), phase 1b (the halo-dependent
senders and slots) and phase 2 (the node kernels), each timed alone over K passes."""
import json
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
worlds = [int(a) for a in sys.argv[1:] if not a.startswith("-")] or [1, 2, 4, 8]
out = []
for world in worlds:
    sd = ShardedDeviceGraph(g, 0, world, "cuda:0", backend="gloo")
    snap = sd.d.snapshot(DeviceGraph.PASS_INPUTS)
    sd.d.stage_inputs(K)

    def timed(fn):
        sd.d.fill_inputs(snap)
        for i in range(3):
            sd.d.use_inputs(i)
            fn()
        sd.d.fill_inputs(snap)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        for i in range(K):
            sd.d.use_inputs(i)
            fn()
        b.record()
        host = (time.perf_counter() - t0) / K
        torch.cuda.synchronize()
        sd.d.use_inputs(None)
        return a.elapsed_time(b) / K * 1e3, host * 1e6

    whole, host = timed(lambda: sd.pass_(p))
    ph = [timed(lambda q=q: sd._phase(p, q))[0] for q in range(3)]
    phased, host_ph = timed(lambda: [sd._phase(p, q) for q in range(3)])
    r = {"world": world, "rank0_slots": int(sd.plan.slot_hi[0] - sd.plan.slot_lo[0]), "pass_us": whole,
         "host_us_per_call": host, "phase_1a_us": ph[0], "phase_1b_us": ph[1], "phase_2_us": ph[2],
         "three_phases_us": phased, "host_us_three_phases": host_ph, "halo_bytes": sd.halo_bytes,
         "split": sd.split_sizes}
    out.append(r)
    print("N=%d rank0 slots %d: pass %.1f us (host %.1f us/call); phases 1a %.1f + 1b %.1f + 2 %.1f us, "
          "back to back %.1f us; split %s; halo %d B/pass" %
          (world, r["rank0_slots"], whole, host, ph[0], ph[1], ph[2], phased, sd.split_sizes, sd.halo_bytes),
          flush=True)
if "--json" in sys.argv:
    print(json.dumps(out))
