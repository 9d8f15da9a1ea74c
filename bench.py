#!/usr/bin/env python
"""Benchmark: edges/s of the fused extrapolate -> update -> KL-clustering pass.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c3|c2]

One step = one fused pass (gtf_pass: k_sender_scan, k_extrapolate, fused node
kernel) over one synthetic TrackML-shaped event held in HBM, preceded by a
device-to-device restore of the arrays the pass mutates (activation mask,
state-dict ranks, merged states) so every step processes the same input; the
restore is inside the timed region. Default workload "c4" = BASELINE.json
configs[3], a pileup-200-shaped event (~180k hits, ~1.0M directed edges),
the config the north-star 1-GPU target is quoted on; it fits one GPU.

Multi-GPU (torchrun, one process per GPU): every rank processes its own event
(seed differs per rank) -- events are independent, so there is no data-path
collective ("scaling": "weak"); the barrier and max-over-ranks timing bracket
the timed steps. value = edges of all ranks x steps / max elapsed.

The CPU baseline (rank 0, N = 1 only) times the repository's NumPy restatement
of the same pass (oracle/gtf_oracle.py, kind "port", 1 core) on a bounded
sample event of the same generator.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402


def cpu_baseline(n_tracks, params):
    """NumPy restatement of the pass on a bounded sample (1 core)."""
    import gtf_oracle as O
    from gtf import synth
    g = synth.event(seed=12345, n_tracks=n_tracks, fake_mean=synth.C4_FAKE)
    t0 = time.perf_counter()
    O.full_pass(g, params)
    dt = time.perf_counter() - t0
    return {"value": g.n_edges / dt, "unit": "edges/s", "cores": 1, "kind": "port",
            "sample": "oracle/gtf_oracle.full_pass (NumPy restatement) on one synthetic event of %d hits / "
                      "%d directed edges (pileup-200 density), %.1f s" % (g.n_nodes, g.n_edges, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c4", choices=["c2", "c3", "c4"])
    ap.add_argument("--cpu-tracks", type=int, default=4000, help="CPU-baseline sample size (tracks)")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from gtf import synth
    from gtf.device import DeviceGraph
    from gtf.params import Params
    from gtf import roofline as rf

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = "cuda:%d" % local
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(dev))

    def barrier():
        if world > 1:
            dist.barrier()

    p = Params()
    g = synth.workload(args.workload, seed=1000 * rank)
    d = DeviceGraph(g, dev)
    snap = d.snapshot(DeviceGraph.PASS_INPUTS)
    K, W = args.steps, args.warmup
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(K)]
    for row in evs:      # torch creates the HIP event on first record
        for e in row:
            e.record()
    handles = [[e.cuda_event for e in row] for row in evs]

    d.clear_errors()
    for _ in range(W):
        d.restore(snap)
        d.full_pass(p)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        d.restore(snap)
        d.full_pass(p, events=handles[i])
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    flags = d.errors()

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    edges = torch.tensor([float(g.n_edges)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(edges, op=dist.ReduceOp.SUM)
    elapsed = float(t.item())
    total_edges = float(edges.item())

    scan = np.mean([evs[i][0].elapsed_time(evs[i][1]) for i in range(K)])
    extr = np.mean([evs[i][1].elapsed_time(evs[i][2]) for i in range(K)])
    node = np.mean([evs[i][2].elapsed_time(evs[i][3]) for i in range(K)])
    kernels = {"k_sender": scan, "k_extrapolate": extr, "k_node_seq": node}
    # roofline for the dominant kernel (algorithmic bytes, gtf/roofline.py)
    if node >= scan + extr:
        name, ms, nbytes = "k_node_seq (node-local stages)", node, rf.node_bytes(g.n_edges, g.n_nodes)
    else:
        name, ms, nbytes = "k_sender+k_extrapolate", scan + extr, rf.extrap_bytes(g.n_edges, g.n_nodes)
    achieved = nbytes / (ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.cpu_tracks, p)

    if rank == 0:
        out = {
            "metric": "edges/sec (extrapolate+update+KL) on TrackML hit graph; 1/2/4/8-GPU scaling",
            "value": total_edges * K / elapsed,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded TrackML-shaped generator, gtf/synth.py)",
            "config": {"workload": {"c4": "pileup-200 TrackML-shaped event (configs[3]) per GPU",
                                    "c3": "64 C2-like events fused into one CSR per GPU (configs[2])",
                                    "c2": "single ~30k-hit / ~90k-edge event per GPU (configs[1])"}[args.workload],
                       "nodes_per_gpu": g.n_nodes, "directed_edges_per_gpu": g.n_edges,
                       "parallelism": "event-parallel x%d (no collective)" % world,
                       "pass": "gtf_pass: extrapolate (a6-a8) + update (a3,a9,a10x2,a11) + KL cluster (a12-a14)"},
            "kernel_ms": {k: round(float(v), 5) for k, v in kernels.items()},
            "roofline": {"bound": "hbm", "kernel": name, "achieved": achieved, "peak": rf.HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / rf.HBM_PEAK_GBS, "traffic": None,
                         "algorithmic_bytes": nbytes},
            "cpu_baseline": cpu,
            "device_error_flags": flags,
        }
        if cpu:
            out["speedup_vs_cpu"] = out["value"] / cpu["value"]
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
