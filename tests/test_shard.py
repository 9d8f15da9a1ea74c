"""Single-event sharding (§8e): the host plan on CPU, the exchange protocol over gloo
with world size 2 on CPU, and the sharded pass on the GPU (two ranks on one GPU over
gloo) against the one-GPU pass, bit for bit."""
import os
import socket

import numpy as np
import pytest

from gtf import synth
from gtf.shard import ShardPlan


def _event():
    return synth.event(seed=3, n_tracks=700, fake_mean=synth.C4_FAKE)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_plan_partitions_receivers_and_slots(world):
    g = _event()
    pl = ShardPlan(g, world)
    assert pl.node_lo[0] == 0 and pl.node_hi[-1] == g.n_nodes
    assert (pl.node_lo[1:] == pl.node_hi[:-1]).all()
    assert pl.slot_lo[0] == 0 and pl.slot_hi[-1] == g.n_slots and (pl.slot_lo[1:] == pl.slot_hi[:-1]).all()
    dmax = int(np.diff(g.slot_ptr).max())
    assert (pl.slot_hi - pl.slot_lo).max() <= g.n_slots / world + dmax + 1   # balanced by slots
    owner = np.repeat(np.arange(world), pl.node_hi - pl.node_lo)
    dst = g.slot_dst()
    for r in range(world):
        sched, n_g, n_big = pl.schedule(r)
        assert sorted(sched.tolist()) == list(range(pl.node_lo[r], pl.node_hi[r]))
        assert sum(n_g) + n_big == sched.size
        snd = set(pl.senders(r).tolist())
        # every sender of an owned edge, and every owned node with out-edges, is scanned
        e = g.slot["is_edge"].astype(bool) & (owner[dst] == r)
        assert set(g.slot["slot_src"][e].tolist()) <= snd
        outdeg = np.diff(g.out_ptr)
        assert {v for v in range(pl.node_lo[r], pl.node_hi[r]) if outdeg[v] > 0} <= snd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_allgather_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from gtf.shard import allgather_bytes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    chunk = torch.full((1000,), rank + 7, dtype=torch.uint8)
    out = torch.zeros(1000 * world, dtype=torch.uint8)
    allgather_bytes(chunk, out, "gloo")
    q.put((rank, out.numpy().copy()))
    dist.destroy_process_group()


def test_exchange_allgather_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gloo_allgather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    exp = np.concatenate([np.full(1000, 7, np.uint8), np.full(1000, 8, np.uint8)])
    for r in range(2):
        assert (res[r] == exp).all()


# ---------------------------------------------------------------- GPU (2 ranks, 1 GPU)
PASSES = 2
OUT_NODE = ("has_merged", "merged_state", "merged_cov", "merged_prior", "has_uts", "degree")
OUT_SLOT = ("act", "edge_mw", "uts_rank", "uts_sv", "uts_tau", "uts_cov", "uts_xyzr", "uts_lik", "uts_mw",
            "uts_prior", "uts_lr", "uts_side", "tse_rank", "tse_prior", "tse_mw")


def _shard_worker(rank, world, port, q, backend="gloo"):
    import torch
    import torch.distributed as dist
    from gtf.params import Params
    from gtf.shard import ShardedDeviceGraph
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda:0"))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    g = _event()
    sd = ShardedDeviceGraph(g, rank, world, "cuda:0", backend=backend)
    if backend == "nccl":   # the device all-gather itself (exchange() skips it at world 1)
        from gtf.shard import allgather_bytes
        c = torch.arange(4096, device="cuda:0").to(torch.uint8)
        o = torch.zeros(4096 * world, dtype=torch.uint8, device="cuda:0")
        allgather_bytes(c, o, "nccl")
        assert torch.equal(o[4096 * rank:4096 * (rank + 1)], c)
    p = Params()
    for _ in range(PASSES):
        sd.step(p)
    torch.cuda.synchronize()
    h = sd.d.download(g.copy())
    pl = sd.plan
    nl, nh, sl, sh = (int(x[rank]) for x in (pl.node_lo, pl.node_hi, pl.slot_lo, pl.slot_hi))
    out = {"node": {f: h.node[f][nl:nh] for f in OUT_NODE}, "slot": {f: h.slot[f][sl:sh] for f in OUT_SLOT},
           "replica": {f: h.node[f] for f in ("has_merged", "merged_state", "merged_cov")}, "act": h.slot["act"],
           "flags": sd.d.errors()}
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def _reference_passes():
    from gtf.device import DeviceGraph
    from gtf.params import Params
    g = _event()
    d = DeviceGraph(g)
    for _ in range(PASSES):
        d.full_pass(Params())
    return g, d.download(g.copy())


@pytest.mark.gpu
def test_sharded_path_over_rccl_world1():
    """the RCCL all-gather path of the exchange (one rank: the GPU box has one GPU)"""
    import torch.multiprocessing as mp
    g, ref = _reference_passes()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_shard_worker, args=(0, 1, _free_port(), q, "nccl"))
    p.start()
    _, res = q.get(timeout=300)
    p.join(60)
    assert p.exitcode == 0
    for f in OUT_SLOT:
        a = res["slot"][f]
        assert np.array_equal(a, ref.slot[f], equal_nan=a.dtype.kind == "f"), f
    for f in OUT_NODE:
        assert np.array_equal(res["node"][f], ref.node[f], equal_nan=True), f


@pytest.mark.gpu
def test_sharded_pass_equals_single_gpu_pass():
    import torch.multiprocessing as mp
    g, ref = _reference_passes()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    pl = ShardPlan(g, world)
    for r in range(world):
        nl, nh, sl, sh = (int(x[r]) for x in (pl.node_lo, pl.node_hi, pl.slot_lo, pl.slot_hi))
        for f in OUT_NODE:
            assert np.array_equal(res[r]["node"][f], ref.node[f][nl:nh], equal_nan=True), (r, f)
        for f in OUT_SLOT:
            a, b = res[r]["slot"][f], ref.slot[f][sl:sh]
            assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), (r, f)
        # after the exchange every replica holds every rank's published state
        for f in ("has_merged", "merged_state", "merged_cov"):
            assert np.array_equal(res[r]["replica"][f], ref.node[f], equal_nan=True), (r, f)
        assert np.array_equal(res[r]["act"], ref.slot["act"]), r
