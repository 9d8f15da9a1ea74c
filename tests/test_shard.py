"""Single-event sharding (§8e): the host plan (ranges, wedge node order, schedules, halo
lists) on CPU, the exchange collectives over gloo with world size 2 on CPU, and the
sharded pass on the GPU (two ranks on one GPU over gloo; one rank over RCCL) against the
one-GPU pass, bit for bit."""
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
        sched, n_g, n_big, n_g2 = pl.schedule(r)
        assert sorted(sched.tolist()) == list(range(pl.node_lo[r], pl.node_hi[r]))
        assert sum(n_g) + n_big == sched.size and 0 <= n_g2 <= n_g[0]
        deg = np.diff(g.slot_ptr)
        assert (deg[sched[:n_g2]] <= 2).all() and (deg[sched[n_g2:n_g[0]]] > 2).all()
        snd = set(pl.senders(r).tolist())
        # every sender of an owned edge, and every owned node with out-edges, is scanned
        e = g.slot["is_edge"].astype(bool) & (owner[dst] == r)
        assert set(g.slot["slot_src"][e].tolist()) <= snd
        outdeg = np.diff(g.out_ptr)
        assert {v for v in range(pl.node_lo[r], pl.node_hi[r]) if outdeg[v] > 0} <= snd
        osched, n_o = pl.sender_schedule(r)
        q = osched.reshape(-1, 4)
        assert sorted(q[:, 0].tolist()) == sorted(snd) and sum(n_o) == len(snd)
        assert (q[:, 1] == g.out_ptr[q[:, 0]]).all() and (q[:, 2] == g.out_ptr[q[:, 0] + 1]).all()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_split_phases_partition_and_interior_rule(world):
    """ShardPlan.split (the pass in phases, gtf_shard.phases): the interior senders and the
    others partition senders(r); the interior / other slots partition the owned slots; a
    sender is interior exactly when the rank owns it and every receiver of its out-edges
    (brute force), and an owned slot is interior exactly when its sender is -- so nothing
    phase 1a reads is written by the halo exchange (HaloPlan lists) and every owned slot is
    extrapolated once"""
    from gtf.shard import HaloPlan, shard_layout
    g0 = synth.event(seed=4, n_tracks=2000, fake_mean=synth.C4_FAKE)
    g, _, _, cuts = shard_layout(g0, world, 512)
    pl = ShardPlan(g, world, cuts)
    hp = HaloPlan(pl)
    owner = np.repeat(np.arange(world), pl.node_hi - pl.node_lo)
    dst = g.slot_dst()
    n_in = 0
    for r in range(world):
        s_in, s_out, k_in, k_out = pl.split(r)
        snd = pl.senders(r)
        assert np.array_equal(np.sort(np.concatenate([s_in, s_out])), snd)
        assert np.array_equal(np.sort(np.concatenate([k_in, k_out])), np.arange(pl.slot_lo[r], pl.slot_hi[r]))
        brute = [u for u in snd.tolist() if owner[u] == r and
                 all(owner[dst[g.out_slot[i]]] == r for i in range(g.out_ptr[u], g.out_ptr[u + 1]))]
        assert s_in.tolist() == brute
        src, ise = g.slot["slot_src"][k_in], g.slot["is_edge"][k_in].astype(bool)
        assert np.isin(src[ise & (src >= 0)], s_in).all()        # the edges of phase 1a: interior senders'
        src_o = g.slot["slot_src"][k_out]
        assert g.slot["is_edge"][k_out].all() and (src_o >= 0).all() and not np.isin(src_o, s_in).any()
        # phase 1b's slots are exactly the owned out-edges of the other senders (the fused form)
        lo, hi = pl.slot_lo[r], pl.slot_hi[r]
        outs_o = np.concatenate([g.out_slot[g.out_ptr[u]:g.out_ptr[u + 1]] for u in s_out] or [np.zeros(0, np.int64)])
        assert np.array_equal(np.sort(outs_o[(outs_o >= lo) & (outs_o < hi)]), k_out)
        # the halo this rank receives never touches an interior sender or its out-edges
        assert not np.isin(hp.need_nodes[r], s_in).any()
        outs = np.concatenate([g.out_slot[g.out_ptr[u]:g.out_ptr[u + 1]] for u in s_in] or [np.zeros(0, np.int64)])
        assert not np.isin(hp.need_slots[r], outs).any()
        n_in += s_in.size
        if world == 1:
            assert s_out.size == 0 or (owner[s_out] == 0).all()
    assert n_in > 0


@pytest.mark.parametrize("world", [2, 4, 8])
def test_wedge_layout_is_a_permutation_with_small_halo(world):
    from gtf.graph import check_layout
    from gtf.shard import HaloPlan, shard_layout
    g = synth.event(seed=4, n_tracks=3000, fake_mean=synth.C4_FAKE)
    gd, order, slot_perm, cuts = shard_layout(g, world, 512)
    check_layout(gd)
    assert sorted(order.tolist()) == list(range(g.n_nodes))
    assert sorted(slot_perm.tolist()) == list(range(g.n_slots))
    assert np.array_equal(gd.node["gnn"], g.node["gnn"][order])
    assert np.array_equal(gd.slot["slot_key"], g.slot["slot_key"][slot_perm])
    pl = ShardPlan(gd, world, cuts)
    sizes = pl.slot_hi - pl.slot_lo
    assert sizes.max() <= 1.1 * g.n_slots / world + 64          # wedges balanced by slots
    h = HaloPlan(pl)
    halo = sum(x.size for x in h.need_nodes)
    assert halo < 0.1 * g.n_nodes, halo                            # azimuthal wedges: a thin halo
    # against layer-range cuts of the host order, the round-1 partition
    h0 = HaloPlan(ShardPlan(g, world))
    assert halo < 0.5 * sum(x.size for x in h0.need_nodes)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_halo_plan_is_what_the_next_pass_reads(world):
    """rank r needs exactly: the merged state of every sender it scans that another rank
    owns, and the activation of every out-edge of those senders (and of its own) whose
    receiver another rank owns; each item comes from its owner, once"""
    from gtf.shard import HaloPlan
    g = _event()
    pl = ShardPlan(g, world)
    h = HaloPlan(pl)
    on = pl.owner_of_nodes()
    dst = g.slot_dst()
    for r in range(world):
        snd = pl.senders(r)
        exp_n = sorted(u for u in snd.tolist() if on[u] != r)
        exp_s = sorted(int(g.out_slot[e]) for u in snd.tolist() for e in range(g.out_ptr[u], g.out_ptr[u + 1])
                       if on[dst[g.out_slot[e]]] != r)
        assert h.need_nodes[r].tolist() == exp_n and h.need_slots[r].tolist() == exp_s
        got_n, got_s = [], []
        for q in range(world):
            nodes, slots = h.message(q, r)
            assert (on[nodes] == q).all() and (on[dst[slots]] == q).all()
            got_n += nodes.tolist()
            got_s += slots.tolist()
        assert sorted(got_n) == exp_n and sorted(got_s) == exp_s
        # send / receive layouts agree pairwise
        for q in range(world):
            if q != r:
                assert h.lists(q, True)[4][r] == h.lists(r, False)[4][q]


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


def _gloo_alltoall_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from gtf.shard import alltoall_bytes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank r sends (r + 1) * (d + 1) bytes of value 10 r + d to rank d
    send_sizes = [(rank + 1) * (d + 1) for d in range(world)]
    send = torch.cat([torch.full((n,), 10 * rank + d, dtype=torch.uint8) for d, n in enumerate(send_sizes)])
    recv_sizes = [(s + 1) * (rank + 1) for s in range(world)]
    recv = torch.zeros(sum(recv_sizes), dtype=torch.uint8)
    alltoall_bytes(send, recv, send_sizes, recv_sizes, "gloo")
    q.put((rank, recv.numpy().copy(), recv_sizes))
    dist.destroy_process_group()


def test_exchange_alltoall_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gloo_alltoall_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: (a, sz) for r, a, sz in (q.get(timeout=120) for _ in ps)}
    for p in ps:
        p.join(60)
    for r in range(2):
        a, sz = res[r]
        exp = np.concatenate([np.full(n, 10 * s + r, np.uint8) for s, n in enumerate(sz)])
        assert (a == exp).all()


def _gloo_tag_exchange_worker(rank, world, port, q):
    """the sharded tag sweep's buffer protocol (gtf_tag_sweep_shard): owned tags, INT64_MIN
    elsewhere, this rank's flip count at word n + rank, 0 in the other count words"""
    import torch
    import torch.distributed as dist
    from gtf.shard import allreduce_max_i64
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1000
    lo, hi = [0, 300, 1000][rank], [300, 1000, 1000][rank]
    buf = torch.full((n + world,), torch.iinfo(torch.int64).min, dtype=torch.int64)
    buf[lo:hi] = torch.arange(lo, hi, dtype=torch.int64) * 7 - 3000
    buf[n:] = 0
    buf[n + rank] = 11 * (rank + 1)
    allreduce_max_i64(buf, "gloo")
    q.put((rank, buf.numpy().copy()))
    dist.destroy_process_group()


def test_exchange_tag_allreduce_max_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gloo_tag_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    exp = np.concatenate([np.arange(1000, dtype=np.int64) * 7 - 3000, [11, 22]])
    for r in range(2):
        assert np.array_equal(res[r], exp)


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
    sd = ShardedDeviceGraph(g, rank, world, "cuda:0", backend=backend, tile=256)
    if backend == "nccl":   # the device collectives themselves (exchange() skips them at world 1)
        from gtf.shard import allgather_bytes, alltoall_bytes
        c = torch.arange(4096, device="cuda:0").to(torch.uint8)
        o = torch.zeros(4096 * world, dtype=torch.uint8, device="cuda:0")
        allgather_bytes(c, o, "nccl")
        assert torch.equal(o[4096 * rank:4096 * (rank + 1)], c)
        o2 = torch.zeros(4096, dtype=torch.uint8, device="cuda:0")
        alltoall_bytes(c, o2, [4096], [4096], "nccl")
        assert torch.equal(o2, c)
    p = Params()
    for _ in range(PASSES):
        sd.step(p)
    sd.sync()
    torch.cuda.synchronize()
    h = sd.d.download(g.copy())
    nodes, slots = sd.owned_host_nodes(), sd.owned_host_slots()
    out = {"nodes": nodes, "slots": slots, "node": {f: h.node[f][nodes] for f in OUT_NODE},
           "slot": {f: h.slot[f][slots] for f in OUT_SLOT},
           "replica": {f: h.node[f] for f in ("has_merged", "merged_state", "merged_cov")}, "act": h.slot["act"],
           "flags": sd.d.errors(), "halo_bytes": sd.halo_bytes}
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
    nodes, slots = res["nodes"], res["slots"]
    assert nodes.size == g.n_nodes and slots.size == g.n_slots
    for f in OUT_SLOT:
        a = res["slot"][f]
        assert np.array_equal(a, ref.slot[f][slots], equal_nan=a.dtype.kind == "f"), f
    for f in OUT_NODE:
        assert np.array_equal(res["node"][f], ref.node[f][nodes], equal_nan=True), f


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
    assert sorted(np.concatenate([res[r]["nodes"] for r in range(world)]).tolist()) == list(range(g.n_nodes))
    for r in range(world):
        nodes, slots = res[r]["nodes"], res[r]["slots"]
        assert res[r]["flags"] == 0 and 0 < res[r]["halo_bytes"]
        for f in OUT_NODE:
            assert np.array_equal(res[r]["node"][f], ref.node[f][nodes], equal_nan=True), (r, f)
        for f in OUT_SLOT:
            a, b = res[r]["slot"][f], ref.slot[f][slots]
            assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), (r, f)
        # after sync() every replica holds every rank's published state
        for f in ("has_merged", "merged_state", "merged_cov"):
            assert np.array_equal(res[r]["replica"][f], ref.node[f], equal_nan=True), (r, f)
        assert np.array_equal(res[r]["act"], ref.slot["act"]), r


@pytest.mark.parametrize("widen", [1, 2, 5])
def test_widened_schedule_covers_every_receiver_once(widen):
    g = _event()
    pl = ShardPlan(g, 3)
    deg = np.diff(g.slot_ptr)
    sizes = (4, 8, 16, 32, 64)
    for r in range(3):
        sched, n_g, n_big, n_g2 = pl.schedule(r, widen)
        assert sorted(sched.tolist()) == list(range(pl.node_lo[r], pl.node_hi[r])) and n_g2 == 0
        at = 0
        for G, n in zip(sizes, n_g):
            assert (deg[sched[at:at + n]] <= G).all()     # every node fits its group
            at += n


@pytest.mark.gpu
@pytest.mark.parametrize("widen", [1, 2])
def test_widened_shard_pass_equals_single_gpu_pass(widen):
    """one rank (no exchange) with every node on 2x / 4x the lanes: the pass is the same
    bit for bit"""
    from gtf.params import Params
    from gtf.shard import ShardedDeviceGraph
    g, ref = _reference_passes()
    sd = ShardedDeviceGraph(g, 0, 1, "cuda:0", backend="gloo", tile=256, widen=widen)
    for _ in range(PASSES):
        sd.step(Params())
    h = sd.d.download(g.copy())
    for f in OUT_NODE:
        assert np.array_equal(h.node[f], ref.node[f], equal_nan=True), f
    for f in OUT_SLOT:
        assert np.array_equal(h.slot[f], ref.slot[f], equal_nan=h.slot[f].dtype.kind == "f"), f
