"""graph.renumber (the DeviceGraph "schedule" layout) on the host: a relabelling that
keeps every receiver's slot segment and every sender's out-list in order."""
import numpy as np

from gtf import graph, synth
from gtf.device import schedule_order


def test_renumber_round_trip_and_layout():
    g = synth.event(seed=2, n_tracks=200, fake_mean=synth.C4_FAKE)
    order = np.random.default_rng(1).permutation(g.n_nodes)
    h, perm = graph.renumber(g, order)
    # segments move whole: the new segment of node i' is the old segment of order[i']
    assert np.array_equal(np.diff(h.slot_ptr), np.diff(g.slot_ptr)[order])
    assert np.array_equal(h.slot["act"], g.slot["act"][perm])
    # slot_src relabelled, same sender per slot
    src_old = g.slot["slot_src"][perm]
    assert np.array_equal(np.where(src_old >= 0, np.argsort(order)[np.maximum(src_old, 0)], -1), h.slot["slot_src"])
    # each sender's successors, in order, are the same receivers
    inv = np.argsort(order)
    for u in range(0, g.n_nodes, 97):
        a = g.slot_dst()[g.out_slot[g.out_ptr[u]:g.out_ptr[u + 1]]]
        b = h.slot_dst()[h.out_slot[h.out_ptr[inv[u]]:h.out_ptr[inv[u] + 1]]]
        assert np.array_equal(inv[a], b)
    # the inverse relabelling restores every array
    back, perm2 = graph.renumber(h, np.argsort(order))
    for k in g.node:
        assert np.array_equal(back.node[k], g.node[k], equal_nan=True), k
    for k in g.slot:
        assert np.array_equal(back.slot[k], g.slot[k], equal_nan=g.slot[k].dtype.kind == "f"), k
    assert np.array_equal(back.out_slot, g.out_slot) and np.array_equal(back.slot_ptr, g.slot_ptr)


def test_schedule_order_groups_buckets():
    g = synth.event(seed=5, n_tracks=300, fake_mean=synth.C4_FAKE)
    order = schedule_order(g.slot_ptr)
    assert np.array_equal(np.sort(order), np.arange(g.n_nodes))
    h, _ = graph.renumber(g, order)
    deg = np.diff(h.slot_ptr)
    bucket = np.searchsorted([4, 8, 16, 32, 64], deg)   # 0..5 = g4, g8, g16, g32, g64, beyond
    assert np.all(np.diff(bucket) >= 0)                  # one contiguous node range per bucket


def test_schedule_arrays():
    """gtf_graph.sched_seg and out_sched as DeviceGraph uploads them"""
    from gtf.device import sched_segments, sender_schedule
    g = synth.event(seed=6, n_tracks=150, fake_mean=synth.C4_FAKE)
    order = schedule_order(g.slot_ptr)
    seg = sched_segments(g.slot_ptr, order).reshape(-1, 2)
    assert np.array_equal(seg[:, 0], g.slot_ptr[order]) and np.array_equal(seg[:, 1], g.slot_ptr[order + 1])
    q, counts = sender_schedule(g.out_ptr)
    q = q.reshape(-1, 4)
    od = np.diff(g.out_ptr)
    assert sum(counts) == int((od > 0).sum()) == q.shape[0]
    u = q[:, 0]
    assert np.array_equal(q[:, 1], g.out_ptr[u]) and np.array_equal(q[:, 2], g.out_ptr[u + 1])
    b = np.repeat([0, 1, 2], counts)
    assert np.all(od[u][b == 0] <= 4) and np.all((od[u][b == 1] >= 5) & (od[u][b == 1] <= 8)) and np.all(od[u][b == 2] > 8)


def test_pack_schedule():
    """gtf_graph.pack_ent / pack_wave: every <= 64-slot node once, segments back to back,
    no wavefront over 64 lanes"""
    from gtf.device import pack_schedule
    g = synth.event(seed=8, n_tracks=300, fake_mean=synth.C4_FAKE)
    ent, wave = pack_schedule(g.slot_ptr)
    ent = ent.reshape(-1, 4)
    deg = np.diff(g.slot_ptr)
    assert np.array_equal(np.sort(ent[:, 0]), np.nonzero(deg <= 64)[0])
    assert np.array_equal(ent[:, 1], g.slot_ptr[ent[:, 0]]) and np.array_equal(ent[:, 2], g.slot_ptr[ent[:, 0] + 1])
    size = np.maximum(ent[:, 2] - ent[:, 1], 1)
    for w in range(wave.size - 1):
        a, b = wave[w], wave[w + 1]
        assert a < b and ent[a, 3] == 0
        assert np.array_equal(ent[a + 1:b, 3], np.cumsum(size[a:b])[:-1])
        assert ent[b - 1, 3] + size[b - 1] <= 64
