"""The graph-static slot tables the node kernel reads (gtf.device: slot_class / slot_sflags /
slot_xclass, slot_static, slot_sxzr; include/gtf.h ABI v5 / v7) against a brute-force
statement of their definitions, on receivers of every segment size up to 64 slots. No GPU."""
import numpy as np

from gtf import synth
from gtf.device import STATIC_MAX, slot_classes, slot_sender_xzr, slot_static_words


def _brute_masks(g, v):
    lo, hi = int(g.slot_ptr[v]), int(g.slot_ptr[v + 1])
    src = g.slot["slot_src"][lo:hi].astype(np.int64)
    ok = src >= 0
    layer = np.where(ok, g.node["layer"][np.maximum(src, 0)], np.nan)
    sx = np.where(ok, g.node["gnn"][np.maximum(src, 0), 0], np.nan)
    d = hi - lo
    lm, xm = [], []
    for i in range(d):
        lm.append(sum(1 << j for j in range(d) if j == i or layer[j] == layer[i]))
        xm.append(sum(1 << j for j in range(d) if j == i or sx[j] == sx[i]))
    return lo, d, lm, xm, sx


def test_slot_tables_match_definitions():
    g = synth.workload("c2", seed=3)
    cls, sfl, xcls = slot_classes(g)
    words = slot_static_words(g, cls, sfl)
    sxzr = slot_sender_xzr(g)
    deg = np.diff(g.slot_ptr)
    rx = g.node["gnn"][:, 0]
    rng = np.random.default_rng(0)
    picks = []
    for lo, hi in ((1, 2), (3, 4), (5, 8), (9, 16), (17, 32), (33, 64), (65, 10 ** 9)):
        v = np.nonzero((deg >= lo) & (deg <= hi))[0]
        picks += list(rng.choice(v, size=min(25, v.size), replace=False)) if v.size else []
    assert any(deg[v] > 32 for v in picks), "no 33..64-slot receiver in the sample"
    for v in picks:
        lo, d, lm, xm, sx = _brute_masks(g, v)
        for i in range(d):
            k = lo + i
            c, xc = int(cls[k]), int(xcls[k])
            if d <= 32:
                assert c == lm[i] | (xm[i] << 32) and xc == 0
            elif d <= 64:
                assert c == lm[i] and xc == xm[i]
            else:
                assert c == 0 and xc == 0
            assert int(sfl[k]) == int(sx[i] < rx[v])
            w = int(words[k])
            if d <= STATIC_MAX:
                assert w & 0xff == lm[i] and (w >> 8) & 0xff == xm[i]
                assert (w >> 16) & 1 == g.slot["is_edge"][k] and (w >> 17) & 1 == g.slot["rev_edge"][k]
                assert (w >> 18) & 1 == sfl[k]
            else:
                assert w == 0
            s = int(g.slot["slot_src"][k])
            if s >= 0:
                assert np.array_equal(sxzr[k], g.node["gnn"][s, [0, 2, 3]])
            else:
                assert np.isnan(sxzr[k]).all()
