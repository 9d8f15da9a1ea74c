"""Load tests/golden/*.npz fixtures into TrackGraphs (test helper)."""
import ast
import os

import numpy as np

from gtf.graph import TrackGraph, NODE_FIELDS, SLOT_FIELDS, empty_arrays

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    sp = z["in__slot_ptr"]
    N, S = sp.shape[0] - 1, int(sp[-1])
    node, slot = empty_arrays(NODE_FIELDS, N), empty_arrays(SLOT_FIELDS, S)
    for k in z.files:
        if k.startswith("in__node__"):
            node[k[10:]] = z[k].copy()
        elif k.startswith("in__slot__"):
            slot[k[10:]] = z[k].copy()
    g = TrackGraph(N, S, sp.astype(np.int32), z["in__out_ptr"].astype(np.int32),
                   z["in__out_slot"].astype(np.int32), node, slot, int(node["sub_id"].max()) + 1 if N else 0)
    out = {k[5:]: z[k] for k in z.files if k.startswith("out__")}
    extra = {k[3:]: z[k] for k in z.files if k.startswith("x__")}
    meta = ast.literal_eval(str(z["meta"]))
    return g, out, extra, meta


def expected_graph(g, out):
    """copy of g with the fixture's expected output arrays swapped in"""
    e = g.copy()
    for k, v in out.items():
        kind, name = k.split("__", 1)
        (e.node if kind == "node" else e.slot)[name] = v.copy()
    return e
