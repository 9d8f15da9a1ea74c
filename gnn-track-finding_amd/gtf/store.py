"""Compact on-disk form of the packed graph, beside the reference's gpickles.

The reference hands every stage's output to the next one as one pickled networkx
graph per subgraph (helper.save_network, helper.py:585-587), which dominates its
end-to-end time once the kernels are fast. Here a stage's graph is one ``.npz``
holding the TrackGraph arrays as they sit in HBM (CSR pointers, the out view, the
node and slot field arrays), so saving is a handful of contiguous writes and
loading goes straight to a DeviceGraph upload. Groups of node ids (candidates,
fragments) are stored as CSR ``ptr`` / ``ids`` pairs.
"""
from __future__ import annotations

import numpy as np

from .graph import NODE_FIELDS, SLOT_FIELDS, TrackGraph, check_layout, empty_arrays

FORMAT = "gtf-trackgraph-1"


def save_graph(path: str, g: TrackGraph, vivl=None, compressed: bool = False) -> None:
    arrs = {"format": np.array(FORMAT), "slot_ptr": g.slot_ptr, "out_ptr": g.out_ptr, "out_slot": g.out_slot,
            "n_subgraphs": np.array(g.n_subgraphs, np.int64)}
    arrs.update({"node__" + k: v for k, v in g.node.items()})
    arrs.update({"slot__" + k: v for k, v in g.slot.items()})
    if vivl is not None:
        arrs["vivl"] = np.asarray(vivl, np.float64)
    (np.savez_compressed if compressed else np.savez)(path, **arrs)


def load_graph(path: str):
    """-> (TrackGraph, vivl or None). Fields missing from the file keep their
    defaults (graph.NODE_FIELDS / SLOT_FIELDS); unknown fields are an error."""
    with np.load(path, allow_pickle=False) as z:
        if "format" not in z.files or str(z["format"]) != FORMAT:
            raise ValueError("%s is not a %s file" % (path, FORMAT))
        sp = z["slot_ptr"].astype(np.int32)
        N, S = sp.shape[0] - 1, int(sp[-1])
        node, slot = empty_arrays(NODE_FIELDS, N), empty_arrays(SLOT_FIELDS, S)
        for k in z.files:
            if k.startswith("node__"):
                name = k[6:]
                if name not in NODE_FIELDS:
                    raise ValueError("unknown node field %r" % name)
                node[name] = z[k].astype(NODE_FIELDS[name][0]).reshape(node[name].shape)
            elif k.startswith("slot__"):
                name = k[6:]
                if name not in SLOT_FIELDS:
                    raise ValueError("unknown slot field %r" % name)
                slot[name] = z[k].astype(SLOT_FIELDS[name][0]).reshape(slot[name].shape)
        g = TrackGraph(N, S, sp, z["out_ptr"].astype(np.int32), z["out_slot"].astype(np.int32), node, slot,
                       int(z["n_subgraphs"]))
        vivl = z["vivl"].copy() if "vivl" in z.files else None
    check_layout(g)
    return g, vivl


def save_groups(path: str, groups, **arrays) -> None:
    ptr = np.zeros(len(groups) + 1, np.int64)
    ptr[1:] = np.cumsum([len(x) for x in groups])
    ids = np.concatenate([np.asarray(x, np.int64) for x in groups]) if groups else np.zeros(0, np.int64)
    np.savez(path, ptr=ptr, ids=ids, **arrays)


def load_groups(path: str):
    """-> (list of node-id arrays, dict of the other arrays)"""
    with np.load(path, allow_pickle=False) as z:
        ptr, ids = z["ptr"], z["ids"]
        rest = {k: z[k].copy() for k in z.files if k not in ("ptr", "ids")}
    return [ids[ptr[i]:ptr[i + 1]].copy() for i in range(len(ptr) - 1)], rest
