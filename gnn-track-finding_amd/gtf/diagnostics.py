"""The reference's truth-based outlier-masking counts (SURVEY §5 "Metrics / logging"), from
the device's diagnostics outputs -- off the timed path.

The reference's stages print, after their work, how well edge (de)activation matched the
truth particle ids of the hits:

* message_passing (extrapolate_merged_states.py:496-518, counters of :385-402): every
  extrapolated edge (an active out-edge of a sender with a merged state) the chi2 gate
  rejects is an "outlier", correct when its two hits belong to different particles; every
  accepted one counts towards the active edges, correct when they belong to the same one;
* reweight (helper.py:186-225): every active state entry whose new weight falls below the
  threshold is an outlier (its edge is deactivated); the active-edge counters are SET to 1
  (``=`` instead of ``+=``, :199-200) whenever a kept edge is seen;
* cluster (clustering.py:311-369): the states a clustered node left over are outliers (their
  in-edges are deactivated), the states it merged are active edges.

Each printed block is numerator / denominator (correct outliers / outliers), then, when
there was an outlier, tp = correct outliers, fp = outliers - tp, tn = correct active edges,
fn = active edges - tn. ``stage_diagnostics`` runs a stage on a DeviceGraph split into the
reference's calls (the same node-op sequences the fused stage runs in one launch, so the
stage's outputs are the fused stage's) and returns those blocks.
"""
from __future__ import annotations

import numpy as np

from .params import Params


def _block(correct_out, total_out, correct_act, total_act) -> dict:
    b = {"numerator": int(correct_out), "denominator": int(total_out)}
    if total_out:
        b.update(tp=int(correct_out), fp=int(total_out - correct_out), tn=int(correct_act),
                 fn=int(total_act - correct_act))
    return b


def _truth_pair(g, truth, slots):
    """(receiver truth, sender truth) of the given slots"""
    dst = g.slot_dst()[slots]
    src = g.slot["slot_src"][slots]
    return truth[dst], truth[np.maximum(src, 0)]


def message_passing_block(g_before, fresh, truth) -> dict:
    """extrapolate_merged_states.py:496-518 from the state before the stage (g_before, host
    order) and the device's uts_fresh flags after message passing (accepted edges)"""
    S, N = g_before.slot, g_before.node
    src = S["slot_src"]
    ok = (S["is_edge"] == 1) & (S["act"] == 1) & (src >= 0)
    ok &= N["has_merged"][np.maximum(src, 0)] == 1
    ev = np.nonzero(ok)[0]
    tr, ts = _truth_pair(g_before, truth, ev)
    acc = fresh[ev] == 1
    return _block(np.sum(~acc & (tr != ts)), np.sum(~acc), np.sum(acc & (tr == ts)), np.sum(acc))


def reweight_block(g, act_before, act_after, truth) -> dict:
    """helper.py:186-225 for one reweight call: the UTS entries with an active edge before
    it; the active-edge counters keep the reference's '= 1'"""
    S = g.slot
    ent = np.nonzero((S["uts_rank"] >= 0) & (S["is_edge"] == 1) & (act_before == 1))[0]
    tr, ts = _truth_pair(g, truth, ent)
    off = act_after[ent] == 0
    kept = ~off
    return _block(np.sum(off & (tr != ts)), np.sum(off), 1 if np.any(kept & (tr == ts)) else 0,
                  1 if np.any(kept) else 0)


def cluster_block(g, slot_cluster, truth) -> dict:
    """clustering.py:311-369 from the device's slot_cluster diagnostics (1 merged, 2 left)"""
    left = np.nonzero(slot_cluster == 2)[0]
    merged = np.nonzero(slot_cluster == 1)[0]
    tr, ts = _truth_pair(g, truth, left)
    ar, as_ = _truth_pair(g, truth, merged)
    return _block(np.sum(tr != ts), left.size, np.sum(ar == as_), merged.size)


def stage_diagnostics(g, stage: str, truth, p: Params = None, chi2=None, kl=None, key="tse", device="cuda"):
    """Run ``stage`` ("cluster", "extrapolate" or "update") on a copy of ``g`` on the device,
    split into the reference's calls, and return (output graph, [blocks in print order]).
    ``truth``: truth particle id per node (host order)."""
    from .device import DeviceGraph
    p = p or Params()
    truth = np.asarray(truth)
    h = g.copy()
    d = DeviceGraph(h, device)
    d.set_diagnostics(node_err=True, edge_chi2=False, slot_cluster=(stage == "cluster"))
    d.clear_errors()
    d.clear_diagnostics()
    blocks = []

    def act():
        return d.t["act"].cpu().numpy().copy()

    if stage == "cluster":
        d.cluster(key, chi2, kl, p)
        d.download(h)
        blocks.append(cluster_block(h, d.diagnostics()["slot_cluster"], truth))
    elif stage == "extrapolate":
        d.message_passing(p)                                        # :406-451
        d.download(h)
        blocks.append(message_passing_block(g, h.slot["uts_fresh"], truth))
        for _ in range(2):                                          # :554-559
            d.node_ops(["priors_uts"], p)
            a0 = act()
            d.node_ops(["reweight_uts"], p)
            d.download(h)
            blocks.append(reweight_block(h, a0, h.slot["act"], truth))
        d.node_ops(["degree"], p)
        d.download(h)
    elif stage == "update":
        d.node_ops(["prune", "priors_tse", "priors_uts"], p)         # remove_state_metadata.py:31-52
        a0 = act()
        d.node_ops(["reweight_uts"], p)                              # :53
        d.download(h)
        blocks.append(reweight_block(h, a0, h.slot["act"], truth))
    else:
        raise ValueError("stage must be 'cluster', 'extrapolate' or 'update'")
    d.raise_errors()
    return h, blocks
