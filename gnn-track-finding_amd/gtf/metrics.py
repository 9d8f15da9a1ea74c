"""Physics metrics of the extracted candidates: track reconstruction
efficiency and track / particle purities, as src/extract/reconstruction_efficiency.py
computes them, vectorised over arrays (candidate member lists in CSR form, the hit
mapping as columns) instead of pandas row lookups per particle and per candidate.

Reference flow (reconstruction_efficiency.py):
  * reference tracks (:41-91): particles with pT = hypot(px, py) >= 1 GeV (:44-47);
    their hits within [min_volume, max_volume] (:50-59); a particle is a reference
    track when its hits span >= 4 distinct (volume_id, layer_id) (:66-78) and no two
    of them share (volume_id, layer_id, module_id) (:79-81);
  * per candidate, in file order (:118-183): the particle ids of its nodes'
    hit_dissociation, nodes in the candidate's node order and hits in each node's order
    (:125-131); the reconstructed particle = the most frequent id, ties to the id seen
    first (max over a Counter, :132-134); n_good its count;
  * matched when the particle is a reference track, n_good >= 0.5 * its reference hits
    (:150), and track purity n_good / #ids >= 0.5 and particle purity n_good / its hits
    in the region >= 0.5 (:154-163); a particle counts once, at its first matching
    candidate (:166-171);
  * efficiency = reconstructed * 100 / reference tracks, printed with 3 decimals (:213).

A node's hit_dissociation is construct_graph's (helper.py:466-479): the node's unique
hit ids in mapping-row order and each hit's particle id. Integer counting over ~10^3
candidates: host-side NumPy, no kernel.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Optional, Sequence

import numpy as np

PT_CUT = 1.0                  # reconstruction_efficiency.py:46
NUM_DISTINCT_LAYERS = 4       # :66


@dataclasses.dataclass
class HitMapping:
    """Columns of the event's hit mapping (event_truth/*-full-mapping-*.csv)."""
    node_idx: np.ndarray
    hit_id: np.ndarray
    particle_id: np.ndarray
    volume_id: np.ndarray
    layer_id: np.ndarray
    module_id: np.ndarray

    @classmethod
    def from_frame(cls, df):
        return cls(*(df[c].to_numpy(np.int64) for c in ("node_idx", "hit_id", "particle_id", "volume_id",
                                                        "layer_id", "module_id")))


@dataclasses.dataclass
class Result:
    n_reconstructed: int
    n_reference: int
    track_purities: np.ndarray       # one per reconstructed particle, in match order
    particle_purities: np.ndarray
    reconstructed_pid: np.ndarray    # per candidate: majority particle id
    n_good: np.ndarray               # per candidate: its count
    matched: np.ndarray              # per candidate: counted as a reconstruction (first match)

    @property
    def efficiency(self) -> float:
        return self.n_reconstructed * 100 / self.n_reference

    @property
    def efficiency_str(self) -> str:
        return "{:.3f}".format(self.efficiency)   # :214


def high_pt_particles(particle_id, px, py, pt_cut: float = PT_CUT) -> np.ndarray:
    """:44-47: ids of the particles with sqrt(px**2 + py**2) >= pt_cut"""
    px, py = np.asarray(px, np.float64), np.asarray(py, np.float64)
    return np.asarray(particle_id, np.int64)[np.sqrt(px ** 2 + py ** 2) >= pt_cut]


def region_hits(m: HitMapping, truth_hit_id, truth_particle_id, pids, min_volume: int,
                max_volume: int) -> np.ndarray:
    """:50-59: rows of the mapping whose hit the truth file assigns to one of `pids`
    and whose volume lies in [min_volume, max_volume] -> boolean row mask"""
    sel_hits = np.asarray(truth_hit_id, np.int64)[np.isin(np.asarray(truth_particle_id, np.int64), pids)]
    return np.isin(m.hit_id, sel_hits) & (m.volume_id >= min_volume) & (m.volume_id <= max_volume)


def reference_tracks(m: HitMapping, rows: np.ndarray, num_layers: int = NUM_DISTINCT_LAYERS):
    """:63-91 -> (reference particle ids, their hit counts, every region particle's hit
    count as (ids, counts)). `rows` = region_hits mask."""
    pid, vol, lay, mod = m.particle_id[rows], m.volume_id[rows], m.layer_id[rows], m.module_id[rows]
    uniq, inv, nhits = np.unique(pid, return_inverse=True, return_counts=True)
    # distinct (volume, layer) per particle (:67)
    vl = np.unique(np.stack([inv, vol, lay], 1), axis=0)
    n_layers = np.bincount(vl[:, 0], minlength=uniq.size)
    # a (volume, layer, module) occurring twice for a particle (duplicated(keep=False), :79)
    vlm, cnt = np.unique(np.stack([inv, vol, lay, mod], 1), axis=0, return_counts=True)
    dup = np.zeros(uniq.size, bool)
    dup[vlm[cnt > 1, 0]] = True
    good = (n_layers >= num_layers) & ~dup
    return uniq[good], nhits[good], (uniq, nhits)


def node_particles(m: HitMapping, truth_hit_id=None, truth_particle_id=None):
    """construct_graph's hit_dissociation particle lists (helper.py:466-479) as a CSR over
    sorted node ids -> (node ids, ptr, particle ids). A node's hits are its unique hit ids
    in mapping-row order; each hit's particle comes from the truth columns (the mapping's
    own when none are given)."""
    node, hit = m.node_idx, m.hit_id
    # first occurrence of each (node, hit) pair, kept in row order (Series.unique)
    pairs = np.stack([node, hit], 1)
    _, first = np.unique(pairs, axis=0, return_index=True)
    first = np.sort(first)
    node, hit = node[first], hit[first]
    if truth_hit_id is None:
        th, tp = m.hit_id, m.particle_id
    else:
        th, tp = np.asarray(truth_hit_id, np.int64), np.asarray(truth_particle_id, np.int64)
    o = np.argsort(th, kind="stable")
    pos = np.searchsorted(th[o], hit)
    if np.any(pos >= th.size) or np.any(th[o][np.minimum(pos, th.size - 1)] != hit):
        raise ValueError("a mapped hit has no truth row (helper.__get_particle_id .item())")
    part = tp[o][pos]
    order = np.argsort(node, kind="stable")            # group by node, rows in order
    node, part = node[order], part[order]
    ids, starts = np.unique(node, return_index=True)
    ptr = np.append(starts, node.size).astype(np.int64)
    return ids, ptr, part


def candidate_particles(cand_ptr, cand_ids, node_ids, node_ptr, node_part):
    """per candidate, its nodes' particle lists concatenated in node order
    (:125-131) -> (candidate index per entry, particle per entry)"""
    cand_ptr, cand_ids = np.asarray(cand_ptr, np.int64), np.asarray(cand_ids, np.int64)
    k = np.searchsorted(node_ids, cand_ids)
    if np.any(k >= node_ids.size) or np.any(node_ids[np.minimum(k, node_ids.size - 1)] != cand_ids):
        raise ValueError("a candidate node has no hit_dissociation")
    lens = node_ptr[k + 1] - node_ptr[k]
    cand_of_node = np.repeat(np.arange(cand_ptr.size - 1), np.diff(cand_ptr))
    tot = int(lens.sum())
    starts = np.repeat(node_ptr[k], lens)
    offs = np.arange(tot) - np.repeat(np.cumsum(lens) - lens, lens)
    return np.repeat(cand_of_node, lens), node_part[starts + offs]


def majority(n_cand: int, cand_of, part):
    """Counter + max(freq, key=freq.get) per candidate (:132-134): the most frequent id,
    ties to the first seen -> (particle id, count, total ids) per candidate"""
    pos = np.arange(part.size)
    key = np.lexsort((pos, part, cand_of))                 # by candidate, particle, position
    c, p = cand_of[key], part[key]
    new = np.ones(c.size, bool)
    new[1:] = (c[1:] != c[:-1]) | (p[1:] != p[:-1])
    grp = np.flatnonzero(new)
    g_cand, g_part, g_first = c[grp], p[grp], pos[key][grp]
    g_cnt = np.diff(np.append(grp, c.size))
    # best per candidate: max count, then smallest first position
    o = np.lexsort((g_first, -g_cnt, g_cand))
    take = np.ones(o.size, bool)
    take[1:] = g_cand[o][1:] != g_cand[o][:-1]
    best = o[take]
    pid = np.zeros(n_cand, np.int64)
    cnt = np.zeros(n_cand, np.int64)
    pid[g_cand[best]], cnt[g_cand[best]] = g_part[best], g_cnt[best]
    total = np.bincount(cand_of, minlength=n_cand)
    return pid, cnt, total


def reconstruction_efficiency(cand_ptr, cand_ids, m: HitMapping, particle_id, px, py, min_volume: int,
                              max_volume: int, truth_hit_id=None, truth_particle_id=None,
                              node_lists: Optional[Sequence[Sequence[int]]] = None) -> Result:
    """The whole script on arrays. Candidates as CSR (cand_ptr, cand_ids) of node ids in
    file order and node order; `node_lists` optionally gives the candidates' particle
    lists directly (their hit_dissociation as stored in the gpickles) instead."""
    th = m.hit_id if truth_hit_id is None else truth_hit_id
    tpid = m.particle_id if truth_particle_id is None else truth_particle_id
    rows = region_hits(m, th, tpid, high_pt_particles(particle_id, px, py), min_volume, max_volume)
    ref_ids, ref_hits, (reg_ids, reg_hits) = reference_tracks(m, rows)
    n_cand = len(cand_ptr) - 1
    if node_lists is None:
        nid, nptr, npart = node_particles(m, truth_hit_id, truth_particle_id)
        cand_of, part = candidate_particles(cand_ptr, cand_ids, nid, nptr, npart)
    else:
        cand_of = np.repeat(np.arange(n_cand), [len(x) for x in node_lists])
        part = np.concatenate([np.asarray(x, np.int64) for x in node_lists]) if n_cand else np.zeros(0, np.int64)
    pid, n_good, total = majority(n_cand, cand_of, part)
    ri = np.searchsorted(ref_ids, pid)
    is_ref = (ri < ref_ids.size) & (ref_ids[np.minimum(ri, max(ref_ids.size - 1, 0))] == pid) if ref_ids.size \
        else np.zeros(n_cand, bool)
    ref_n = np.where(is_ref, ref_hits[np.minimum(ri, max(ref_hits.size - 1, 0))] if ref_hits.size else 0, 1)
    gi = np.searchsorted(reg_ids, pid)
    reg_n = np.where(is_ref, reg_hits[np.minimum(gi, max(reg_ids.size - 1, 0))] if reg_ids.size else 0, 1)
    good_n = n_good * 1.0
    with np.errstate(divide="ignore", invalid="ignore"):
        tpur = good_n / total
        ppur = good_n / reg_n
    ok = is_ref & (good_n >= 0.5 * ref_n) & (tpur >= 0.5) & (ppur >= 0.5)
    # each particle once, at its first passing candidate (:166-171)
    idx = np.flatnonzero(ok)
    _, first = np.unique(pid[idx], return_index=True)
    first = np.sort(idx[first])
    matched = np.zeros(n_cand, bool)
    matched[first] = True
    return Result(int(first.size), int(ref_ids.size), tpur[first], ppur[first], pid, n_good, matched)


def summary(r: Result) -> Dict[str, object]:
    return {"reconstructed": r.n_reconstructed, "reference": r.n_reference, "efficiency_pct": r.efficiency_str,
            "mean_track_purity": float(np.mean(r.track_purities)) if r.track_purities.size else None,
            "mean_particle_purity": float(np.mean(r.particle_purities)) if r.particle_purities.size else None}
