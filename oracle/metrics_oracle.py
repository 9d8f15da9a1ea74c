"""CPU oracle for the physics metrics: a plain-Python restatement of
src/extract/reconstruction_efficiency.py, loop for loop over pandas rows and a
collections.Counter, as the reference script runs it.

TEST INFRASTRUCTURE ONLY (see gtf_oracle.py): only tests/ may import it, as the
checker of gtf.metrics. Pinned by tests/golden/metrics_vol7.npz, the reference
script's own outputs on the reference's own candidates (make_golden_metrics.py).
"""
from __future__ import annotations

import itertools
from collections import Counter

import numpy as np
import pandas as pd


def reference_tracks(particles: pd.DataFrame, truth: pd.DataFrame, hits: pd.DataFrame, min_volume: int,
                     max_volume: int):
    """reconstruction_efficiency.py:41-91 -> (reference_tracks_dict, pixel_hits)"""
    particles = particles.assign(pT=lambda row: (np.sqrt(row.px ** 2 + row.py ** 2)))      # :45
    particles = particles.loc[particles.pT >= 1.0]                                       # :47
    particle_ids = particles.particle_id.to_list()
    hit_ids = truth.loc[truth.particle_id.isin(particle_ids)].hit_id.to_list()          # :51-52
    pixel_hits = hits.loc[(hits.hit_id.isin(hit_ids)) & (hits.volume_id >= min_volume)
                          & (hits.volume_id <= max_volume)]                              # :57-59
    ref = {}
    for p in pixel_hits.particle_id.unique():                                            # :70
        ref_track = pixel_hits.loc[pixel_hits.particle_id == p]
        if len(set(zip(ref_track.volume_id, ref_track.layer_id))) >= 4:                  # :73-75
            dup = ref_track[ref_track.duplicated(['volume_id', 'layer_id', 'module_id'], keep=False)]
            if len(dup) == 0:                                                            # :80
                ref[p] = ref_track.hit_id.to_list()
    return ref, pixel_hits


def hit_dissociation(truth_map: pd.DataFrame):
    """helper.construct_graph (helper.py:466-479): node -> particle ids of its unique hits"""
    out = {}
    for node, rows in truth_map.groupby('node_idx'):
        out[int(node)] = [truth_map.loc[truth_map.hit_id == h]['particle_id'].item() for h in rows['hit_id'].unique()]
    return out


def efficiency(candidates, particles_of, reference, pixel_hits):
    """:118-183, 213. candidates: node-id lists in file order / node order;
    particles_of: node -> particle list (hit_dissociation values()[1])."""
    n_reco = 0
    track_purities, particle_purities = [], []
    seen = set()
    for track in candidates:
        ids = list(itertools.chain(*[particles_of[int(n)] for n in track]))             # :125-131
        freq = Counter(ids)
        pid = max(freq, key=freq.get)                                                    # :133
        n_good = freq[pid] * 1.0
        if pid in reference:
            if n_good >= 0.5 * len(reference[pid]):                                      # :150
                track_purity = n_good / len(ids)
                particle_purity = n_good / len(pixel_hits.loc[pixel_hits.particle_id == pid])
                if (track_purity >= 0.5) and (particle_purity >= 0.5):
                    if pid not in seen:
                        seen.add(pid)
                        track_purities.append(track_purity)
                        particle_purities.append(particle_purity)
                        n_reco += 1
    eff = "{:.3f}".format(n_reco * 100 / len(reference))
    return n_reco, len(reference), np.array(track_purities), np.array(particle_purities), eff
