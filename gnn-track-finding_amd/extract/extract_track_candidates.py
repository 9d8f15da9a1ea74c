"""Drop-in for src/extract/extract_track_candidates.py (same CLI flags
-i -c -r -f -p -n -s -t -e -z -a -b).

The per-candidate work -- CCA over the activated edges, close-proximity merging,
the one-hit-per-layer check, rotate_track, the xy / rz Kalman fits and their
chi-square p-values -- runs on the GPU (gtf_extract_candidates). The host keeps the
stage's file handling and networkx bookkeeping: it reads the numbered gpickles
(:383-391), gives the kernel each candidate's node order as networkx produces it
(subgraph views iterate a set for small components), applies the reference's in-place
GNN_Measurement mutation for merged nodes, and writes candidates (this iteration's
first, then the previous ones, :444-455), pvals.csv, remaining and fragments
(:423-430, :464-467).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import networkx as nx  # noqa: E402
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

from gtf import extract as ex  # noqa: E402
from gtf import stages as _st  # noqa: E402
from gtf.graph import pack  # noqa: E402

SUFFIX = "_subgraph.gpickle"


def read_numbered(d):
    """the stage's own reader: 0_subgraph.gpickle, 1_... until one is missing (:383-391)"""
    import pickle
    out, i = [], 0
    while os.path.isfile(d + str(i) + SUFFIX):
        with open(d + str(i) + SUFFIX, "rb") as f:
            out.append(pickle.load(f))
        i += 1
    return out


def candidates_nx(subGraph):
    """CCA (:332-346) as networkx objects: the candidate graphs the reference builds,
    in its order, with their node order"""
    subCopy = subGraph.copy()
    off = [e for e in subCopy.edges() if subCopy[e[0]][e[1]]["activated"] == 0]
    if not off:
        return [subCopy]
    subCopy.remove_edges_from(off)
    return [subCopy.subgraph(c).copy() for c in nx.weakly_connected_components(subCopy)]


def extract(subGraphs, params: ex.Params, iteration):
    """-> (extracted graphs, pvals_xy, pvals_zr, remaining graphs, fragment graphs)"""
    g = pack(subGraphs)
    cands = [candidates_nx(s) for s in subGraphs]
    pos, vi = {}, 0
    for s in subGraphs:
        for n in s.nodes:
            pos[(id(s), n)] = vi
            vi += 1
    order_key = np.zeros(g.n_nodes, np.int32)
    for s, cs in zip(subGraphs, cands):
        for c in cs:
            for k, n in enumerate(c.nodes):
                order_key[pos[(id(s), n)]] = k
    vivl = np.array([[float(a["vivl_id"][0]), float(a["vivl_id"][1])] for s in subGraphs
                     for _, a in s.nodes(data=True)]).reshape(-1, 2)
    res = ex.run(g, vivl, params, order_key=order_key)
    # the reference's in-place GNN_Measurement mutation of merged nodes (:111-114)
    moved = np.nonzero(np.any(res["gnn"] != g.node["gnn"], axis=1))[0]
    vi = 0
    gm_of = {}
    for s in subGraphs:
        for n, a in s.nodes(data=True):
            gm_of[vi] = a["GNN_Measurement"]
            vi += 1
    for v in moved:
        gm = gm_of[int(v)]
        gm.x, gm.y, gm.z, gm.r = (float(c) for c in res["gnn"][v])
    extracted, pxy, pzr = [], [], []
    for s, cs in zip(subGraphs, cands):
        remove = []
        for c in cs:
            root = pos[(id(s), min(c.nodes, key=lambda n: pos[(id(s), n)]))]
            if res["status"][root] == ex.EXTRACTED:
                c.graph["iteration"] = str(iteration)
                extracted.append(c)
                pxy.append(res["pxy"][root])
                pzr.append(res["pzr"][root])
                remove.extend(c.nodes())
        s.remove_nodes_from(remove)
    remaining = [s for s in subGraphs if s.number_of_nodes() >= params.numhits]
    fragments = [s for s in subGraphs if 0 < s.number_of_nodes() < params.numhits]
    return extracted, pxy, pzr, remaining, fragments


def main():
    parser = argparse.ArgumentParser(description='extract track candidates')
    parser.add_argument('-i', '--input', help='input directory of outlier removal')
    parser.add_argument('-c', '--candidates', help='output directory to save track candidates')
    parser.add_argument('-r', '--remain', help='output directory to save remaining network')
    parser.add_argument('-f', '--fragments', help='output directory to save track fragments')
    parser.add_argument('-p', '--pval', help='chi-squared track candidate acceptance level')
    parser.add_argument('-s', '--separation_3d_threshold', help="3d distance cut between close proximity nodes")
    parser.add_argument('-t', '--threshold_distance_node_merging', help="threshold_distance_node_merging")
    parser.add_argument('-e', '--sigma0xy', help="sigma0 rms of track position measurements in xy plane")
    parser.add_argument('-z', '--sigma0rz', help="sigma0 rms of track position measurements in rz plane")
    parser.add_argument('-n', '--numhits', help="minimum number of hits for good track candidate")
    parser.add_argument('-a', '--iteration', help="iteration number of algorithm")
    parser.add_argument('-b', '--endcapboundary', help="endcap boundary z coordinate")
    a = parser.parse_args()
    params = ex.Params(float(a.pval), int(a.numhits), float(a.separation_3d_threshold),
                       float(a.threshold_distance_node_merging), float(a.sigma0xy), float(a.sigma0rz),
                       float(a.endcapboundary))
    subGraphs = read_numbered(a.input)
    extracted, pxy, pzr, remaining, fragments = extract(subGraphs, params, str(a.iteration))
    extracted = extracted + read_numbered(a.candidates)                      # :444-451
    pd.DataFrame({'pvals_xy': pxy, 'pvals_zr': pzr}).to_csv(a.candidates + 'pvals.csv')
    for i, sub in enumerate(extracted):
        _st.save_network(a.candidates, i, sub)
    for i, sub in enumerate(remaining):
        _st.save_network(a.remain, i, sub)
    for i, sub in enumerate(fragments):
        _st.save_network(a.fragments, i, sub)


if __name__ == "__main__":
    main()
