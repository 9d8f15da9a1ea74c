"""Golden fixtures for the drop-in event conversion (src/trackml_mod/event_conversion.py),
made by running the REFERENCE's own functions (run here, where /root/reference exists):

    python tests/golden/make_golden_event_conversion.py

* event_conversion_vol7.pkl -- the reference's event conversion of the committed
  volume-7 134 event (make_golden.build_network: load_nodes_edges, construct_graph with
  the committed full-mapping truth, nx.DiGraph, weakly connected subgraphs, TSE,
  activation, priors, mixture weights, degree): the first 120 subgraphs whole (every node
  and edge attribute) and, for all of them, the node lists in file order;
* event_conversion_vol7_truth.npz -- the truth-mapping rows of the vol-7 nodes (the
  columns of event000001000-full-mapping-minCurv-0.3-134.csv), which the test writes
  back as the CSV the CLI reads (the raw TrackML truth / hits files are absent);
* truth_aggregation.npz -- helper.load_save_truth (helper.py:548-582) on raw TrackML-format
  tables for the volume-7 nodes of the 800' event: nodes_to_hits and particles are the
  reference's committed files (rows of those nodes / their particles); truth.csv and
  hits.csv are absent upstream, so they are restated from the committed 800' mapping
  (one row per hit, which is what that mapping was joined from); the expected output is
  the mapping the reference's function writes from them.
"""
import os
import pickle
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as M  # noqa: E402

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

NET800 = os.path.join(M.REF, "src/trackml_mod/event_network/minCurv_0.3_800/event_1_filtered_graph_")
TRUTH800 = os.path.join(M.REF, "src/trackml_mod/event_truth/event000001000-")
N_WHOLE = 120


def event_conversion():
    with M._Quiet():
        subs = M.build_network()
    nodes = [np.asarray(list(s.nodes), np.int64) for s in subs]
    out = {"subs": subs[:N_WHOLE], "n_subgraphs": len(subs),
           "node_ptr": np.concatenate([[0], np.cumsum([n.size for n in nodes])]).astype(np.int64),
           "nodes": np.concatenate(nodes) if nodes else np.zeros(0, np.int64),
           "n_edges": np.asarray([s.number_of_edges() for s in subs], np.int64)}
    path = os.path.join(HERE, "event_conversion_vol7.pkl")
    with open(path, "wb") as f:
        pickle.dump(out, f, pickle.HIGHEST_PROTOCOL)
    print("wrote", path, "%.0f KB" % (os.path.getsize(path) / 1024), len(subs), "subgraphs")
    ids = set(out["nodes"].tolist())
    t = pd.read_csv(M.TRUTH134)
    t = t[t["node_idx"].isin(ids)]
    path = os.path.join(HERE, "event_conversion_vol7_truth.npz")
    np.savez_compressed(path, **{c: t[c].to_numpy() for c in t.columns})
    print("wrote", path, len(t), "truth rows")


def truth_aggregation():
    nodes = pd.read_csv(NET800 + "nodes.csv")
    keep = set(nodes.loc[nodes["layer_id"].between(7000, 8000), "node_idx"].astype(int))
    n2h = pd.read_csv(NET800 + "nodes_to_hits.csv")
    n2h = n2h[n2h["node_idx"].isin(keep)].reset_index(drop=True)
    mapping = pd.read_csv(TRUTH800 + "full-mapping-minCurv-0.3-800.csv")
    per_hit = mapping.drop_duplicates("hit_id")
    per_hit = per_hit[per_hit["hit_id"].isin(set(n2h["hit_id"]))]
    truth = per_hit[["hit_id", "particle_id"]].reset_index(drop=True)
    hits = per_hit[["hit_id", "volume_id", "layer_id", "module_id"]].reset_index(drop=True)
    parts = pd.read_csv(TRUTH800 + "particles.csv")
    parts = parts[parts["particle_id"].isin(set(truth["particle_id"]))].reset_index(drop=True)
    tmp = tempfile.mkdtemp()
    ev, tr = os.path.join(tmp, "event_1_filtered_graph_"), os.path.join(tmp, "event000001000-")
    n2h.to_csv(ev + "nodes_to_hits.csv", index=False)
    truth.to_csv(tr + "truth.csv", index=False)
    hits.to_csv(tr + "hits.csv", index=False)
    parts.to_csv(tr + "particles.csv", index=False)
    out_file = os.path.join(tmp, "mapping.csv")
    M.h.load_save_truth(ev, tr, out_file)          # the reference's function
    with open(out_file) as f:
        text = f.read()
    arrays = {"n2h_" + c: n2h[c].to_numpy() for c in n2h.columns}
    arrays.update({"truth_" + c: truth[c].to_numpy() for c in truth.columns})
    arrays.update({"hits_" + c: hits[c].to_numpy() for c in hits.columns})
    arrays.update({"particles_" + c: parts[c].to_numpy() for c in parts.columns})
    arrays["particles_columns"] = np.asarray(list(parts.columns))
    arrays["expected_csv"] = np.frombuffer(text.encode(), np.uint8)
    path = os.path.join(HERE, "truth_aggregation.npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, len(n2h), "node-hit rows", "%.0f KB" % (os.path.getsize(path) / 1024))


if __name__ == "__main__":
    truth_aggregation()
    event_conversion()
