"""Build tests/golden/kat134/ from the reference's committed 134 event (run in the
survey container, where /root/reference exists; the outputs are committed data).

* event_1_filtered_graph_{nodes,edges}.csv: the reference's
  learn_KL_parabolic_model/src/output/track_sim_trackml_parabolic_model/minCurv_0.3_134/
  event_network files, trimmed to volume 7 (layer_id in [7000, 8000], the
  helper.load_nodes_edges window, helper.py:524-531) and to edges with both ends kept;
  header lines unchanged.
* truth_vol7.csv: node_idx -> truth_particle as helper.construct_graph derives it
  (helper.py:468-471, 493): the first distinct particle_id of the node's rows in
  event_truth/event000001000-full-mapping-minCurv-0.3-134.csv.
* 1_events_training_data.csv: the reference's KL training rows for that graph
  (event_graph_data/), copied unchanged.
"""
import os
import shutil
import sys

import numpy as np
import pandas as pd

REF = "/root/reference/learn_KL_parabolic_model/src/output/track_sim_trackml_parabolic_model/minCurv_0.3_134"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat134")


def main():
    os.makedirs(OUT, exist_ok=True)
    nodes = pd.read_csv(REF + "/event_network/event_1_filtered_graph_nodes.csv")
    keep = nodes["layer_id"].between(7000, 8000)
    kept = nodes[keep]
    with open(REF + "/event_network/event_1_filtered_graph_nodes.csv") as f, \
            open(OUT + "/event_1_filtered_graph_nodes.csv", "w") as g:   # rows verbatim
        g.write(f.readline())
        for line, k in zip(f, keep.to_numpy()):
            if k:
                g.write(line)
    ids = set(kept["node_idx"].astype(int))
    with open(REF + "/event_network/event_1_filtered_graph_edges.csv") as f, \
            open(OUT + "/event_1_filtered_graph_edges.csv", "w") as g:
        g.write(f.readline())
        g.write(f.readline())
        for line in f:
            a, b = line.split(",")[:2]
            if int(a) in ids and int(b) in ids:
                g.write(line)
    truth = pd.read_csv(REF + "/event_truth/event000001000-full-mapping-minCurv-0.3-134.csv")
    truth = truth[truth["node_idx"].isin(ids)]
    first = truth.groupby("node_idx", sort=True)["particle_id"].apply(lambda s: s.unique()[0])
    pd.DataFrame({"node_idx": first.index.astype(np.int64), "particle_id": first.values.astype(np.int64)}) \
        .to_csv(OUT + "/truth_vol7.csv", index=False)
    shutil.copy(REF + "/event_graph_data/1_events_training_data.csv", OUT + "/1_events_training_data.csv")
    print("wrote", OUT, len(kept), "nodes", len(first), "truth rows", file=sys.stderr)


if __name__ == "__main__":
    main()
