"""Build tests/golden/kat800/ from the reference's committed minCurv_0.3_800 event (run in
the survey container, where /root/reference exists; the outputs are committed data).

Source: learn_KL_parabolic_model/src/output/track_sim_trackml_parabolic_model/minCurv_0.3_800/
(SURVEY §8a "C2": the 800' all-volume event, 29,590 nodes / 89,028 directed edges).

* event_1_filtered_graph_{nodes,edges}.csv: the event_network files, copied unchanged
  (every volume: the all-volume fixtures of make_golden_800.py read them whole);
* truth.csv: node_idx -> truth_particle as helper.construct_graph derives it
  (helper.py:468-471, 493): the first distinct particle_id of the node's rows in
  event_truth/event000001000-full-mapping-minCurv-0.3-800.csv;
* 3_events_training_data.csv: the reference's KL training rows (event_graph_data/, KAT-2,
  SURVEY §8c), copied unchanged. Only event 1's graph is committed; its volume-7 rows
  (1,055 pairs) are the ones a test can recompute.
"""
import os
import shutil
import sys

import numpy as np
import pandas as pd

REF = "/root/reference/learn_KL_parabolic_model/src/output/track_sim_trackml_parabolic_model/minCurv_0.3_800"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat800")


def main():
    os.makedirs(OUT, exist_ok=True)
    for f in ("event_1_filtered_graph_nodes.csv", "event_1_filtered_graph_edges.csv"):
        shutil.copy(os.path.join(REF, "event_network", f), os.path.join(OUT, f))
    truth = pd.read_csv(REF + "/event_truth/event000001000-full-mapping-minCurv-0.3-800.csv")
    first = truth.groupby("node_idx", sort=True)["particle_id"].apply(lambda s: s.unique()[0])
    pd.DataFrame({"node_idx": first.index.astype(np.int64), "particle_id": first.values.astype(np.int64)}) \
        .to_csv(OUT + "/truth.csv", index=False)
    shutil.copy(REF + "/event_graph_data/3_events_training_data.csv", OUT + "/3_events_training_data.csv")
    print("wrote", OUT, len(first), "truth rows", file=sys.stderr)


if __name__ == "__main__":
    main()
