"""Drop-in for src/trackml_mod/event_conversion.py (same CLI flags), the first stage of
run_gnn_trackml_mod.sh (:62):

    python trackml_mod/event_conversion.py -o OUT/ -n EVENT_NETWORK -t EVENT_TRUTH -a 7 -z 7 \\
        -e 0.3 -r 0.4 -m 0.6 -b 550

As the reference (:16-115): the truth mapping of the event is written from the TrackML
files (helper.load_save_truth, :51-53; here gtf.io.aggregate_truth, vectorised) and read
back; the graph is built from the event network's nodes / edges with every construct_graph
attribute (gtf.io.build_networkx), made a DiGraph and split into weakly connected
subgraphs; the track state estimates run on the GPU (gtf_track_state_estimates through
utilities.helper), then edge activation, priors, mixture weights and node degree; every
subgraph is saved as <i>_subgraph.gpickle in CCA order.

One opt-in deviation, for repositories that ship without the raw TrackML files (the
reference's own copy lacks event000001000-truth.csv and -hits.csv, .MISSING_LARGE_BLOBS):
with GTF_REUSE_TRUTH_MAPPING=1, when they are absent and the mapping file is present, the
mapping is read as it is (a note on stderr; its node set is checked against
nodes_to_hits.csv when that file exists) instead of failing on the missing files. By
default the CLI fails there like the reference. The reference's timing prints are not
produced.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gtf import io as _io  # noqa: E402
from utilities import helper as h  # noqa: E402


def main():
    parser = argparse.ArgumentParser(description='Convert trackml csv to GNN')
    parser.add_argument('-o', '--outputDir', help="Full directory path of where to save graph networks")
    parser.add_argument('-n', '--eventNetwork', help="Full directory path to event nodes, edges & nodes-to-hits")
    parser.add_argument('-t', '--eventTruth', help="Full directory path to event truth from TrackML")
    parser.add_argument('-a', '--min_volume', help="Minimum volume integer number in TrackML model to consider")
    parser.add_argument('-z', '--max_volume', help="Maximum volume integer number in TrackML model to consider")
    parser.add_argument('-e', '--sigma0xy', help="sigma0 rms of track position measurements in xy plane")
    parser.add_argument('-r', '--sigma0rz', help="sigma0 rms of track position measurements in rz plane")
    parser.add_argument('-m', '--sigma0rz2', help="sigma0 rms of track position measurements in rz plane - "
                                                  "orientation of barrel and endcap layer")
    parser.add_argument('-b', '--endcapboundary', help="endcap boundary z coordinate - orientation of barrel and "
                                                       "endcap layer")
    args = parser.parse_args()
    outputDir = args.outputDir
    min_volume, max_volume = int(args.min_volume), int(args.max_volume)
    sigma0xy, sigma0rz, sigma0rz2 = float(args.sigma0xy), float(args.sigma0rz), float(args.sigma0rz2)
    endcap_boundary = float(args.endcapboundary)

    # the reference's fixed file names (:41-44)
    event_network = args.eventNetwork + "/event_1_filtered_graph_"
    event_truth = args.eventTruth + "/event000001000-"
    event_truth_file = event_truth + "full-mapping-minCurv-0.3-800.csv"

    import pandas as pd
    raw = [event_truth + f for f in ("truth.csv", "particles.csv", "hits.csv")] + [event_network + "nodes_to_hits.csv"]
    missing = [f for f in raw if not os.path.isfile(f)]
    reuse = os.environ.get("GTF_REUSE_TRUTH_MAPPING", "0") == "1"
    if missing and reuse and os.path.isfile(event_truth_file):
        # opt-in only: the reference fails here (its load_save_truth reads the raw files)
        print("event_conversion: %s absent; reading the existing truth mapping %s (GTF_REUSE_TRUTH_MAPPING=1)"
              % (", ".join(os.path.basename(f) for f in missing), event_truth_file), file=sys.stderr)
        truth = pd.read_csv(event_truth_file)
        n2h = event_network + "nodes_to_hits.csv"
        if os.path.isfile(n2h):   # a mapping left from another event would give wrong truth silently
            want = set(pd.read_csv(n2h, usecols=["node_idx"])["node_idx"].tolist())
            if set(truth["node_idx"].tolist()) != want:
                raise SystemExit("event_conversion: %s does not map the nodes of %s" % (event_truth_file, n2h))
    else:
        _io.aggregate_truth(event_network, event_truth, event_truth_file)                # :51-53
        truth = pd.read_csv(event_truth_file)

    subGraphs = _io.build_networkx(event_network, min_volume, max_volume, truth=truth)    # :63-86
    subGraphs = h.compute_track_state_estimates(subGraphs, sigma0xy, sigma0rz, sigma0rz2, endcap_boundary)  # :94
    h.initialize_edge_activation(subGraphs)
    h.compute_prior_probabilities(subGraphs, 'track_state_estimates')
    h.compute_mixture_weights(subGraphs, 'track_state_estimates')
    for s in subGraphs:                                                                     # :100-103
        for node_num, _ in s.nodes(data=True):
            s.nodes[node_num]['degree'] = h.query_node_degree_in_edges(s, node_num)
    for i, sub in enumerate(subGraphs):                                                     # :113-114
        h.save_network(outputDir, i, sub)


if __name__ == "__main__":
    main()
