"""Drop-in for calculate_distance_between_updated_states/
calculate_distance_between_updated_track_states.py (same -i flag).

    python calculate_distance_between_updated_track_states.py -i IN/ [-o pairs.csv]

The reference script loads the subgraphs of -i (glob order, :113-120) and, for every
node with more than one active in-edge and an updated_track_states dict (:134-147),
was written to compute mahalanobis_distance (:27-104) for every pair of the node's
states (the pair loop :150-195 is commented out in the reference, which only prints the
dicts). Here the pair loop runs: gtf_updated_state_distances computes chi2, <tau>,
<theta>, delta theta and the truth flag of every pair on the GPU, and -o writes them as
CSV rows (subgraph, node, neighbour 1, neighbour 2, chi2, tau_average, theta_average,
delta_theta, truth).
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gtf import stages as _st  # noqa: E402


def pairwise_distances(subGraphs):
    """per subgraph {node: [(chi2, tau_average, theta_average, delta_theta, truth, nbr1, nbr2), ...]}"""
    return _st.updated_state_distances(subGraphs)


def main(argv=None):
    parser = argparse.ArgumentParser(description='track hit-pair simulator')
    parser.add_argument('-i', '--inputDir', help='input directory containing network gpickle file')
    parser.add_argument('-o', '--output', default=None, help='CSV of the pairwise distances (optional)')
    args = parser.parse_args(argv)
    subGraphs = _st.read_subgraphs(args.inputDir)
    tables = pairwise_distances(subGraphs)
    n_pairs = sum(len(r) for t in tables for r in t.values())
    print("%d subgraphs, %d nodes with pairs, %d pairs" % (len(subGraphs), sum(len(t) for t in tables), n_pairs))
    if args.output:
        with open(args.output, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["subgraph", "node", "neighbour1", "neighbour2", "chi2", "tau_average", "theta_average",
                        "delta_theta", "truth"])
            for si, t in enumerate(tables):
                for node, rows in t.items():
                    for chi2, tau, theta, dtheta, tr, n1, n2 in rows:
                        w.writerow([si, node, n1, n2, repr(chi2), repr(tau), repr(theta), repr(dtheta), tr])
    return tables


if __name__ == "__main__":
    main()
