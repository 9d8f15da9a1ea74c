"""Drop-in for src/extract/reconstruction_efficiency.py (same flags -t -o -a -z -i):
track reconstruction efficiency and purities of the extracted candidates (gtf.metrics).

    python reconstruction_efficiency.py -t EVENT_TRUTH -o ROOTDIR -a 7 -z 7 -i 3

Reads ROOTDIR/iteration_<i>/candidates/ in either form:
  * the reference's numbered gpickles (<n>_subgraph.gpickle), using each node's
    hit_dissociation as stored (:102-110, :125-131);
  * run_pipeline.py's candidates.npz (gtf.store), with hit_dissociation rebuilt from
    the mapping as event conversion builds it (helper.py:466-479).
EVENT_TRUTH/event000001000-{particles.csv, full-mapping-<--mapping>.csv} are read as the
script reads them; truth.csv (hit -> particle) when present, else the mapping's own
hit_id / particle_id columns (the mapping is built from it). --cumulative counts the
candidates of iterations i, i-1, ..., 1 (the accumulation extract_track_candidates.py
intends); without it, as the run script leaves the directory, iteration i's only (its
`cp -r` nests the earlier ones one level down). Writes extracted_track_purities.csv and
extracted_particle_purities.csv into ROOTDIR (:186-187) and prints the summary (:212-218).
"""
import argparse
import os
import pickle
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

from gtf import metrics, store  # noqa: E402

SUFFIX = "_subgraph.gpickle"


def read_candidates(cdir):
    """-> (ptr, node ids, particle lists or None) of one candidates directory"""
    npz = os.path.join(cdir, "candidates.npz")
    if os.path.isfile(npz):
        groups, _ = store.load_groups(npz)
        ptr = np.zeros(len(groups) + 1, np.int64)
        ptr[1:] = np.cumsum([len(g) for g in groups])
        ids = np.concatenate(groups) if groups else np.zeros(0, np.int64)
        return ptr, ids, None
    subs, i = [], 0
    while os.path.isfile(os.path.join(cdir, str(i) + SUFFIX)):
        with open(os.path.join(cdir, str(i) + SUFFIX), "rb") as f:
            subs.append(pickle.load(f))
        i += 1
    ptr = np.zeros(len(subs) + 1, np.int64)
    ptr[1:] = np.cumsum([s.number_of_nodes() for s in subs])
    ids = np.array([int(n) for s in subs for n in s.nodes], np.int64)
    lists = [[p for d in s.nodes(data=True) for p in list(d[1]["hit_dissociation"].values())[1]] for s in subs]
    return ptr, ids, lists


def score(event_truth, root, min_volume, max_volume, iterations, mapping="full-mapping-minCurv-0.3-800.csv",
          cumulative=False, verbose=False):
    """-> gtf.metrics.Result for the candidates under ROOT/iteration_<iterations>
    (and, cumulative, every earlier iteration's)"""
    pre = os.path.join(event_truth, "event000001000-")
    particles = pd.read_csv(pre + "particles.csv")
    m = metrics.HitMapping.from_frame(pd.read_csv(pre + mapping))
    th = tp = None
    if os.path.isfile(pre + "truth.csv"):
        truth = pd.read_csv(pre + "truth.csv", usecols=["hit_id", "particle_id"])
        th, tp = truth.hit_id.to_numpy(np.int64), truth.particle_id.to_numpy(np.int64)
    its = range(iterations, 0, -1) if cumulative else [iterations]
    ptrs, idss, lists = [np.zeros(1, np.int64)], [], []
    gp = True
    for it in its:
        ptr, ids, ls = read_candidates(os.path.join(root, "iteration_%d" % it, "candidates"))
        ptrs.append(ptr[1:] + ptrs[-1][-1])
        idss.append(ids)
        gp = gp and ls is not None
        lists.extend(ls or [])
    ptr = np.concatenate(ptrs)
    ids = np.concatenate(idss) if idss else np.zeros(0, np.int64)
    if verbose:
        print("number of track candidates to process:", len(ptr) - 1)
    return metrics.reconstruction_efficiency(ptr, ids, m, particles.particle_id.to_numpy(), particles.px.to_numpy(),
                                             particles.py.to_numpy(), min_volume, max_volume, th, tp,
                                             node_lists=lists if gp and len(ptr) > 1 else None)


def main(argv=None):
    ap = argparse.ArgumentParser(description="track reconstruction efficiency")
    ap.add_argument("-t", "--eventTruth", required=True, help="directory holding the event's truth files")
    ap.add_argument("-o", "--output", required=True, help="ROOTDIR of the run")
    ap.add_argument("-a", "--min_volume", type=int, required=True)
    ap.add_argument("-z", "--max_volume", type=int, required=True)
    ap.add_argument("-i", "--iterations", type=int, required=True)
    ap.add_argument("--mapping", default="full-mapping-minCurv-0.3-800.csv",
                    help="mapping file name under EVENT_TRUTH (the script's hard-coded default)")
    ap.add_argument("--cumulative", action="store_true", help="count the candidates of every iteration")
    args = ap.parse_args(argv)
    r = score(args.eventTruth, args.output, args.min_volume, args.max_volume, args.iterations, args.mapping,
              args.cumulative, verbose=True)
    np.savetxt(os.path.join(args.output, "extracted_track_purities.csv"), r.track_purities, delimiter=",")
    np.savetxt(os.path.join(args.output, "extracted_particle_purities.csv"), r.particle_purities, delimiter=",")
    print("\n-------------------------------------------------------")
    print("Total num of reconstructed tracks:", r.n_reconstructed)
    print("Total num of reference tracks:", r.n_reference)
    print("Track reconstruction efficiency: ", r.efficiency_str, "%")
    print("-------------------------------------------------------")
    return 0


if __name__ == "__main__":
    sys.exit(main())
