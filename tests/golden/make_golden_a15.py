"""Golden pairs of SURVEY §8 a15 from the REFERENCE's own function.

    python tests/golden/make_golden_a15.py      # writes tests/golden/a15_pairs.npz

calculate_distance_between_updated_states/calculate_distance_between_updated_track_states.py
is a script (argparse and a gpickle loop at module level, :108-146), so it cannot be
imported. Its function ``mahalanobis_distance`` (:27-104) is taken out of the file with
``ast`` and executed on its own, in a namespace holding what the file's own imports bind
(numpy as np, ``from math import *``). The file itself is read here and never copied.

Inputs: the updated_track_states of two committed golden networks (volume 7 of
minCurv_0.3_134): ``extrapolate_full`` (the reference's full-load extrapolation) and
``pass_full`` (the fused pass chain). The pair loop follows the script's commented loop
(:134-195): nodes with more than one active in-edge (:139-140) and an
``updated_track_states`` dict (:143), every pair i > j of the dict's entries in dict order
(:174-176), means = the entries' state vectors, covariances = their (aliased) joint
covariances, coordinates = the node's and the neighbours' node attribute ``xyzr``
(:162-163, :182-183), and the truth flag of :190-193 (truth = the committed hit mapping).
"""
import ast
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_FILE = ("/root/reference/calculate_distance_between_updated_states/"
            "calculate_distance_between_updated_track_states.py")
sys.path[:0] = [os.path.join(REPO, "gnn-track-finding_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402

OUT = os.path.join(HERE, "a15_pairs.npz")
FIXTURES = ("extrapolate_full", "pass_full")


def reference_function():
    """the reference's mahalanobis_distance, compiled from its own source"""
    with open(REF_FILE) as f:
        tree = ast.parse(f.read(), REF_FILE)
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "mahalanobis_distance"]
    assert len(fn) == 1
    mod = ast.Module(body=fn, type_ignores=[])
    ns = {"np": np}
    ns.update({k: getattr(math, k) for k in dir(math) if not k.startswith("_")})   # from math import *
    exec(compile(mod, REF_FILE, "exec"), ns)
    return ns["mahalanobis_distance"]


def pair_table(g, truth, fn):
    """per-node pair rows in the script's loop order; returns (pair_ptr, rows)"""
    from gtf.graph import mat_from_cov5
    S = g.slot
    sp = g.slot_ptr
    ptr = [0]
    rows = []
    for v in range(g.n_nodes):
        lo, hi = sp[v], sp[v + 1]
        nact = int(np.sum((S["is_edge"][lo:hi] == 1) & (S["act"][lo:hi] == 1)))
        keys = [k for k in range(lo, hi) if S["uts_rank"][k] >= 0]
        keys.sort(key=lambda k: S["uts_rank"][k])
        if g.node["has_uts"][v] != 1 or nact <= 1:
            ptr.append(ptr[-1])
            continue
        node_coords = g.node["xyzr"][v]
        for i in range(len(keys)):
            for j in range(i):
                ki, kj = keys[i], keys[j]
                mi = np.array([S["uts_sv"][ki][0], S["uts_sv"][ki][1], S["uts_tau"][ki]])
                mj = np.array([S["uts_sv"][kj][0], S["uts_sv"][kj][1], S["uts_tau"][kj]])
                ci, cj = mat_from_cov5(S["uts_cov"][ki]), mat_from_cov5(S["uts_cov"][kj])
                ui, uj = S["slot_src"][ki], S["slot_src"][kj]
                chi2, tau, theta, dtheta = fn(mi, ci, mj, cj, node_coords, g.node["xyzr"][ui], g.node["xyzr"][uj])
                tr = int(truth[v] == truth[ui] and truth[ui] == truth[uj] and truth[v] == truth[uj])
                rows.append((chi2, tau, theta, dtheta, tr))
        ptr.append(len(rows))
    return np.array(ptr, np.int64), np.array(rows, dtype=np.float64).reshape(-1, 5)


def main():
    from fixtures import load, expected_graph
    from gtf import io
    fn = reference_function()
    out = {}
    for name in FIXTURES:
        g, o, _, _ = load(name)
        e = expected_graph(g, o)
        truth = io.read_truth(os.path.join(HERE, "kat134", "truth_vol7.csv"), e.node["node_id"])
        ptr, rows = pair_table(e, truth, fn)
        out[name + "__pair_ptr"] = ptr
        out[name + "__chi2"] = rows[:, 0]
        out[name + "__avg_tau"] = rows[:, 1]
        out[name + "__avg_theta"] = rows[:, 2]
        out[name + "__delta_theta"] = rows[:, 3]
        out[name + "__truth"] = rows[:, 4].astype(np.int8)
        out[name + "__node_truth"] = truth
        print("%s: %d nodes with pairs, %d pairs, %d truth pairs" % (
            name, int(np.sum(np.diff(ptr) > 0)), rows.shape[0], int(rows[:, 4].sum())))
    np.savez_compressed(OUT, **out)
    print("wrote %s (%.1f kB)" % (OUT, os.path.getsize(OUT) / 1e3))


if __name__ == "__main__":
    main()
