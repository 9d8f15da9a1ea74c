"""Golden fixture for candidate extraction (§8f next #1), from the REFERENCE.

Run here (the container that holds /root/reference), never on the GPU box:

    python tests/golden/make_golden_extract.py    # writes tests/golden/extract_it1.npz

Builds the volume-7 network (make_golden.build_network), runs the reference's
iteration-1 clustering (-c 1.0 -k 2.0) and then the reference's
src/extract/extract_track_candidates.py main() exactly as run_gnn_trackml_mod.sh:131
calls it (-p 0.01 -n 4 -s 10 -t 8.0 -a 1 -e 0.3 -z 0.4 -b 550), through its own
gpickle directories. Stores the packed stage input, each node's (volume_id,
in_volume_layer_id), and the outputs: extracted candidates (node ids, p-values, in
output order), remaining and fragment subgraphs (node ids), and the GNN_Measurement
coordinates the stage mutates in place (close-proximity merging).
"""
import glob
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (reference import + shims)
import pandas as pd  # noqa: E402

from extract import extract_track_candidates as ref_ex  # noqa: E402  (reference)

ARGS = dict(p=0.01, n=4, s=10.0, t=8.0, a=1)


def _flat(groups):
    ptr = np.zeros(len(groups) + 1, np.int64)
    ptr[1:] = np.cumsum([len(g) for g in groups])
    ids = np.concatenate([np.asarray(sorted(int(x) for x in g), np.int64) for g in groups]) if groups else \
        np.zeros(0, np.int64)
    return ptr, ids


def run_reference(subs):
    """extract_track_candidates.main through its own directories -> (cand, rem, frag, pvals)"""
    with tempfile.TemporaryDirectory() as d:
        dirs = {k: os.path.join(d, k) + "/" for k in ("in", "cand", "rem", "frag")}
        for v in dirs.values():
            os.makedirs(v)
        for i, s in enumerate(subs):
            mg.h.save_network(dirs["in"], i, s)
        sys.argv = ["extract_track_candidates.py", "-i", dirs["in"], "-c", dirs["cand"], "-r", dirs["rem"],
                    "-f", dirs["frag"], "-p", str(ARGS["p"]), "-n", str(ARGS["n"]), "-s", str(ARGS["s"]),
                    "-t", str(ARGS["t"]), "-a", str(ARGS["a"]), "-e", str(mg.P["sigma0xy"]),
                    "-z", str(mg.P["sigma0rz"]), "-b", str(mg.P["endcap_boundary"])]
        with mg._Quiet():
            ref_ex.main()

        def read(dd):
            out, i = [], 0
            while os.path.isfile(dd + "%d_subgraph.gpickle" % i):
                out.append(mg._read_gpickle(dd + "%d_subgraph.gpickle" % i))
                i += 1
            return out
        return read(dirs["cand"]), read(dirs["rem"]), read(dirs["frag"]), pd.read_csv(dirs["cand"] + "pvals.csv")


def dropin_fixture(it1, n_sub=150):
    """reference gpickle objects for the drop-in CLI test: the first n_sub subgraphs of
    the stage input and the reference's outputs on them"""
    import copy
    import pickle
    subs = copy.deepcopy(it1[:n_sub])
    inp = copy.deepcopy(subs)
    cand, rem, frag, pv = run_reference(subs)
    path = os.path.join(HERE, "dropin_extract.pkl")
    with open(path, "wb") as f:
        pickle.dump({"input": inp, "candidates": cand, "remaining": rem, "fragments": frag,
                     "pvals": pv[["pvals_xy", "pvals_zr"]].to_numpy(), "args": ARGS, "P": mg.P}, f,
                    pickle.HIGHEST_PROTOCOL)
    print("wrote dropin_extract.pkl %.1f KB: %d candidates" % (os.path.getsize(path) / 1024, len(cand)))


def main():
    with mg._Quiet():
        net = mg.build_network()
    it1 = mg.run_cluster(net, "track_state_estimates", 1.0, 2.0)
    dropin_fixture(it1)
    g = mg.pack(it1)
    vivl = np.array([[float(a["vivl_id"][0]), float(a["vivl_id"][1])] for s in it1 for _, a in s.nodes(data=True)])
    gnn_before = g.node["gnn"].copy()
    with tempfile.TemporaryDirectory() as d:
        dirs = {k: os.path.join(d, k) + "/" for k in ("in", "cand", "rem", "frag")}
        for v in dirs.values():
            os.makedirs(v)
        for i, s in enumerate(it1):
            mg.h.save_network(dirs["in"], i, s)
        sys.argv = ["extract_track_candidates.py", "-i", dirs["in"], "-c", dirs["cand"], "-r", dirs["rem"],
                    "-f", dirs["frag"], "-p", str(ARGS["p"]), "-n", str(ARGS["n"]), "-s", str(ARGS["s"]),
                    "-t", str(ARGS["t"]), "-a", str(ARGS["a"]), "-e", str(mg.P["sigma0xy"]),
                    "-z", str(mg.P["sigma0rz"]), "-b", str(mg.P["endcap_boundary"])]
        with mg._Quiet():
            ref_ex.main()

        def read(dd):
            out, i = [], 0
            while os.path.isfile(dd + "%d_subgraph.gpickle" % i):
                out.append(mg._read_gpickle(dd + "%d_subgraph.gpickle" % i))
                i += 1
            return out
        cand, rem, frag = read(dirs["cand"]), read(dirs["rem"]), read(dirs["frag"])
        pv = pd.read_csv(dirs["cand"] + "pvals.csv")
    row = {int(n): i for i, n in enumerate(g.node["node_id"])}
    gnn_after = gnn_before.copy()
    for s in cand + rem + frag:
        for n, a in s.nodes(data=True):
            gm = a["GNN_Measurement"]
            gnn_after[row[int(n)]] = (gm.x, gm.y, gm.z, gm.r)
    arrs = {"in__" + k: v for k, v in mg.pick(g, mg.IN_FIELDS).items()}
    cptr, cids = _flat([s.nodes for s in cand])
    rptr, rids = _flat([s.nodes for s in rem])
    fptr, fids = _flat([s.nodes for s in frag])
    arrs.update({"x__vivl": vivl, "x__cand_ptr": cptr, "x__cand_ids": cids,
                 "x__cand_pval_xy": pv["pvals_xy"].to_numpy(), "x__cand_pval_zr": pv["pvals_zr"].to_numpy(),
                 "x__cand_edges": np.array([s.number_of_edges() for s in cand]),
                 "x__rem_ptr": rptr, "x__rem_ids": rids, "x__frag_ptr": fptr, "x__frag_ids": fids,
                 "x__gnn_after": gnn_after})
    arrs["meta"] = np.array(repr(dict(src="extract_track_candidates.main on iteration-1 clustering (vol 7, 134)",
                                      **mg.P, **ARGS)))
    path = os.path.join(HERE, "extract_it1.npz")
    np.savez_compressed(path, **arrs)
    moved = int((np.abs(gnn_after - gnn_before).sum(1) > 0).sum())
    print("wrote extract_it1.npz %.1f KB: %d candidates, %d remaining, %d fragments, %d GNN_M moved" % (
        os.path.getsize(path) / 1024, len(cand), len(rem), len(frag), moved))


if __name__ == "__main__":
    main()
