"""Golden fixture for the whole track-finding loop (run_gnn_trackml_mod.sh:61-146,
START=1 END=3) on the committed volume-7 event, from the REFERENCE's own stages.

Run here (the container that holds /root/reference), never on the GPU box:

    python tests/golden/make_golden_pipeline.py    # writes tests/golden/pipeline_vol7.npz

iteration 1: clustering on track_state_estimates (-c 1.0 -k 2.0) -> extraction
iteration 2: extrapolation (-c 2.0) -> extraction -> remove_state_metadata on the remaining
iteration 3: clustering on updated_track_states (-c 1000 -k 100) -> extraction
Each next iteration starts from the previous remaining subgraphs (run script :140).
Stores, per iteration, the extracted candidates (node-id sets and p-values), the
remaining and the fragment subgraphs (node-id sets). The reference renumbers files in
glob() order, so sets (not orders) are what the fixture pins.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402
import make_golden_extract as mx  # noqa: E402


def _flat(groups):
    ptr = np.zeros(len(groups) + 1, np.int64)
    ptr[1:] = np.cumsum([len(g) for g in groups])
    ids = np.concatenate([np.asarray(sorted(int(x) for x in g), np.int64) for g in groups]) if groups else \
        np.zeros(0, np.int64)
    return ptr, ids


def main():
    with mg._Quiet():
        inp = mg.build_network()
    arrs = {}
    for it in (1, 2, 3):
        if it == 1:
            out = mg.run_cluster(inp, "track_state_estimates", 1.0, 2.0)
        elif it % 2 == 0:
            out = mg.run_extrapolate(inp)
        else:
            out = mg.run_cluster(inp, "updated_track_states", 1000.0, 100.0)
        mx.ARGS["a"] = it
        cand, rem, frag, pv = mx.run_reference(out)
        if it % 2 == 0:
            rem = mg.run_update(rem)
        for name, groups in (("cand", [s.nodes for s in cand]), ("rem", [s.nodes for s in rem]),
                             ("frag", [s.nodes for s in frag])):
            ptr, ids = _flat(groups)
            arrs["it%d__%s_ptr" % (it, name)] = ptr
            arrs["it%d__%s_ids" % (it, name)] = ids
        arrs["it%d__pval_xy" % it] = pv["pvals_xy"].to_numpy()
        arrs["it%d__pval_zr" % it] = pv["pvals_zr"].to_numpy()
        print("iteration %d: %d candidates, %d remaining, %d fragments" % (it, len(cand), len(rem), len(frag)))
        inp = rem
    arrs["meta"] = np.array(repr(dict(src="run_gnn_trackml_mod.sh iterations 1-3 on vol 7 of minCurv_0.3_134",
                                      **mg.P, p=mx.ARGS["p"], n=mx.ARGS["n"], s=mx.ARGS["s"], t=mx.ARGS["t"])))
    path = os.path.join(HERE, "pipeline_vol7.npz")
    np.savez_compressed(path, **arrs)
    print("wrote %s %.1f KB" % (path, os.path.getsize(path) / 1024))


if __name__ == "__main__":
    main()
