"""Golden fixture for the physics metrics: the REFERENCE's own
src/extract/reconstruction_efficiency.py run on the candidates of the reference's own
three-iteration loop on the committed volume-7 event (minCurv_0.3_134).

Run here (the container that holds /root/reference), never on the GPU box:

    python tests/golden/make_golden_metrics.py    # writes tests/golden/metrics_vol7.npz

The script's inputs are laid out as run_gnn_trackml_mod.sh leaves them:
  * ROOTDIR/iteration_3/candidates/<i>_subgraph.gpickle -- the reference's candidate
    files. Two layouts are run: "script", what the run script really leaves there (its
    `cp -r iteration_{i-1}/candidates/ iteration_i/candidates/` copies the directory
    INTO the existing one, so the extraction's reload of earlier candidates,
    extract_track_candidates.py:477-484, finds none and only iteration 3's own
    extractions are counted), and "cumulative", the accumulation the extraction code
    intends (this iteration's candidates first, then the earlier files in their order).
  * EVENT_TRUTH/event000001000-particles.csv: the reference's committed file.
  * EVENT_TRUTH/event000001000-full-mapping-minCurv-0.3-800.csv: the script hard-codes
    this name (:58); the event's own mapping (minCurv-0.3-134) is placed under it.
  * EVENT_TRUTH/event000001000-truth.csv: absent from the reference (.MISSING_LARGE_BLOBS);
    its two columns the script reads (hit_id, particle_id) are the mapping's own, which
    event_conversion built from that truth file (helper.load_save_truth). Input data
    derived from the reference's data, not code.

Stored: the inputs the metric needs (volume-7 mapping rows, pT of the particles that
occur in them) and, per layout, the candidates' member lists in file and node order
and the script's outputs (purity CSVs, counts, printed efficiency).
"""
import contextlib
import io
import os
import re
import runpy
import shutil
import sys
import tempfile

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (binds nx.read/write_gpickle, imports the reference)
import make_golden_extract as mx  # noqa: E402

PARTICLES = os.path.join(mg.REF, "src/trackml_mod/event_truth/event000001000-particles.csv")
SCRIPT = os.path.join(mg.REF, "src/extract/reconstruction_efficiency.py")


def reference_iterations():
    """the reference's loop (make_golden_pipeline.py): candidate subgraphs per iteration"""
    with mg._Quiet():
        inp = mg.build_network()
    cands = []
    for it in (1, 2, 3):
        if it == 1:
            out = mg.run_cluster(inp, "track_state_estimates", 1.0, 2.0)
        elif it % 2 == 0:
            out = mg.run_extrapolate(inp)
        else:
            out = mg.run_cluster(inp, "updated_track_states", 1000.0, 100.0)
        mx.ARGS["a"] = it
        cand, rem, frag, pv = mx.run_reference(out)
        # the extraction CLI lists this iteration's candidates first (:471-484); with the
        # temp-dir harness its candidates dir starts empty, so `cand` is this iteration's
        if it % 2 == 0:
            rem = mg.run_update(rem)
        cands.append(cand)
        print("iteration %d: %d candidates" % (it, len(cand)))
        inp = rem
    return cands


def run_script(candidates, truth_dir):
    """reconstruction_efficiency.py -t truth_dir -o ROOT -a 7 -z 7 -i 3 on `candidates`"""
    with tempfile.TemporaryDirectory() as root:
        cdir = os.path.join(root, "iteration_3", "candidates") + "/"
        os.makedirs(cdir)
        for i, s in enumerate(candidates):
            mg.h.save_network(cdir, i, s)
        argv = sys.argv
        sys.argv = [SCRIPT, "-t", truth_dir, "-o", root, "-a", "7", "-z", "7", "-i", "3"]
        buf = io.StringIO()
        try:
            with contextlib.redirect_stdout(buf):
                runpy.run_path(SCRIPT, run_name="__main__")
        finally:
            sys.argv = argv
        text = buf.getvalue()
        tp = np.atleast_1d(np.loadtxt(os.path.join(root, "extracted_track_purities.csv"), delimiter=","))
        pp = np.atleast_1d(np.loadtxt(os.path.join(root, "extracted_particle_purities.csv"), delimiter=","))
    n_reco = int(re.search(r"Total num of reconstructed tracks: (\d+)", text).group(1))
    n_ref = int(re.search(r"Total num of reference tracks: (\d+)", text).group(1))
    eff = re.search(r"Track reconstruction efficiency:  ([0-9.]+) %", text).group(1)
    return tp, pp, n_reco, n_ref, eff


def _members(cands):
    ptr = np.zeros(len(cands) + 1, np.int64)
    ptr[1:] = np.cumsum([s.number_of_nodes() for s in cands])
    ids = np.array([int(n) for s in cands for n in s.nodes], np.int64)
    return ptr, ids


def main():
    mapping = pd.read_csv(mg.TRUTH134)
    cands = reference_iterations()
    layouts = {"script": cands[2], "cumulative": cands[2] + cands[1] + cands[0]}
    arrs = {}
    with tempfile.TemporaryDirectory() as tdir:
        pre = os.path.join(tdir, "event000001000-")
        shutil.copy(PARTICLES, pre + "particles.csv")
        shutil.copy(mg.TRUTH134, pre + "full-mapping-minCurv-0.3-800.csv")
        mapping[["hit_id", "particle_id"]].to_csv(pre + "truth.csv", index=False)
        for name, cl in layouts.items():
            tp, pp, n_reco, n_ref, eff = run_script(cl, tdir)
            ptr, ids = _members(cl)
            arrs[name + "__cand_ptr"], arrs[name + "__cand_ids"] = ptr, ids
            arrs[name + "__track_purity"], arrs[name + "__particle_purity"] = tp, pp
            arrs[name + "__counts"] = np.array([n_reco, n_ref], np.int64)
            arrs[name + "__efficiency"] = np.array(eff)
            print("%s: %d candidates -> %d reconstructed / %d reference tracks, efficiency %s %%"
                  % (name, len(cl), n_reco, n_ref, eff))
    m7 = mapping[mapping.volume_id == 7]
    for c in ("node_idx", "hit_id", "particle_id", "volume_id", "layer_id", "module_id"):
        arrs["map__" + c] = m7[c].to_numpy(np.int64)
    parts = pd.read_csv(PARTICLES)
    parts = parts[parts.particle_id.isin(m7.particle_id)]
    for c in ("particle_id", "px", "py"):
        arrs["particles__" + c] = parts[c].to_numpy()
    arrs["meta"] = np.array(repr(dict(src="reconstruction_efficiency.py -a 7 -z 7 -i 3 on the reference's "
                                          "iterations 1-3 of vol 7 of minCurv_0.3_134", pt_cut=1.0,
                                      num_distinct_layers=4)))
    path = os.path.join(HERE, "metrics_vol7.npz")
    np.savez_compressed(path, **arrs)
    print("wrote %s %.1f KB" % (path, os.path.getsize(path) / 1024))


if __name__ == "__main__":
    main()
