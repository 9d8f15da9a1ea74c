"""Physics metrics: reconstruction efficiency and purities.

Pinned by tests/golden/metrics_vol7.npz -- the reference's own
reconstruction_efficiency.py on the reference's own candidates of its three-iteration
run of the volume-7 event (make_golden_metrics.py), in two directory layouts:
"script" (what run_gnn_trackml_mod.sh really leaves in iteration_3/candidates: its
`cp -r` nests the earlier iterations' files one level down, so only iteration 3's 2
candidates are counted -> 0.613 %) and "cumulative" (iterations 3, 2, 1, as the
extraction code intends -> 81.595 %). Bars: counts and the printed efficiency exact,
purity arrays exact and in order (same float divisions).

The GPU test runs the device pipeline end to end (gtf.pipeline) and scores its
candidates: the physics parity of the GPU pipeline against the reference's CPU one."""
import os
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

import metrics_oracle as MO
from fixtures import GOLDEN
from gtf import metrics, store

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PREFIX = os.path.join(GOLDEN, "kat134", "event_1_filtered_graph_")
LAYOUTS = ("script", "cumulative")
PER_ITERATION = (1055, 110, 2)     # the reference run's candidates of iterations 1, 2, 3


def _z():
    return np.load(os.path.join(GOLDEN, "metrics_vol7.npz"), allow_pickle=False)


def _mapping(z):
    return metrics.HitMapping(*(z["map__" + c] for c in ("node_idx", "hit_id", "particle_id", "volume_id",
                                                          "layer_id", "module_id")))


def _frames(z):
    hits = pd.DataFrame({c: z["map__" + c] for c in ("node_idx", "hit_id", "particle_id", "volume_id", "layer_id",
                                                      "module_id")})
    parts = pd.DataFrame({c: z["particles__" + c] for c in ("particle_id", "px", "py")})
    return hits, parts


def _cands(z, layout):
    ptr, ids = z[layout + "__cand_ptr"], z[layout + "__cand_ids"]
    return ptr, ids


def _expect(z, layout):
    n_reco, n_ref = (int(x) for x in z[layout + "__counts"])
    return n_reco, n_ref, z[layout + "__track_purity"], z[layout + "__particle_purity"], str(z[layout + "__efficiency"])


def test_fixture_values():
    z = _z()
    assert _expect(z, "script")[:2] == (1, 163) and str(z["script__efficiency"]) == "0.613"
    assert _expect(z, "cumulative")[:2] == (133, 163) and str(z["cumulative__efficiency"]) == "81.595"
    assert len(z["cumulative__cand_ptr"]) - 1 == sum(PER_ITERATION)


@pytest.mark.parametrize("layout", LAYOUTS)
def test_oracle_matches_reference_script(layout):
    z = _z()
    hits, parts = _frames(z)
    ref, pixel = MO.reference_tracks(parts, hits[["hit_id", "particle_id"]], hits, 7, 7)
    diss = MO.hit_dissociation(hits)
    ptr, ids = _cands(z, layout)
    cands = [ids[ptr[i]:ptr[i + 1]] for i in range(len(ptr) - 1)]
    n_reco, n_ref, tp, pp, eff = MO.efficiency(cands, diss, ref, pixel)
    e = _expect(z, layout)
    assert (n_reco, n_ref, eff) == (e[0], e[1], e[4])
    assert np.array_equal(tp, e[2]) and np.array_equal(pp, e[3])


@pytest.mark.parametrize("layout", LAYOUTS)
def test_metrics_match_reference_script(layout):
    z = _z()
    ptr, ids = _cands(z, layout)
    r = metrics.reconstruction_efficiency(ptr, ids, _mapping(z), z["particles__particle_id"], z["particles__px"],
                                          z["particles__py"], 7, 7)
    e = _expect(z, layout)
    assert (r.n_reconstructed, r.n_reference, r.efficiency_str) == (e[0], e[1], e[4])
    assert np.array_equal(r.track_purities, e[2]) and np.array_equal(r.particle_purities, e[3])
    assert int(r.matched.sum()) == e[0]


def _truth_dir(z, d):
    os.makedirs(d, exist_ok=True)
    hits, parts = _frames(z)
    parts.to_csv(os.path.join(d, "event000001000-particles.csv"), index=False)
    hits.to_csv(os.path.join(d, "event000001000-full-mapping-minCurv-0.3-134.csv"), index=False)
    return d


def _read_csv(path):
    return np.atleast_1d(np.loadtxt(path, delimiter=","))


@pytest.mark.parametrize("layout", LAYOUTS)
def test_cli_on_pipeline_layout(tmp_path, layout):
    """the drop-in CLI on run_pipeline.py's directory layout (candidates.npz per iteration)"""
    z = _z()
    tdir = _truth_dir(z, str(tmp_path / "truth"))
    ptr, ids = _cands(z, "cumulative")
    groups = [ids[ptr[i]:ptr[i + 1]] for i in range(len(ptr) - 1)]
    cut = np.cumsum([0, PER_ITERATION[2], PER_ITERATION[1], PER_ITERATION[0]])
    for it, (a, b) in zip((3, 2, 1), zip(cut[:-1], cut[1:])):
        cdir = tmp_path / "run" / ("iteration_%d" % it) / "candidates"
        os.makedirs(cdir)
        store.save_groups(str(cdir / "candidates.npz"), groups[a:b])
    cli = os.path.join(ROOT, "gnn-track-finding_amd", "extract", "reconstruction_efficiency.py")
    args = [sys.executable, cli, "-t", tdir, "-o", str(tmp_path / "run"), "-a", "7", "-z", "7", "-i", "3",
            "--mapping", "full-mapping-minCurv-0.3-134.csv"] + (["--cumulative"] if layout == "cumulative" else [])
    out = subprocess.run(args, check=True, capture_output=True, text=True).stdout
    e = _expect(z, layout)
    assert "Track reconstruction efficiency:  %s %%" % e[4] in out
    assert np.array_equal(_read_csv(str(tmp_path / "run" / "extracted_track_purities.csv")), e[2])
    assert np.array_equal(_read_csv(str(tmp_path / "run" / "extracted_particle_purities.csv")), e[3])


def _toy():
    # nodes 0..5; hits 10..17; particles 1 (4 layers), 2 (4 layers), 3 (2 layers)
    rows = [  # node, hit, particle, volume, layer, module
        (0, 10, 1, 7, 2, 1), (1, 11, 1, 7, 4, 1), (2, 12, 1, 7, 6, 1), (3, 13, 1, 7, 8, 1),
        (0, 14, 2, 7, 2, 2), (1, 15, 2, 7, 4, 2), (4, 16, 2, 7, 6, 2), (5, 17, 2, 7, 8, 2),
    ]
    a = np.array(rows, np.int64).T
    m = metrics.HitMapping(*a)
    pid = np.array([1, 2, 3])
    return m, pid, np.array([2.0, 2.0, 2.0]), np.zeros(3)


def test_ties_go_to_the_first_seen_particle():
    """Counter + max(key=get): equal counts resolve to the id seen first (:133)"""
    m, pid, px, py = _toy()
    # candidate [4, 5, 2, 3]: particle ids [2, 2, 1, 1] -> particle 2 first
    r = metrics.reconstruction_efficiency(np.array([0, 4]), np.array([4, 5, 2, 3]), m, pid, px, py, 7, 7)
    assert r.reconstructed_pid[0] == 2 and r.n_good[0] == 2
    r = metrics.reconstruction_efficiency(np.array([0, 4]), np.array([2, 3, 4, 5]), m, pid, px, py, 7, 7)
    assert r.reconstructed_pid[0] == 1


def test_each_particle_counted_once_and_empty_input():
    m, pid, px, py = _toy()
    ptr, ids = np.array([0, 4, 8]), np.array([0, 1, 2, 3, 0, 1, 2, 3])
    r = metrics.reconstruction_efficiency(ptr, ids, m, pid, px, py, 7, 7)
    assert r.n_reconstructed == 1 and list(r.matched) == [True, False]
    assert r.n_reference == 2 and r.efficiency_str == "50.000"
    r = metrics.reconstruction_efficiency(np.array([0]), np.zeros(0, np.int64), m, pid, px, py, 7, 7)
    assert r.n_reconstructed == 0 and r.track_purities.size == 0
    # low pT: no reference tracks -> the script divides by zero too
    with pytest.raises(ZeroDivisionError):
        metrics.reconstruction_efficiency(ptr, ids, m, pid, np.zeros(3), py, 7, 7).efficiency


@pytest.mark.gpu
def test_gpu_pipeline_physics_parity():
    """the device pipeline's candidates score exactly as the reference's own run"""
    from gtf import pipeline
    z = _z()
    g, vivl = pipeline.build_event(PREFIX, 7, 7)
    its = pipeline.run(g, vivl, iterations=3)
    assert [len(i.candidates) for i in its] == list(PER_ITERATION)
    m = _mapping(z)
    for layout, lists in (("script", its[2].candidates),
                          ("cumulative", its[2].candidates + its[1].candidates + its[0].candidates)):
        ptr = np.concatenate([[0], np.cumsum([len(c) for c in lists])])
        r = metrics.reconstruction_efficiency(ptr, np.concatenate(lists), m, z["particles__particle_id"],
                                              z["particles__px"], z["particles__py"], 7, 7)
        e = _expect(z, layout)
        assert (r.n_reconstructed, r.n_reference, r.efficiency_str) == (e[0], e[1], e[4]), layout
        # candidate order within an iteration follows glob() in the reference: compare as multisets
        assert np.array_equal(np.sort(r.track_purities), np.sort(e[2]))
        assert np.array_equal(np.sort(r.particle_purities), np.sort(e[3]))


def test_cli_on_reference_gpickles(tmp_path):
    """the drop-in CLI on the reference's own candidate gpickles (the extraction drop-in
    fixture: the reference's candidates of 150 iteration-1 subgraphs), reading each
    node's stored hit_dissociation; scored like the oracle scores the same lists"""
    import pickle
    with open(os.path.join(GOLDEN, "dropin_extract.pkl"), "rb") as f:
        cands = pickle.load(f)["candidates"]
    assert len(cands) > 10
    cdir = tmp_path / "run" / "iteration_1" / "candidates"
    os.makedirs(cdir)
    for i, s in enumerate(cands):
        with open(str(cdir / ("%d_subgraph.gpickle" % i)), "wb") as f:
            pickle.dump(s, f, pickle.HIGHEST_PROTOCOL)
    z = _z()
    tdir = _truth_dir(z, str(tmp_path / "truth"))
    cli = os.path.join(ROOT, "gnn-track-finding_amd", "extract", "reconstruction_efficiency.py")
    out = subprocess.run([sys.executable, cli, "-t", tdir, "-o", str(tmp_path / "run"), "-a", "7", "-z", "7", "-i",
                          "1", "--mapping", "full-mapping-minCurv-0.3-134.csv"],
                         check=True, capture_output=True, text=True).stdout
    hits, parts = _frames(z)
    ref, pixel = MO.reference_tracks(parts, hits[["hit_id", "particle_id"]], hits, 7, 7)
    diss = {int(n): list(d["hit_dissociation"].values())[1] for s in cands for n, d in s.nodes(data=True)}
    n_reco, n_ref, tp, pp, eff = MO.efficiency([list(s.nodes) for s in cands], diss, ref, pixel)
    assert n_reco > 0
    assert "Total num of reconstructed tracks: %d" % n_reco in out and "efficiency:  %s %%" % eff in out
    assert np.array_equal(_read_csv(str(tmp_path / "run" / "extracted_track_purities.csv")), tp)
    assert np.array_equal(_read_csv(str(tmp_path / "run" / "extracted_particle_purities.csv")), pp)


@pytest.mark.gpu
def test_gpu_run_pipeline_scores_its_run(tmp_path):
    """run_pipeline.py --truth: the run script's last step (reconstruction_efficiency.py)
    on the device pipeline's own output directories -> metrics.json"""
    import json
    z = _z()
    tdir = _truth_dir(z, str(tmp_path / "truth"))
    cli = os.path.join(ROOT, "gnn-track-finding_amd", "run_pipeline.py")
    out = str(tmp_path / "out")
    subprocess.check_call([sys.executable, cli, "-n", os.path.join(GOLDEN, "kat134"), "-o", out, "-a", "7", "-z", "7",
                           "--truth", tdir, "--mapping", "full-mapping-minCurv-0.3-134.csv"])
    with open(os.path.join(out, "metrics.json")) as f:
        got = json.load(f)
    for name, layout in (("last_iteration", "script"), ("cumulative", "cumulative")):
        e = _expect(z, layout)
        assert (got[name]["reconstructed"], got[name]["reference"], got[name]["efficiency_pct"]) == (e[0], e[1], e[4])
