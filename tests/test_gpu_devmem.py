"""DeviceGraph(mem="hip"): the stage path on libgtf's own allocations (gtf.devmem,
gtf_malloc / gtf_memcpy_* of include/gtf.h) instead of torch tensors -- the drop-in CLIs'
path, since a CLI process never imports torch (gtf.dropin.device_memory).

- in this (torch) process both allocators on the same event give the same arrays bit for
  bit after extrapolate, update and cluster (the kernels are the same; only where the
  bytes live differs);
- the extrapolation and clustering CLIs run in fresh processes end to end without ever
  importing torch and write the reference's own outputs (tests/golden/dropin_*.pkl)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from gtf import synth
from gtf.device import DeviceGraph, MUTABLE_NODE, STATIC_SLOT
from gtf.graph import SLOT_FIELDS
from gtf.params import Params
from test_dropin import PKG, _load, _read, _write, graphs_equal

pytestmark = pytest.mark.gpu


def _run(mem, g, p):
    d = DeviceGraph(g, mem=mem)
    d.clear_errors()
    d.extrapolate(p)
    d.update(p)
    d.cluster("uts", p.cluster_chi2, p.cluster_kl, p)
    flags = d.errors()
    d.download(g)
    return flags


@pytest.mark.parametrize("seed", [0, 1])
def test_hip_memory_equals_torch_memory(seed):
    import copy
    p = Params()
    base = synth.workload("tiny400", seed=seed)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    fa = _run("torch", a, p)
    fb = _run("hip", b, p)
    assert fa == fb
    for f in MUTABLE_NODE:
        assert np.array_equal(a.node[f], b.node[f], equal_nan=a.node[f].dtype.kind == "f"), f
    for f in SLOT_FIELDS:
        if f in STATIC_SLOT or f == "slot_key":
            continue
        assert np.array_equal(a.slot[f], b.slot[f], equal_nan=a.slot[f].dtype.kind == "f"), f


def test_hip_memory_refuses_torch_only_methods():
    d = DeviceGraph(synth.workload("tiny50"), mem="hip")
    with pytest.raises(NotImplementedError, match="mem='torch'"):
        d.snapshot()


# runs a drop-in CLI in this fresh interpreter and fails if torch got imported
_NO_TORCH = r"""
import runpy, sys
sys.argv = sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
assert "torch" not in sys.modules, "the drop-in CLI imported torch"
from gtf import _native
assert _native._lean, "libgtf was not loaded lean"
"""


def _cli_no_torch(module, args, cwd):
    env = dict(os.environ)
    env["PYTHONPATH"] = PKG + os.pathsep + env.get("PYTHONPATH", "")
    env.pop("GTF_DROPIN_MEM", None)
    r = subprocess.run([sys.executable, "-c", _NO_TORCH, os.path.join(PKG, module)] + args, cwd=cwd, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]


def test_extrapolate_cli_without_torch(tmp_path):
    d = _load("extrapolate")
    _write(d["in"], str(tmp_path / "in"))
    os.makedirs(tmp_path / "out")
    _cli_no_torch("extrapolate/extrapolate_merged_states.py",
                  ["-i", str(tmp_path / "in") + "/", "-o", str(tmp_path / "out") + "/", "-c", "2.0", "-e", "0.3",
                   "-z", "0.4", "-m", "0.6", "-b", "550.0"], str(tmp_path))
    errs = graphs_equal(_read(str(tmp_path / "out")), d["out"])
    assert errs == [], "\n".join(errs[:20])


def test_clustering_cli_without_torch(tmp_path):
    d = _load("cluster_tse")
    _write(d["in"], str(tmp_path / "in"))
    os.makedirs(tmp_path / "out")
    _cli_no_torch("clustering/clustering.py",
                  ["-i", str(tmp_path / "in") + "/", "-o", str(tmp_path / "out") + "/", "-d", "track_state_estimates",
                   "-c", "1.0", "-k", "2.0", "-l", "x.lut", "-t", "1", "-z", "0.4", "-m", "0.6", "-b", "550.0"],
                  str(tmp_path))
    errs = graphs_equal(_read(str(tmp_path / "out")), d["out"])
    assert errs == [], "\n".join(errs[:20])


def test_extract_cli_without_torch(tmp_path):
    """the extraction CLI (GPU CCA + fits) in a torch-free process: the reference's
    candidate, remaining and fragment files (counts and node lists; test_dropin.py checks
    every attribute of the same run on the default path)"""
    import pickle
    d = _load("extract")
    a = d["args"]
    dirs = {k: str(tmp_path / k) + "/" for k in ("in", "cand", "rem", "frag")}
    for v in dirs.values():
        os.makedirs(v)
    for i, s in enumerate(d["input"]):
        with open(dirs["in"] + "%d_subgraph.gpickle" % i, "wb") as f:
            pickle.dump(s, f, pickle.HIGHEST_PROTOCOL)
    _cli_no_torch("extract/extract_track_candidates.py",
                  ["-i", dirs["in"], "-c", dirs["cand"], "-r", dirs["rem"], "-f", dirs["frag"], "-p", str(a["p"]),
                   "-n", str(a["n"]), "-s", str(a["s"]), "-t", str(a["t"]), "-a", str(a["a"]),
                   "-e", str(d["P"]["sigma0xy"]), "-z", str(d["P"]["sigma0rz"]), "-b", str(d["P"]["endcap_boundary"])],
                  str(tmp_path))
    for key, dd in (("candidates", "cand"), ("remaining", "rem"), ("fragments", "frag")):
        got = _read_numbered(dirs[dd])
        assert len(got) == len(d[key]), key
        for gs, es in zip(got, d[key]):
            assert list(gs.nodes) == list(es.nodes), key


def _read_numbered(dd):
    import pickle
    out, i = [], 0
    while os.path.isfile(dd + "%d_subgraph.gpickle" % i):
        with open(dd + "%d_subgraph.gpickle" % i, "rb") as f:
            out.append(pickle.load(f))
        i += 1
    return out


def test_tag_propagation_hip_memory_equals_torch():
    """tag propagation (k_tag_prepare + sweeps until the reference's stop test) on both
    allocators: same final tags, same flips per sweep"""
    g = synth.workload("tiny400", seed=3)
    rng = np.random.default_rng(0)
    tags = rng.integers(0, g.n_nodes, g.n_nodes)
    radius = g.node["xyzr"][:, 3]
    a = DeviceGraph(g, mem="torch").tag_propagation(tags, radius)
    b = DeviceGraph(g, mem="hip").tag_propagation(tags, radius)
    assert np.array_equal(a[0], b[0]) and a[1] == b[1] and len(a[1]) >= 1
