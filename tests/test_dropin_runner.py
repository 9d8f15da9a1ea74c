"""gtf.dropin.run_dir, the drop-in CLIs' directory runner (gpickle in -> stage -> gpickle out
with the pickle work on forked worker processes), on the CPU: the worker machinery --
chunking in glob order, pack per worker, concatenation, the split of the results back to
the workers, unpack, the file numbering -- carries the CPU checker's stage (the oracle,
in place of the device) to the reference's own stage outputs (tests/golden/dropin_*.pkl),
for several worker counts including more workers than files."""
import os
import pickle

import pytest

import gtf_oracle as O
from gtf.dropin import run_dir
from gtf.params import Params
from test_dropin import _load, _read, _write, graphs_equal


def _oracle_extrapolate(p):
    def stage(g):
        O.extrapolate_stage(g, p)
        return 0
    return stage


@pytest.mark.parametrize("workers", [1, 3, 200])
def test_run_dir_extrapolate_matches_reference(tmp_path, workers):
    d = _load("extrapolate")
    ind, outd = str(tmp_path / "in") + "/", str(tmp_path / "out") + "/"
    _write(d["in"], ind)
    os.makedirs(outd)
    p = Params(**{k: d["args"][k] for k in ("sigma0xy", "sigma0rz", "sigma0rz2", "endcap_boundary", "chi2_cut")})
    info = run_dir(ind, outd, None, workers=workers, host_stage=_oracle_extrapolate(p))
    assert info["files"] == info["written"] == len(d["in"])
    assert sorted(os.listdir(outd)) == sorted("%d_subgraph.gpickle" % i for i in range(len(d["in"])))
    errs = graphs_equal(_read(outd), d["out"])
    assert errs == [], "\n".join(errs[:20])


def test_run_dir_update_in_place(tmp_path):
    """remove_state_metadata writes back into its input directory: every file is read
    before any is written"""
    d = _load("update")
    rem = str(tmp_path / "rem") + "/"
    _write(d["in"], rem)

    def stage(g):
        O.update_stage(g, Params())
        return 0
    run_dir(rem, rem, None, workers=4, host_stage=stage)
    errs = graphs_equal(_read(rem), d["out"])
    assert errs == [], "\n".join(errs[:20])


def test_run_dir_reference_exception_writes_nothing(tmp_path):
    """a reference exception flagged by the stage raises the reference's class and no
    output file is written (the reference's stage loses its output too)"""
    d = _load("extrapolate")
    ind, outd = str(tmp_path / "in") + "/", str(tmp_path / "out") + "/"
    _write(d["in"], ind)
    os.makedirs(outd)
    with pytest.raises(ValueError):
        run_dir(ind, outd, None, workers=3, host_stage=lambda g: 8)    # GTF_ERR_TIE_EMPTIED
    assert os.listdir(outd) == []


def test_run_dir_empty_directory(tmp_path):
    ind = str(tmp_path / "in") + "/"
    os.makedirs(ind)
    info = run_dir(ind, ind, None, workers=4, host_stage=lambda g: 0)
    assert info["files"] == info["written"] == 0


def test_pool_survives_a_bad_file_and_is_reused(tmp_path):
    """the worker pool is forked once and reused by later directories; a file a worker
    cannot read raises in the caller, the pool is dropped, and the next directory runs on a
    fresh pool with the same results"""
    from gtf import dropin
    d = _load("extrapolate")
    p = Params(**{k: d["args"][k] for k in ("sigma0xy", "sigma0rz", "sigma0rz2", "endcap_boundary", "chi2_cut")})
    good, bad = str(tmp_path / "good") + "/", str(tmp_path / "bad") + "/"
    _write(d["in"], good)
    _write(d["in"][:5], bad)
    with open(bad + "2_subgraph.gpickle", "wb") as fh:
        fh.write(b"not a pickle")
    outs = [str(tmp_path / ("out%d" % i)) + "/" for i in range(3)]
    for o in outs:
        os.makedirs(o)
    run_dir(good, outs[0], None, workers=3, host_stage=_oracle_extrapolate(p))
    pool = dropin._POOL
    assert pool is not None and pool.alive()
    run_dir(good, outs[1], None, workers=3, host_stage=_oracle_extrapolate(p))
    assert dropin._POOL is pool                      # reused, not re-forked
    with pytest.raises(RuntimeError, match="drop-in worker"):
        run_dir(bad, outs[2], None, workers=3, host_stage=_oracle_extrapolate(p))
    assert dropin._POOL is None                      # dropped after the failure
    run_dir(good, outs[2], None, workers=3, host_stage=_oracle_extrapolate(p))
    for o in outs:
        assert graphs_equal(_read(o), d["out"]) == []
    dropin._drop_pool()
