"""oracle/cpu_ref.cpp (the C++ fp64 restatement of the fused pass with OpenMP, bench.py's
all-cores CPU baseline) against the reference's own fixtures and the full-size C4 digest.

Same bar as the HIP path: masks, dict positions, flags and degree exact; floats within
1e-6 relative (C4: plus 100x the oracle's perturbation noise at the digest's samples).
"""
import os

import numpy as np
import pytest

from compare import compare
from fixtures import GOLDEN, load, expected_graph
from gtf import synth, toymc
from gtf.params import Params

cpu_ref = pytest.importorskip("cpu_ref")
if not os.path.exists(cpu_ref.LIB):
    pytest.skip("oracle/build/libcpuref.so not built (make -C oracle)", allow_module_level=True)


def _params(meta):
    return Params(sigma0xy=meta["sigma0xy"], sigma0rz=meta["sigma0rz"], sigma0rz2=meta["sigma0rz2"],
                  endcap_boundary=meta["endcap_boundary"], chi2_cut=meta.get("chi2_cut", 2.0),
                  cluster_chi2=meta.get("chi2", 1000.0), cluster_kl=meta.get("kl", 100.0))


@pytest.mark.parametrize("threads", [1, 4])
def test_pass_full_fixture(threads):
    g, out, _, meta = load("pass_full")
    exp = expected_graph(g, out)
    assert cpu_ref.full_pass(g, _params(meta), threads) == 0
    errs = compare(g, exp, rtol=1e-6)
    assert errs == [], "\n".join(errs)


def test_c4_digest():
    from test_gpu_c4_digest import digest_errors
    z = np.load(os.path.join(GOLDEN, "c4_digest.npz"), allow_pickle=False)
    g = synth.workload("c4", seed=0)
    assert cpu_ref.full_pass(g, Params(), 0) == 0
    errs, diff_und = digest_errors(g, z)
    assert errs == [], "\n".join(errs)


def test_c1_equals_oracle():
    from test_toymc import cpu_c1
    start, ref, _ = cpu_c1()
    g = start.copy()
    assert cpu_ref.full_pass(g, Params(), 2) == 0
    errs = compare(g, ref, rtol=1e-9)
    assert errs == [], "\n".join(errs)


@pytest.mark.parametrize("name,key", [("cluster_tse", "tse"), ("cluster_uts", "uts"), ("cluster_tie", "tse")])
def test_clustering_fixtures_bit_exact(name, key):
    """clustering on the reference's own states: numpy's BLAS rounding restated, so every
    output equals the reference's bit for bit (rtol 0), ties included"""
    g, out, _, meta = load(name)
    exp = expected_graph(g, out)
    assert cpu_ref.cluster(g, key, meta["chi2"], meta["kl"], _params(meta), 2) == 0
    errs = compare(g, exp, rtol=0.0, atol=0.0)
    assert errs == [], "\n".join(errs)
