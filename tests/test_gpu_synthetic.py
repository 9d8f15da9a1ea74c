"""HIP pass vs the oracle on seeded synthetic TrackML-shaped events.

Synthetic "full load" events (every node extrapolates its first neighbour's
parabola) contain numerically ill-conditioned states (near-singular 2x2 blocks,
Joseph-form cancellation). There the reference's own value depends on the
rounding of the implementation, so the bar is: masks exact except decisions that
flip when the oracle's inputs are perturbed by ~1 ulp, and floats within 1e-6
relative plus 100x the oracle's own ulp-perturbation noise (compare.py). The
counts of such entries are printed. The golden-fixture tests
(test_gpu_parity.py) hold the strict 1e-6 bar on the reference's real data.
"""
import numpy as np
import pytest

import gtf_oracle as O
from compare import compare_noise, noise_envelope
from gtf import synth
from gtf.params import Params

pytestmark = pytest.mark.gpu


def _gpu_pass(g, p):
    from gtf.device import DeviceGraph
    d = DeviceGraph(g)
    d.clear_errors()
    d.full_pass(p)
    flags = d.errors()
    return d.download(g.copy()), flags


@pytest.mark.parametrize("seed,tracks", [(0, 300), (1, 1200), (2, 3300)])
def test_pass_matches_oracle(seed, tracks):
    g = synth.event(seed=seed, n_tracks=tracks, fake_mean=synth.C4_FAKE)
    p = Params()

    def run(x):
        O.full_pass(x, p, tie_policy="stop")
        return x

    ref, noise, flips = noise_envelope(run, g)
    got, flags = _gpu_pass(g, p)
    errs, stats = compare_noise(got, ref, noise, flips)
    print("seed %d: %d edges, %s, device flags %d" % (seed, g.n_edges, stats, flags))
    assert errs == [], "\n".join(errs)
    assert stats["mask_undetermined"] <= 0.001 * g.n_edges
    assert flags == 0, flags
