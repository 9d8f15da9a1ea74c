"""HIP pass vs the oracle on seeded synthetic TrackML-shaped events.

Synthetic "full load" events (every node extrapolates its first neighbour's
parabola) contain numerically ill-conditioned states (near-singular 2x2 blocks,
Joseph-form cancellation). There the reference's own value depends on the
rounding of the implementation, so the comparison tolerates: masks that flip when
the oracle's inputs are perturbed by ~1 ulp, and floats within 1e-6 relative plus
100x the oracle's own ulp-perturbation noise (compare.py). With the generator's edges
kept within the reference event's azimuth gap (gtf/synth.py) none of that is needed
for the masks: they must match exactly (0 undetermined decisions, checked), and at most
a couple of floats per ~1M may sit inside the noise envelope instead of 1e-6 (measured:
1 of 940,794 on seed 2). The golden-fixture tests (test_gpu_parity.py) hold the strict
1e-6 bar on the reference's real data.
"""
import numpy as np
import pytest

import gtf_oracle as O
from compare import compare_noise, noise_envelope
from gtf import synth
from gtf.params import Params

pytestmark = pytest.mark.gpu


def _gpu_pass(g, p, layout="natural"):
    from gtf.device import DeviceGraph
    d = DeviceGraph(g, layout=layout)
    d.clear_errors()
    d.full_pass(p)
    flags = d.errors()
    return d.download(g.copy()), flags


@pytest.mark.parametrize("seed,tracks,layout", [(0, 300, "natural"), (1, 1200, "natural"), (2, 3300, "natural"),
                                                (2, 3300, "tiled")])
def test_pass_matches_oracle(seed, tracks, layout):
    g = synth.event(seed=seed, n_tracks=tracks, fake_mean=synth.C4_FAKE)
    p = Params()

    def run(x):
        O.full_pass(x, p, tie_policy="stop")
        return x

    ref, noise, flips = noise_envelope(run, g)
    got, flags = _gpu_pass(g, p, layout)
    errs, stats = compare_noise(got, ref, noise, flips)
    print("seed %d (%s): %d edges, %s, device flags %d" % (seed, layout, g.n_edges, stats, flags))
    assert errs == [], "\n".join(errs)
    assert stats["mask_undetermined"] == 0 and stats["mask_ill_differs"] == 0 and stats["ill_nodes"] == 0, stats
    assert stats["float_ill"] <= 2e-6 * stats["float_checked"] + 1, stats
    assert flags == 0, flags
