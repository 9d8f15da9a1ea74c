"""gtf.shard.SplitDeviceGraph: one event's pass on one GPU as two receiver wedges on two
HIP streams, the halo exchanged through device memory. After one and after two passes
the merged results equal the one-stream pass (DeviceGraph, the bench's tiled layout) bit
for bit -- activations, dict ranks and membership, merged states, every updated-state
field -- on the C4 event and on a small one; no device flag; staged inputs give the same
results as the resident arrays."""
import numpy as np
import pytest

from compare import compare
from gtf import synth
from gtf.device import DeviceGraph
from gtf.params import Params
from gtf.shard import SplitDeviceGraph

pytestmark = pytest.mark.gpu


def _single(g, passes):
    d = DeviceGraph(g, layout="tiled")
    d.clear_errors()
    outs = []
    for _ in range(passes):
        d.full_pass(Params())
        outs.append(d.download(g.copy()))
    assert d.errors() == 0
    return outs


@pytest.mark.parametrize("linear", [False, True])
@pytest.mark.parametrize("workload", ["c4", "tiny300"])
def test_split_pass_equals_one_stream_pass(workload, linear):
    """linear: the exchange joined into the first stream (SplitDeviceGraph.step(linear=True))"""
    g = synth.workload(workload, seed=0)
    ref = _single(g, 2)
    sp = SplitDeviceGraph(g)
    sp.clear_errors()
    for k in range(2):
        sp.step(Params(), linear=linear)
        got = sp.download(g.copy())
        errs = compare(got, ref[k], rtol=0.0, atol=0.0)
        assert errs == [], "pass %d: %s" % (k + 1, errs[:10])
    assert sp.errors() == 0


def test_split_staged_inputs_leave_the_resident_event():
    """the bench's timed path: passes on staged input copies, then a pass on the resident
    arrays equals the one-stream first pass (the staged passes touched only their copies)"""
    g = synth.workload("c4", seed=0)
    ref = _single(g, 1)[0]
    sp = SplitDeviceGraph(g)
    snap = sp.snapshot()
    sp.stage_inputs(3)
    sp.fill_inputs(snap)
    sp.clear_errors()
    for i in range(3):
        sp.use_inputs(i)
        sp.step(Params())
    sp.use_inputs(None)
    assert sp.errors() == 0
    sp.step(Params())
    errs = compare(sp.download(g.copy()), ref, rtol=0.0, atol=0.0)
    assert errs == [], errs[:10]
