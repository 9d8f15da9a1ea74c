"""GPU box: device error flags of each of the 64 C3 events run alone (natural order) and
of the fused CSR (tiled), to localise a reference-exception flag in the batch."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "gnn-track-finding_amd")]
import numpy as np
from gtf import synth
from gtf.graph import concat
from gtf.params import Params
from gtf.device import DeviceGraph

p = Params()
evs = [synth.event(s, synth.C2_TRACKS, synth.C2_FAKE) for s in range(64)]
for i, ev in enumerate(evs):
    for lay in ("natural", "tiled"):
        d = DeviceGraph(ev, layout=lay)
        d.clear_errors(); d.full_pass(p)
        f = d.errors()
        if f:
            print("event", i, lay, "flags", f, flush=True)
f = concat(evs)
for lay in ("natural", "tiled"):
    d = DeviceGraph(f, layout=lay)
    d.clear_errors(); d.full_pass(p)
    print("fused", lay, "flags", d.errors(), flush=True)
