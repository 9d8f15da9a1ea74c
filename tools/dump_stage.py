"""GPU box: save the device state of a C2 event after its extrapolation + update stages
(the clustering input) as gpurun_out/stage_<seed>.npz, to study a clustering flag on CPU."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "gnn-track-finding_amd")]
from gtf import synth
from gtf.params import Params
from gtf.device import DeviceGraph
from gtf.store import save_graph

seed = int(sys.argv[1])
p = Params()
ev = synth.event(seed, synth.C2_TRACKS, synth.C2_FAKE)
d = DeviceGraph(ev)
d.clear_errors()
d.extrapolate(p)
d.update(p)
print("flags after extrapolate+update", d.errors())
save_graph("gpurun_out/stage_%d.npz" % seed, d.download(ev.copy()), compressed=True)
d.cluster("uts", p.cluster_chi2, p.cluster_kl, p)
print("flags after cluster", d.errors())
