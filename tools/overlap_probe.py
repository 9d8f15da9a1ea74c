"""Upper bound of overlapping two halves of the C4 pass on two streams (diagnostics): the
event split into two receiver wedges as a two-rank shard, both ranks' replicas in this
one process, each rank's pass on its own stream, K passes back to back; compared with
the one-stream full pass. No exchange (the halves would race on shared state without it
in a real overlapped pass; here each has its own replica), so this bounds the gain.
    python tools/overlap_probe.py [K]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd")]
import torch  # noqa: E402
from gtf import synth  # noqa: E402
from gtf.device import DeviceGraph  # noqa: E402
from gtf.params import Params  # noqa: E402
from gtf.shard import ShardedDeviceGraph  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 50
g = synth.workload("c4", seed=0)
p = Params()
res = {}
d = DeviceGraph(g, "cuda:0", layout="tiled")
snap = d.snapshot(DeviceGraph.PASS_INPUTS)
d.stage_inputs(K)
d.fill_inputs(snap)
for i in range(3):
    d.use_inputs(i); d.full_pass(p)
d.fill_inputs(snap)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for i in range(K):
    d.use_inputs(i)
    d.full_pass(p)
b.record()
torch.cuda.synchronize()
res["one_stream_full_pass_us"] = a.elapsed_time(b) / K * 1e3
del d
W = int(os.environ.get("GTF_PARTS", "2"))
streams = [torch.cuda.Stream() for _ in range(W)]
sds = []
for r in range(W):
    with torch.cuda.stream(streams[r]):
        sds.append(ShardedDeviceGraph(g, r, W, "cuda:0", backend="gloo"))
snaps = []
for r in range(W):
    with torch.cuda.stream(streams[r]):
        snaps.append(sds[r].d.snapshot(DeviceGraph.PASS_INPUTS))
        sds[r].d.stage_inputs(K)
        sds[r].d.fill_inputs(snaps[r])
        for i in range(3):   # warm-up; also fixes the shard's stream
            sds[r].d.use_inputs(i)
            sds[r].pass_(p)
torch.cuda.synchronize()


def timed(ranks):
    for r in ranks:
        with torch.cuda.stream(streams[r]):
            sds[r].d.fill_inputs(snaps[r])
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record(streams[0])
    for r in ranks:
        streams[r].wait_event(t0)
    for i in range(K):
        for r in ranks:
            with torch.cuda.stream(streams[r]):   # (a shard caches the stream current at its first pass)
                sds[r].d.use_inputs(i)
                sds[r].pass_(p)
    for r in ranks:
        if r != 0:
            e = torch.cuda.Event()
            e.record(streams[r])
            streams[0].wait_event(e)
    t1.record(streams[0])
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / K * 1e3


res["parts"] = W
res["part0_alone_us"] = timed([0])
res["all_parts_concurrent_us"] = timed(list(range(W)))
print(json.dumps(res))
