"""C4: the one-stream pass (DeviceGraph, tiled) against the two-stream split pass
(SplitDeviceGraph), K steps on staged inputs each, wall time between synchronizes as
bench.py measures it, alternating; prints JSON.
    python tools/split_time.py [K] [rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd")]
import torch  # noqa: E402
from gtf import synth  # noqa: E402
from gtf.device import DeviceGraph  # noqa: E402
from gtf.params import Params  # noqa: E402
from gtf.shard import SplitDeviceGraph  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
R = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g = synth.workload("c4", seed=0)
p = Params()
d = DeviceGraph(g, "cuda:0", layout="tiled")
dsnap = d.snapshot(DeviceGraph.PASS_INPUTS)
d.stage_inputs(K)
sp = SplitDeviceGraph(g, "cuda:0")
ssnap = sp.snapshot()
sp.stage_inputs(K)


def run_one():
    d.fill_inputs(dsnap)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        d.use_inputs(i)
        d.full_pass(p)
    torch.cuda.synchronize()
    d.use_inputs(None)
    return (time.perf_counter() - t0) / K


def run_split(exchange=True, join=True, linear=False):
    sp.fill_inputs(ssnap)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        sp.use_inputs(i)
        sp.step(p, exchange, join, linear)
    torch.cuda.synchronize()
    sp.use_inputs(None)
    return (time.perf_counter() - t0) / K


for f in (run_one, run_split):
    f()
out = {"one_stream_ms": [], "split_ms": [], "split_no_exchange_ms": [], "split_no_join_ms": [],
       "split_passes_only_ms": [], "split_linear_ms": []}
host = []
for _ in range(R):
    out["one_stream_ms"].append(run_one() * 1e3)
    out["split_ms"].append(run_split() * 1e3)
    out["split_no_exchange_ms"].append(run_split(False, True) * 1e3)
    out["split_no_join_ms"].append(run_split(True, False) * 1e3)
    out["split_passes_only_ms"].append(run_split(False, False) * 1e3)
    out["split_linear_ms"].append(run_split(linear=True) * 1e3)
# host time to enqueue one split step (no synchronize)
sp.fill_inputs(ssnap)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(K):
    sp.use_inputs(i)
    sp.step(p)
out["split_host_issue_ms"] = (time.perf_counter() - t0) / K * 1e3
torch.cuda.synchronize()
sp.use_inputs(None)
out["flags"] = [d.errors(), sp.errors()]
print(json.dumps(out))

# the split step captured as one hipGraph per staged input (cross-stream waits become graph
# edges), replayed back to back (GTF_SPLIT_GRAPH=1). Capture-safe by construction: every
# event is created before the capture (an event's first record creates it), the two part
# streams fork from the capture stream and join back into it, and nothing inside the
# capture synchronises or allocates; progress lines are flushed so a failure names its step.
if os.environ.get("GTF_SPLIT_GRAPH", "0") == "1":
    mode = os.environ.get("GTF_CAPTURE_MODE", "thread_local")
    graphs = []
    cap = torch.cuda.Stream()
    fork = [torch.cuda.Event() for _ in range(K)]
    joins = [[torch.cuda.Event() for _ in sp.streams] for _ in range(K)]
    for e in fork + [x for row in joins for x in row]:
        e.record(cap)                     # created here, outside any capture
    sp.fill_inputs(ssnap)
    torch.cuda.synchronize()
    print("capture: mode %s, %d graphs" % (mode, K), flush=True)
    for i in range(K):
        sp.use_inputs(i)
        gr = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(gr, stream=cap, capture_error_mode=mode):
                fork[i].record(cap)
                for s_ in sp.streams:
                    s_.wait_event(fork[i])
                # without the step's closing mutual stream waits (the eager path's guard against the
                # next step's pack overwriting a buffer the other stream still unpacks): the
                # capture's join below orders both streams, and the two mutual waits -- each stream
                # made to depend on the other's last node -- crashed hipStreamEndCapture (rc 139,
                # tools/capture_probe.py modes "exchange" vs "step", profiles/r04/capture/)
                sp.step(p, join=False, linear=os.environ.get("GTF_SPLIT_LINEAR", "0") == "1")
                for r_, s_ in enumerate(sp.streams):
                    joins[i][r_].record(s_)
                    cap.wait_event(joins[i][r_])
        except Exception as ex:
            print("capture %d failed: %r" % (i, ex), flush=True)
            raise
        print("captured %d" % i, flush=True)
        graphs.append(gr)
    sp.use_inputs(None)
    torch.cuda.synchronize()
    res = []
    for _ in range(R):
        sp.fill_inputs(ssnap)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for gr in graphs:
            gr.replay()
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) / K * 1e3)
    # the replayed passes against the one-stream pass: same outputs after K passes
    print(json.dumps({"split_graph_ms": res, "flags": sp.errors(), "capture_mode": mode,
                      "linear": os.environ.get("GTF_SPLIT_LINEAR", "0") == "1"}), flush=True)
