"""Which step of the two-stream split pass breaks hipGraph capture?

    python -X faulthandler tools/capture_probe.py MODE

MODE (each a superset of the previous):
  one      DeviceGraph.full_pass captured on one stream (the single-stream pass)
  shard    one part's gtf_pass_shard on its own stream, captured there
  halo     + that part's gtf_halo_pack / gtf_halo_unpack on the same stream
  fork     both parts' passes on their two streams, forked from and joined into the capture stream
  exchange SplitDeviceGraph.step without its closing mutual stream waits (join=False): the
           capture's own join orders the two streams
  step     SplitDeviceGraph.step (passes, cross-stream halo exchange, mutual joins) as round 3 captured it
  torchx   no libgtf: two streams of torch element-wise kernels with the same mid-capture cross
           waits (each stream waits on the other's event, then launches) -- a runtime repro
  linear   the exchange joined into one stream instead (stream 0 waits on stream 1's pack, both
           unpacks on stream 0, stream 1 forked back): one kernel node with two dependencies
  linstep  SplitDeviceGraph.step(linear=True) with its join (stream 1 waits for stream 0's
           unpacks): the capture-safe form of the split step
Each mode captures, instantiates (capture_end), replays once and checks the outputs against
the same calls run directly. Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gtf import synth  # noqa: E402
from gtf.device import DeviceGraph  # noqa: E402
from gtf.params import Params  # noqa: E402
from gtf.shard import SplitDeviceGraph  # noqa: E402

mode = sys.argv[1]
if mode == "torchx":
    sa, sb, cap = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.zeros(1 << 20, device="cuda")
    y = torch.zeros(1 << 20, device="cuda")
    ev = [torch.cuda.Event() for _ in range(5)]
    for e in ev:
        e.record(cap)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=cap, capture_error_mode="thread_local"):
        ev[0].record(cap)
        sa.wait_event(ev[0])
        sb.wait_event(ev[0])
        with torch.cuda.stream(sa):
            x.add_(1.0)
        with torch.cuda.stream(sb):
            y.add_(2.0)
        ev[1].record(sa)
        ev[2].record(sb)
        sa.wait_event(ev[2])
        sb.wait_event(ev[1])
        with torch.cuda.stream(sa):
            x.add_(y)
        with torch.cuda.stream(sb):
            y.add_(x)
        ev[3].record(sa)
        ev[4].record(sb)
        cap.wait_event(ev[3])
        cap.wait_event(ev[4])
    print(json.dumps({"mode": mode, "step": "captured"}), flush=True)
    gr.replay()
    torch.cuda.synchronize()
    print(json.dumps({"mode": mode, "step": "replayed", "x0": float(x[0]), "y0": float(y[0])}), flush=True)
    sys.exit(0)
g = synth.workload("c2", seed=1)
p = Params()
cap = torch.cuda.Stream()


def say(**kw):
    print(json.dumps(dict(mode=mode, **kw)), flush=True)


if mode == "one":
    d = DeviceGraph(g, "cuda:0", layout="tiled")
    snap = d.snapshot(DeviceGraph.PASS_INPUTS)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=cap, capture_error_mode="thread_local"):
        d.full_pass(p)   # d.stream is the current stream: cap
    say(step="captured")
    d.restore(snap)
    gr.replay()
    torch.cuda.synchronize()
    a = d.download(g.copy())
    d.restore(snap)
    d.full_pass(p)
    b = d.download(g.copy())
    same = all(np.array_equal(a.slot[k], b.slot[k], equal_nan=a.slot[k].dtype.kind == "f") for k in ("act", "uts_sv"))
    say(step="replayed", same=bool(same))
    sys.exit(0)

sp = SplitDeviceGraph(g, "cuda:0")
a, b = sp.parts
sa, sb = sp.streams
torch.cuda.synchronize()
fork = torch.cuda.Event()
joins = [torch.cuda.Event(), torch.cuda.Event()]
for e in [fork] + joins:
    e.record(cap)
torch.cuda.synchronize()
gr = torch.cuda.CUDAGraph()
if mode in ("shard", "halo"):
    with torch.cuda.graph(gr, stream=sa, capture_error_mode="thread_local"):
        a.pass_(p)
        if mode == "halo":
            a.halo_pack()
            a.halo_unpack(ctypes.c_void_p(b.send_buf.data_ptr()))
    say(step="captured")
elif mode == "linear":
    packed = torch.cuda.Event()
    packed.record(sb)
    torch.cuda.synchronize()
    with torch.cuda.graph(gr, stream=cap, capture_error_mode="thread_local"):
        fork.record(cap)
        sa.wait_event(fork)
        sb.wait_event(fork)
        a.pass_(p)
        a.halo_pack()
        b.pass_(p)
        b.halo_pack()
        packed.record(sb)
        sa.wait_event(packed)          # stream 1 joined into stream 0
        a.halo_unpack(ctypes.c_void_p(b.send_buf.data_ptr()))
        b.halo_unpack(ctypes.c_void_p(a.send_buf.data_ptr()), stream=sa)
        joins[0].record(sa)
        cap.wait_event(joins[0])
    say(step="captured")
elif mode in ("fork", "exchange", "step", "linstep"):
    with torch.cuda.graph(gr, stream=cap, capture_error_mode="thread_local"):
        fork.record(cap)
        sa.wait_event(fork)
        sb.wait_event(fork)
        if mode == "fork":
            a.pass_(p)
            b.pass_(p)
        elif mode == "linstep":
            sp.step(p, join=True, linear=True)
        else:
            sp.step(p, join=(mode == "step"))
        joins[0].record(sa)
        joins[1].record(sb)
        cap.wait_event(joins[0])
        cap.wait_event(joins[1])
    say(step="captured")
else:
    raise SystemExit("unknown mode")
gr.replay()
torch.cuda.synchronize()
say(step="replayed", flags=sp.errors())
