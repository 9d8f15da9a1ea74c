"""Directory-to-directory stage runner for the drop-in CLIs: gpickle in -> GPU -> gpickle out,
with the per-file host work spread over worker processes.

The reference's stages (extrapolate_merged_states.py:521-572, clustering.py:380-415,
remove_state_metadata.py:11-57) read every ``*_subgraph.gpickle`` of a directory in glob
order, mutate the graphs and save them renumbered 0..n-1 in that order
(helper.save_network, helper.py:585-587). Reading and writing those pickles -- networkx
graphs whose state dicts hold small numpy arrays, ~10 us per array to pickle -- costs
far more host time than the stage itself on the GPU (SURVEY §7 "End-to-end vs kernel
time"). Here the files are split into contiguous chunks, one per worker process:

  worker w: unpickle its files -> pack them (gtf.graph.pack) -> send the packed arrays
  main:     concatenate the chunks (gtf.graph.concat) -> one device stage call ->
            send each worker the mutable arrays of its node / slot range (device
            arrays from libgtf's own allocator, gtf.devmem, unless the process already
            holds torch: device_memory())
  worker w: write them back into its graphs (gtf.graph.unpack) -> pickle each graph to
            the output directory under its global glob index

Subgraphs are independent (no edge crosses two of them), so the concatenated stage
equals the stage on all subgraphs together: same values, same file numbering. The
workers are a pool forked once per process, at its first directory (in a CLI before the
GPU is initialised), and reused by later directories; they never touch the GPU, and only
numpy arrays cross the pipes. Reference exceptions raised on the device are re-raised
as the reference's exception class before any output is written (the reference loses
the stage's output too).
"""
from __future__ import annotations

import glob
import os
import pickle
import time
from typing import Callable, List

import numpy as np

from .graph import SLOT_FIELDS, concat, pack, unpack
from .stages import SUBGRAPH_SUFFIX, _raise_flags

STATIC_SLOT = ("slot_src", "slot_key", "is_edge", "rev_edge", "send_mw")
MUTABLE_NODE = ("has_merged", "merged_state", "merged_cov", "merged_prior", "has_tse", "has_uts", "degree")


def default_workers() -> int:
    """this process's CPU share (the GPU box gives a process 16 CPUs of a large host)"""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, env) if env else min(n, 16))


def device_memory() -> str:
    """DeviceGraph's allocator for a directory: "hip" (gtf.devmem, libgtf's own runtime,
    no torch) unless this process already imported torch, whose runtime libgtf then shares
    ("torch"). A drop-in CLI never imports torch: bringing it up costs 1.9-2.0 s of the
    extrapolation CLI's 2.3 s on the MI355X box (tools/cold_start.py).
    GTF_DROPIN_MEM=torch|hip overrides."""
    from .devmem import default_mem
    return default_mem()


_DEVICE_TOUCHED = False   # this process has (begun to) initialise the GPU


def _warm_device():
    """load libgtf lean and create the device context (one small allocation)"""
    import ctypes
    from . import _native as nat
    global _DEVICE_TOUCHED
    _DEVICE_TOUCHED = True
    try:
        L = nat.lib(lean=True)
        if L.gtf_device_init(0) == 0:
            p = ctypes.c_void_p()
            if L.gtf_malloc(ctypes.byref(p), 256) == 0:
                L.gtf_free(p)
    except Exception:   # DeviceGraph reports any failure itself
        pass


def _chunks(n_files: int, workers: int):
    w = max(1, min(workers, n_files))
    bounds = np.linspace(0, n_files, w + 1).round().astype(int)
    return [(int(bounds[i]), int(bounds[i + 1])) for i in range(w)]


def _job(conn, files, first_index, out_dir, states, merged):
    """one directory share: read + pack, wait for the stage's arrays, unpack + write"""
    t = [time.perf_counter()]
    subs = []
    for f in files:
        with open(f, "rb") as fh:
            subs.append(pickle.load(fh))
    t.append(time.perf_counter())
    g = pack(subs)
    t.append(time.perf_counter())
    conn.send(g)
    t.append(time.perf_counter())
    msg = conn.recv()
    t.append(time.perf_counter())
    if msg is None:            # the stage raised: write nothing
        conn.send(("ok", 0, {}))
        return
    node, slot = msg
    g.node.update(node)
    g.slot.update(slot)
    if g.n_nodes:
        unpack(g, subs, states=states, merged=merged)
    t.append(time.perf_counter())
    for i, s in enumerate(subs):
        with open(os.path.join(out_dir, "%d%s" % (first_index + i, SUBGRAPH_SUFFIX)), "wb") as fh:
            pickle.dump(s, fh, pickle.HIGHEST_PROTOCOL)
    t.append(time.perf_counter())
    d = np.diff(t)
    conn.send(("ok", len(subs), {"start": t[0], "load": d[0], "pack": d[1], "send": d[2], "wait": d[3],
                                 "unpack": d[4], "dump": d[5]}))


def _serve(conn):
    """a pool worker: one job (a directory share) after another until None"""
    import gc
    gc.disable()    # the pickles are trees of many small objects: no cycles to collect here (2-3x faster loads)
    while True:
        job = conn.recv()
        if job is None:
            return
        try:
            _job(conn, *job)
        except BaseException as e:     # reported to the main process, which drops the pool
            conn.send(("error", repr(e)))
            return
        gc.collect()    # the job's graphs (networkx views hold cycles), after its reply


class _Pool:
    """Worker processes forked once per process, at the first directory: in a drop-in CLI
    before this process initialises the GPU (forking a process that holds a GPU context
    costs ~10 ms per worker, and the COW-shared pages slow its later host-to-device
    copies), and reused by every later directory of a long-running caller."""

    def __init__(self, n, warm_file):
        import multiprocessing as mp
        if warm_file:
            # import what the pickles need (networkx, GNN_Measurement) here, once, before the
            # fork: otherwise every worker imports networkx (~0.2 s) on its first load
            with open(warm_file, "rb") as fh:
                pickle.load(fh)
        ctx = mp.get_context("fork")   # no exec: this process may hold the GPU
        self.n, self.procs, self.conns = n, [], []
        for _ in range(n):
            a, b = ctx.Pipe()
            p = ctx.Process(target=_serve, args=(b,), daemon=True)
            p.start()
            b.close()
            self.procs.append(p)
            self.conns.append(a)

    def alive(self):
        return all(p.is_alive() for p in self.procs)

    def close(self):
        for c in self.conns:
            try:
                c.send(None)
                c.close()
            except OSError:
                pass
        for p in self.procs:
            p.join(10)
            if p.is_alive():
                p.kill()


_POOL = None


def _get_pool(n, warm_file):
    global _POOL
    if _POOL is not None and (_POOL.n != n or not _POOL.alive()):
        _drop_pool()
    if _POOL is None:
        import atexit
        if _DEVICE_TOUCHED:
            # a fork of a process that holds a GPU context works, but the children share its
            # pages copy-on-write and its later host-to-device copies slow down (_Pool)
            import warnings
            warnings.warn("gtf.dropin: re-forking the worker pool after this process initialised the GPU",
                          RuntimeWarning, stacklevel=3)
        _POOL = _Pool(n, warm_file)
        atexit.register(_drop_pool)
    return _POOL


def _drop_pool():
    global _POOL
    if _POOL is not None:
        _POOL.close()
        _POOL = None


def run_dir(input_dir: str, output_dir: str, body: Callable, *, states=("tse", "uts"), merged=True,
            workers: int = None, host_stage: Callable = None) -> dict:
    """Run one stage over a directory of subgraph pickles. ``body(DeviceGraph)`` issues the
    stage's device calls (e.g. ``lambda d: d.extrapolate(p)``). Returns counts and the
    host / device split of the wall time. ``host_stage(TrackGraph) -> flags`` replaces the
    device (tests run the CPU checker through the same worker machinery)."""
    t0 = time.perf_counter()
    files = glob.glob(input_dir + "*" + SUBGRAPH_SUFFIX)        # the reference's glob order
    workers = workers or default_workers()
    chunks = _chunks(len(files), workers)
    pool = _get_pool(workers, files[0] if files else None)
    conns = pool.conns[:len(chunks)]
    warm = None
    if host_stage is None and files and device_memory() == "hip":
        # bring the HIP runtime up while the workers read (after the fork: a fork of a
        # process that holds a GPU context slows its later copies, _Pool)
        import threading
        warm = threading.Thread(target=_warm_device, daemon=True)
        warm.start()
    try:
        for c, (lo, hi) in zip(conns, chunks):
            c.send((files[lo:hi], lo, output_dir, tuple(states), merged))
        from multiprocessing.connection import wait
        parts = [None] * len(conns)
        pending = {c: i for i, c in enumerate(conns)}
        while pending:                       # in completion order, so no worker blocks on its send
            for c in wait(list(pending)):
                m = c.recv()
                if isinstance(m, tuple) and m and m[0] == "error":
                    raise RuntimeError("drop-in worker: " + m[1])
                parts[pending.pop(c)] = m
        t1 = time.perf_counter()
        nonempty = [g for g in parts if g.n_nodes]
        flags = 0
        out_node, out_slot = None, None
        phases = {}
        if nonempty and host_stage is not None:
            g = concat(nonempty)
            flags = int(host_stage(g) or 0)
            out_node, out_slot = g.node, g.slot
        elif nonempty:
            from .device import DeviceGraph
            global _DEVICE_TOUCHED
            _DEVICE_TOUCHED = True
            if warm is not None:
                warm.join()
            tp = [time.perf_counter()]
            g = concat(nonempty)
            tp.append(time.perf_counter())
            d = DeviceGraph(g, mem=device_memory())
            tp.append(time.perf_counter())
            d.clear_errors()
            body(d)
            flags = d.errors()
            tp.append(time.perf_counter())
            d.download(g)
            tp.append(time.perf_counter())
            out_node, out_slot = g.node, g.slot
            phases = dict(zip(("concat", "upload", "stage", "download"), np.diff(tp).tolist()))
        t2 = time.perf_counter()
        if flags:
            for c in conns:
                c.send(None)
            for c in conns:
                c.recv()
            _raise_flags(flags)
        n0 = s0 = 0
        for c, part in zip(conns, parts):
            if not part.n_nodes:
                c.send(({}, {}))
                continue
            n1, s1 = n0 + part.n_nodes, s0 + part.n_slots
            c.send(({k: out_node[k][n0:n1] for k in MUTABLE_NODE},
                    {k: out_slot[k][s0:s1] for k in SLOT_FIELDS if k not in STATIC_SLOT}))
            n0, s0 = n1, s1
        written = 0
        wt = []
        for c in conns:
            m = c.recv()
            if m[0] != "ok":
                raise RuntimeError("drop-in worker: " + m[1])
            written += m[1]
            wt.append(m[2])
        t3 = time.perf_counter()
    except BaseException:
        if warm is not None:
            warm.join()  # never fork (a later pool) while that thread may hold runtime or malloc locks
        _drop_pool()     # workers may be mid-job: start clean next time
        raise
    # the slowest worker's phases (seconds) and the latest worker start after t0
    wt = [w for w in wt if w]
    worker = {k: max(w[k] for w in wt) for k in ("load", "pack", "send", "unpack", "dump")} if wt else {}
    worker["last_start"] = max(w["start"] for w in wt) - t0 if wt else 0.0
    return {"files": len(files), "written": written, "workers": len(chunks),
            "edges": int(sum(p.n_edges for p in parts)), "read_pack_s": t1 - t0, "device_s": t2 - t1,
            "unpack_write_s": t3 - t2, "wall_s": t3 - t0, "worker_max_s": worker, "device_phases_s": phases}


def _time_extrapolate(argv):
    """python -m gtf.dropin IN/ OUT/ REPS: the drop-in extrapolation stage (reference flags
    -c 2.0 -e 0.3 -z 0.4 -m 0.6 -b 550) over IN/, REPS + 1 times in this fresh process (the
    first run loads the code objects, forks the worker pool and initialises the GPU),
    printing the wall time of each as JSON. bench.py's dropin_stage runs it as a child
    process: its workers are forked before this process touches the GPU."""
    import json
    import sys
    from .params import Params
    ind, outd, reps = argv[0], argv[1], int(argv[2])
    p = Params()
    runs = [run_dir(ind, outd, lambda d: d.extrapolate(p)) for _ in range(reps + 1)]
    _drop_pool()
    json.dump({"runs": runs[1:], "first": runs[0]}, sys.stdout)


if __name__ == "__main__":
    import sys
    _time_extrapolate(sys.argv[1:])
