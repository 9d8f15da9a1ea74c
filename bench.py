#!/usr/bin/env python
"""Benchmark: edges/s of the fused extrapolate -> update -> KL-clustering pass.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c3|c2]

One step = one fused pass (gtf_pass: k_sender_scan, k_extrapolate, fused node
kernel) over one synthetic TrackML-shaped event held in HBM. Every step processes
the same input: the arrays a pass mutates and the next one reads (activation mask,
state-dict ranks, merged states: the 18 MB pass-input arena on C4) are staged in K
device copies before the timed region (DeviceGraph.stage_inputs), and step i runs on
copy i, so no restore copy sits between the passes. The line also reports
ms_per_step_inline_restore: the same K steps with a device-to-device restore of one
arena before each pass (round-1 method). Default workload "c4" = BASELINE.json
configs[3], a pileup-200-shaped event (~180k hits, ~1.0M directed edges),
the config the north-star 1-GPU target is quoted on; it fits one GPU. The event
is uploaded with its nodes renumbered into the node kernel's schedule order tile
by tile (--layout tiled, the default; "schedule" without tiles, "natural" keeps
the host order).

The K steps are timed twice, each run bracketed by barrier + synchronize: first
as a caller runs them (value, ms_per_step), then with HIP events recorded before,
between and after the pass's kernels on their stream (kernel_ms, the roofline of
the dominant kernel, instrumented_ms_per_step) -- every event record costs a few
microseconds of GPU timeline, so it stays out of the headline.

Multi-GPU (torchrun, one process per GPU): the headline is the north star's config 4,
ONE C4 event edge-sharded across the N ranks (gtf/shard.py: azimuthal wedges, each rank
owns the receivers of its wedge, one halo all-to-all over RCCL per pass), total work
fixed ("scaling": "strong"; at N = 1 the same event on one GPU). value = the event's
edges x steps / max elapsed over ranks, with the barrier + synchronize bracket. The
line also carries "event_replicas": every rank running its own C4 event (independent
events, no collective, "weak"), and "c5_event_sharded": config 5 sharded by event, every
rank its own 256-event batch ("weak", no collective).

CPU baselines (rank 0, N = 1 only): the repository's NumPy restatement of the pass
(oracle/gtf_oracle.py, kind "port", 1 core) on a bounded sample event of the same
generator, the C++ restatement (oracle/cpu_ref.cpp) on the bench event on 1 core and
all cores, and the drop-in stage wall time (gpickle in -> gpickle out).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "gnn-track-finding_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(g, params, n_tracks=4000):
    """BASELINE.md plan item 1, the headline denominator: the NumPy restatement of the pass
    (oracle.full_pass, the reference's own NumPy calls) on 1 core, timed on the WHOLE bench
    event (the same seeded C4 event the GPU passes run on; ~55-60 s). Beside it, as a
    secondary figure, the same restatement on a bounded sample event of the generator
    (~38k hits / ~179k edges, ~10 s), the round-1..4 method."""
    import gtf_oracle as O
    from gtf import synth
    h = g.copy()
    t0 = time.perf_counter()
    O.full_pass(h, params)
    dt = time.perf_counter() - t0
    out = {"value": g.n_edges / dt, "unit": "edges/s", "cores": 1, "kind": "port", "seconds": dt,
           "sample": "oracle/gtf_oracle.full_pass (NumPy restatement of the reference's calls) on the whole bench "
                     "event itself (%d hits / %d directed edges), one pass, %.1f s on 1 core" % (g.n_nodes, g.n_edges, dt)}
    if n_tracks:
        s = synth.event(seed=12345, n_tracks=n_tracks, fake_mean=synth.C4_FAKE)
        t0 = time.perf_counter()
        O.full_pass(s, params)
        ds = time.perf_counter() - t0
        out["bounded_sample"] = {"value": s.n_edges / ds, "unit": "edges/s", "seconds": ds,
                                 "sample": "one synthetic event of %d hits / %d directed edges (pileup-200 density)"
                                           % (s.n_nodes, s.n_edges)}
    return out


def cpu_baseline_cpp(g, params, reps=5):
    """BASELINE.md plan item 2: the C++ fp64 restatement (oracle/cpu_ref.cpp, OpenMP over
    senders and receivers) on the benchmark event itself, 1 core and every core of this
    process's share (OMP_NUM_THREADS, else os.cpu_count()); warm passes, median of reps."""
    import cpu_ref
    if not os.path.exists(cpu_ref.LIB):
        return {"error": "oracle/build/libcpuref.so not built"}
    allc = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    out = {"unit": "edges/s", "kind": "port", "cpu_model": cpu_model(), "nproc": os.cpu_count(),
           "sample": "oracle/cpu_ref.cpp full pass on the whole bench event (%d directed edges), median of %d "
                     "warm passes" % (g.n_edges, reps)}
    out["threads_note"] = ("'omp_threads_%d' = OMP_NUM_THREADS of this process (the GPU box gives a process "
                           "a 16-CPU share of an nproc=%d host), not every core of the host" % (allc, os.cpu_count() or 0))
    for label, th in (("1_core", 1), ("omp_threads_%d" % allc, allc)):
        ts = []
        for _ in range(reps + 1):
            h = g.copy()
            b = cpu_ref.Bound(h)
            cp = cpu_ref.params(params)
            import ctypes
            t0 = time.perf_counter()
            flags = cpu_ref.lib().cr_full_pass(ctypes.byref(b.c), ctypes.byref(cp), th)
            ts.append(time.perf_counter() - t0)
        dt = float(np.median(ts[1:]))
        out[label] = {"value": g.n_edges / dt, "cores": th, "s_per_pass": dt, "flags": int(flags)}
    return out


def dropin_input_vol7(params):
    """The reference-schema full-load network of the committed volume-7 134 event: the
    event conversion (event_conversion.py:53-101: construct_graph, weakly connected
    subgraphs, TSE, activation, priors, weights, degree) through the drop-in modules, then
    every node's merged state = a copy of its first TSE entry (SURVEY §8d full load)."""
    import numpy as np_
    from gtf import io, stages as st
    kat = os.path.join(ROOT, "tests", "golden", "kat134")
    subs = io.build_networkx(os.path.join(kat, "event_1_filtered_graph_"), 7, 7, os.path.join(kat, "truth_vol7.csv"))
    subs = st.compute_track_state_estimates(subs, params.sigma0xy, params.sigma0rz, params.sigma0rz2,
                                            params.endcap_boundary)
    for s in subs:
        for e in s.edges:
            s.edges[e]["activated"] = 1
    st.compute_prior_probabilities(subs, "track_state_estimates")
    st.compute_mixture_weights(subs, "track_state_estimates")
    st.node_degrees(subs)
    for s in subs:
        for n in s.nodes:
            tse = s.nodes[n]["track_state_estimates"]
            if tse:
                first = next(iter(tse.values()))
                s.nodes[n]["merged_state"] = np_.array(first["edge_state_vector"], dtype=float).copy()
                s.nodes[n]["merged_cov"] = np_.array(first["edge_covariance"], dtype=float).copy()
                s.nodes[n]["merged_prior"] = first.get("prior", 1.0)
    return subs


def dropin_stage_wall(params, reps=3):
    """the drop-in stage wall time, gpickle in -> gpickle out, of the
    extrapolation stage (extrapolate_merged_states.py:521-572's main body through the
    drop-in runner gtf.dropin.run_dir: the per-file pickle reading / packing and unpacking /
    writing on worker processes, message passing + priors / reweight x2 + degree in one
    device call), on the full-load volume-7 134 network (14,766 directed edges), median of
    reps after the first. Timed in a fresh child process (python -m gtf.dropin), whose
    worker pool forks before it touches the GPU; interpreter start and imports excluded;
    the first directory's wall time (pool start-up, GPU context) reported beside.
    BASELINE.md times the reference's own stage on this input at 788 edges/s as is
    (18.7 s) and 5,367 edges/s with its prints stubbed."""
    import shutil
    import subprocess
    import tempfile
    from gtf import stages as st
    graphs = dropin_input_vol7(params)
    tmp = tempfile.mkdtemp(prefix="gtf_dropin_")
    try:
        ind, outd = os.path.join(tmp, "in") + "/", os.path.join(tmp, "out") + "/"
        os.makedirs(ind)
        os.makedirs(outd)
        for i, s in enumerate(graphs):
            st.save_network(ind, i, s)
        edges = sum(s.number_of_edges() for s in graphs)
        env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "gnn-track-finding_amd"))
        r = subprocess.run([sys.executable, "-m", "gtf.dropin", ind, outd, str(reps)], env=env, cwd=ROOT,
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            return {"error": r.stderr[-400:]}
        out = json.loads(r.stdout)
        runs = out["runs"]
        med = sorted(runs, key=lambda x: x["wall_s"])[len(runs) // 2]
        # the CLI as run_gnn_trackml_mod.sh calls it: one fresh process per stage, whole
        # wall time (interpreter, imports, worker pool, GPU context, stage, exit); the lean
        # runtime (no torch, gtf.devmem) vs the same CLI made to hold torch
        cli = [sys.executable, os.path.join(ROOT, "gnn-track-finding_amd", "extrapolate", "extrapolate_merged_states.py"),
               "-i", ind, "-o", outd, "-c", str(params.chi2_cut), "-e", str(params.sigma0xy), "-z",
               str(params.sigma0rz), "-m", str(params.sigma0rz2), "-b", str(params.endcap_boundary)]
        cli_s = {}
        for mem, n in (("hip", 3), ("torch", 1)):
            ts = []
            for _ in range(n):
                t0 = time.perf_counter()
                rc = subprocess.run(cli, env=dict(env, GTF_DROPIN_MEM=mem), cwd=ROOT, capture_output=True,
                                    text=True, timeout=600)
                ts.append(time.perf_counter() - t0)
                if rc.returncode != 0:
                    return {"error": "CLI (%s): %s" % (mem, rc.stderr[-400:])}
            cli_s[mem] = sorted(ts)[len(ts) // 2]
        return {"stage": "extrapolate (drop-in runner gtf.dropin.run_dir, child process)",
                "input": "vol-7 134 full load", "subgraphs": len(graphs), "edges": edges,
                "wall_s": med["wall_s"], "edges_per_s": edges / med["wall_s"], "workers": med["workers"],
                "read_pack_s": med["read_pack_s"], "device_s": med["device_s"],
                "unpack_write_s": med["unpack_write_s"], "worker_max_s": med.get("worker_max_s"),
                "device_phases_s": med.get("device_phases_s"),
                "first_run_wall_s": out["first"]["wall_s"],
                "first_run_note": "the first directory of the process: forks the worker pool (after importing "
                                  "what the pickles need), creates the GPU context, loads code",
                "cli_process_wall_s": cli_s["hip"], "cli_edges_per_s": edges / cli_s["hip"],
                "cli_process_wall_s_with_torch": cli_s["torch"],
                "cli_note": "extrapolate_merged_states.py -i -o -c -e -z -m -b in a fresh process, whole wall time "
                            "(median of 3); its device arrays come from libgtf (gtf.devmem), no torch in the process; "
                            "_with_torch: the same CLI holding torch tensors (GTF_DROPIN_MEM=torch)",
                "reference_as_is_edges_per_s": 788, "reference_prints_stubbed_edges_per_s": 5367}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def bench_c5(dev, steps, warmup, n_events=256, n_batches=8, hot=True, dtypes=("f64", "f32"), kl_tile=None):
    """Config 5: parabolic-model states + pairwise KL (gtf_parabolic_kl) over a batch of
    256 copies of the committed volume-7 134 event (tests/golden/kat134, coordinates
    jittered per copy), fp64 and fp32, with the fp32-vs-fp64 tolerance sweep.

    Cold timing (the roofline): n_batches independent 256-event batches, each in its own
    device buffers (jitter seeds 0..n_batches-1), launched in rotation, so between two
    launches on one batch the other n_batches - 1 batches stream through the caches;
    the whole footprint (~1 GB at 8 batches) is >= 4x the 256 MB Infinity Cache and no
    launch finds its inputs cached (SURVEY §8d "Avoid caches in roofline runs"). The
    round-2 method -- one batch relaunched back to back, its ~125 MB inside the
    Infinity Cache -- is reported beside it as hot_same_buffers."""
    import torch
    from gtf import io, parabolic, roofline as rf
    kat = os.path.join(ROOT, "tests", "golden", "kat134")
    g = io.load_event(os.path.join(kat, "event_1_filtered_graph_"), 7, 7)
    truth = io.read_truth(os.path.join(kat, "truth_vol7.csv"), g.node["node_id"])
    ptr0, src0 = parabolic.in_edge_csr(g)
    ptr, src, gnn, tr = parabolic.batch(ptr0, src0, g.node["gnn"], truth, n_events)
    if kl_tile is None:
        kl_tile = int(os.environ.get("GTF_KL_TILE", "0"))   # 0: the ordered layout (the tiled one measured no faster)
    # tiled: azimuth-sorted per event (sort window = one event's nodes), then tiles
    tile_b1 = os.environ.get("GTF_KL_TILE_B1", "1") != "0"   # tiled: the 3- / 4-edge nodes in the tiles too
    k = parabolic.ParabolicKL(ptr, src, gnn, tr, dev, ordered=True, tile=kl_tile, sort_window=ptr0.size - 1,
                              tile_b1=tile_b1)
    ks = [k] + [k.replica(gnn=parabolic.batch(ptr0, src0, g.node["gnn"], truth, n_events, seed=e)[2])
                for e in range(1, n_batches)]
    keep = os.environ.get("GTF_KL_KEEP")   # diagnostics: launch only these buckets ("0", "123", ...)
    if keep is not None:
        for kk in ks:
            for q in range(4):
                if str(q) not in keep:
                    kk._g.count[q] = 0
    res = {"workload": "%d x committed vol-7 134 event (jittered copies)" % n_events, "nodes": k.n_nodes,
           "layout": ("tiled, %d %s nodes per tile, LDS window" % (kl_tile, "1..4-edge" if tile_b1 else "1..2-edge")
                      if kl_tile else "ordered (bucket ranges over the batch)"),
           "in_edges": k.n_slots, "pairs": k.n_pairs, "listed_nodes": k.n_listed, "batches_rotated": n_batches}
    outs = {}
    launches = max(steps, 2 * n_batches) // n_batches * n_batches

    def timed(kk, oo, dt, n):
        # n launches back to back between two events: the launch time on the stream, free
        # of the host's per-call enqueue gap (one ctypes call ~8 us, longer than a small
        # kernel), so kernel_ms is the device time per launch
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.record()
        for i in range(n):
            kk[i % len(kk)].run(oo[i % len(kk)], dt)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / n, (time.perf_counter() - t0) / n

    for dt in dtypes:
        oo = [kk.alloc(dt, emp="var") for kk in ks]
        for _ in range(warmup):
            for kk, o in zip(ks, oo):
                kk.run(o, dt)
        ms, wall = timed(ks, oo, dt, launches)                       # cold: rotation over the batches
        ms_hot = timed(ks[:1], oo[:1], dt, launches)[0] if hot else float("nan")   # hot: one batch back to back
        nbytes = rf.parabolic_kl_bytes(k.n_nodes, res["listed_nodes"], k.n_slots, k.n_pairs, dt)
        foot = sum(kk.footprint_bytes(o) for kk, o in zip(ks, oo))
        gbs = nbytes / (ms * 1e-3) / 1e9
        res[dt] = {"pairs_per_s": k.n_pairs / (ms * 1e-3), "kernel_ms": ms, "wall_ms_per_launch": wall * 1e3,
                   "launches": launches,
                   # the order of this dtype's launches in a kernel trace (tools/kstats_c5.py splits
                   # a rocprofv3 trace by it: the cold rotation's average apart from the hot one's)
                   "launch_sequence": {"warmup": warmup * len(ks), "cold": launches, "hot": launches if hot else 0},
                   "roofline": {"bound": "hbm", "achieved": gbs, "peak": rf.HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": gbs / rf.HBM_PEAK_GBS, "algorithmic_bytes_per_launch": nbytes,
                                "footprint_bytes_all_batches": foot, "footprint_bytes_per_batch": foot // len(ks),
                                "timing": "cold: launches rotate over %d resident batches" % len(ks)},
                   "hot_same_buffers": {"kernel_ms": ms_hot, "frac": nbytes / (ms_hot * 1e-3) / 1e9 / rf.HBM_PEAK_GBS,
                                        "note": "one batch relaunched back to back (its footprint fits the "
                                                "256 MB Infinity Cache): not a roofline figure"}}
        outs[dt] = oo[0]
        del oo
    if len(outs) < 2:
        res["device_error_flags"] = max(kk.errors() for kk in ks)
        return res
    a = outs["f64"]["kl"].double().cpu().numpy()
    b = outs["f32"]["kl"].double().cpu().numpy()
    rel = np.abs(b - a) / np.maximum(np.abs(a), 1e-300)
    res["fp32_vs_fp64"] = {
        "rel_err_p50": float(np.percentile(rel, 50)), "rel_err_p99": float(np.percentile(rel, 99)),
        "rel_err_p999": float(np.percentile(rel, 99.9)), "rel_err_max": float(rel.max()),
        "decision_flips": {str(t): int(((a < t) != (b < t)).sum()) for t in (1.0, 2.0, 10.0, 100.0)},
        "truth_identical": bool(torch.equal(outs["f64"]["truth"], outs["f32"]["truth"]))}
    res["device_error_flags"] = max(kk.errors() for kk in ks)
    return res


def bench_components(g, params, dev, reps=5):
    """The north-star loop's other two device stages on the bench event (SURVEY §8 a15,
    a16), after one fused pass, in the headline's tiled node order (host-order inputs and
    outputs are mapped by DeviceGraph):
    the updated-state distance table (calculate_distance_between_updated_track_states.py,
    gtf_updated_state_distances: pair counts, scan, pair kernel) and tag propagation
    (tag_propagation.py:97-164, Jacobi max sweeps until flips / processed <= 10 %, the flip
    count read back after each sweep as the script's stop test needs), initial tag = node
    index, radius = r. Wall times with the device synchronised, median of reps; a15 / a2
    outputs left in the device layout's node order (host_order=False: no reordering
    gathers, as a device-resident caller consumes them)."""
    import torch
    from gtf.device import DeviceGraph
    from gtf import roofline as rf
    d = DeviceGraph(g, dev, layout="tiled")
    d.clear_errors()
    d.full_pass(params)
    out = {}
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ptr, cols = d.updated_state_distances(host_order=False)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    npairs = int(cols["chi2"].numel())
    dt = float(np.median(ts[1:]))
    out["a15_updated_state_distances"] = {"pairs": npairs, "wall_ms": dt * 1e3, "pairs_per_s": npairs / dt}
    out["a16_tag_propagation"] = bench_tags(d, g, dev, reps)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # a2: the initial per-edge states of event conversion (helper.py:238-452 + priors,
    # mixture weights, degree; pipeline.build_event's device half) on the same event
    def tse():
        d.track_state_estimates(params, host_order=False)
        d.node_ops(["priors_tse", "mw_tse", "degree"], params)
    tse()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        tse()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    out["a2_initial_states"] = {"edges": g.n_edges, "call_ms": ms, "edges_per_s": g.n_edges / (ms * 1e-3),
                                "reference_cpu_edges_per_s": 18900,
                                "note": "gtf_track_state_estimates + gtf_node_ops(priors, weights, degree), 10 calls "
                                        "back to back between two events; reference figure: its own helper.py on the "
                                        "134 all-volume event, 1 core (BASELINE.md)"}
    d.raise_errors()
    del d
    out["f_pipeline_vol7"] = bench_pipeline_vol7(params, dev)
    out["f2_event_build_c4"] = bench_event_build(g, dev)
    return out


def bench_event_build(g, dev, reps=3):
    """SURVEY §8f #2 on a C4-sized edge list: the event's undirected edges as shuffled CSV
    rows with random 40-bit node ids, built into the packed CSR by the host builder
    (gtf_build_event_csr, C++) and on the GPU (gtf_build_event_csr_device; the call
    includes uploading the columns and downloading the arrays), the same arrays bit for bit
    (tests/test_gpu_build.py). Median of reps after a first call."""
    from gtf import io
    rng = np.random.default_rng(5)
    dst = np.repeat(np.arange(g.n_nodes), np.diff(g.slot_ptr))
    src = g.slot["slot_src"]
    keep = (src >= 0) & (src < dst)
    a, b = src[keep], dst[keep]
    perm = rng.permutation(a.size)
    ids = rng.choice(2 ** 40, size=g.n_nodes, replace=False).astype(np.int64)
    a, b = ids[a[perm]], ids[b[perm]]
    res = {"nodes": int(g.n_nodes), "rows": int(a.size)}
    for name, device in (("host_cpp_s", None), ("device_s", dev)):
        ts = []
        for _ in range(reps + 1):
            t0 = time.perf_counter()
            o, e, nsub = io.csr_from_rows(ids, a, b, device)
            ts.append(time.perf_counter() - t0)
        res[name] = float(np.median(ts[1:]))
        res["directed_edges"], res["subgraphs"] = e, nsub
    res["speedup"] = res["host_cpp_s"] / res["device_s"]
    return res


def bench_pipeline_vol7(params, dev):
    """event conversion (CSV -> CSR in C++, states on the device) and
    the three iterations of run_gnn_trackml_mod.sh in one process on the committed
    volume-7 134 event, wall times per stage (second run; the first loads code objects).
    The candidate counts are the reference's own (1,055 / 110 / 2)."""
    import torch
    from gtf import pipeline
    prefix = os.path.join(ROOT, "tests", "golden", "kat134", "event_1_filtered_graph_")
    res = None
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g7, vivl = pipeline.build_event(prefix, 7, 7, params, dev)
        t1 = time.perf_counter()
        its = pipeline.run(g7, vivl, 3, params, device=dev)
        t2 = time.perf_counter()
        res = {"event": "vol-7 134 (%d nodes, %d directed edges)" % (g7.n_nodes, g7.n_edges),
               "event_conversion_s": t1 - t0, "three_iterations_s": t2 - t1,
               "iterations": [{"stage": it.stage, "candidates": len(it.candidates),
                               "seconds": {k: round(v, 5) for k, v in it.seconds.items()}} for it in its]}
    return res


def bench_c5_sharded(dev, steps, warmup, rank, world, backend, n_events=256):
    """Config 5 event-sharded across the ranks (events are independent, no
    exchange): every rank runs its own 256-event batch (jitter seed per rank), fp64, K
    launches bracketed by barrier + synchronize, max over ranks. Per-rank work is fixed
    as N grows ("weak")."""
    import torch
    import torch.distributed as dist
    from gtf import io, parabolic
    kat = os.path.join(ROOT, "tests", "golden", "kat134")
    g = io.load_event(os.path.join(kat, "event_1_filtered_graph_"), 7, 7)
    truth = io.read_truth(os.path.join(kat, "truth_vol7.csv"), g.node["node_id"])
    ptr, src = parabolic.in_edge_csr(g)
    ptr, src, gnn, tr = parabolic.batch(ptr, src, g.node["gnn"], truth, n_events, seed=rank)
    k = parabolic.ParabolicKL(ptr, src, gnn, tr, dev, ordered=True)
    out = k.alloc("f64", emp="var")
    for _ in range(warmup):
        k.run(out, "f64")
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        k.run(out, "f64")
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    el = reduce_scalar(time.perf_counter() - t0, dist.ReduceOp.MAX, dev, backend)
    pairs = reduce_scalar(float(k.n_pairs), dist.ReduceOp.SUM, dev, backend)
    flags = int(reduce_scalar(k.errors(), dist.ReduceOp.MAX, dev, backend))
    return {"scaling": "weak", "n_gpus": world, "events_per_rank": n_events, "pairs_total": int(pairs),
            "pairs_per_s": pairs * steps / el, "ms_per_launch": el / steps * 1e3, "dtype": "f64",
            "collective": "none (events are independent)", "device_error_flags": flags}


def bench_tags(d, g, dev, reps=5, descending=False):
    """tag propagation (a16, tag_propagation.py:99-164) on a device graph after a pass: one
    gtf_tag_propagate call (wall), the host-order API, and the prepare / sweep kernels alone
    (K calls between two events) against SURVEY §8(d)'s B_tag = 4 E + 8 N per sweep.
    Initial tag = node index; descending: N - 1 - index, so a node's inner neighbours (the
    lower layers come first in the generator's hit order) carry the larger tags and the
    maximum travels outward layer by layer -- several sweeps instead of one"""
    import torch
    from gtf import roofline as rf
    tags = np.arange(g.n_nodes, dtype=np.int64)
    if descending:
        tags = tags[::-1].copy()
    radius = np.ascontiguousarray(g.node["xyzr"][:, 3])
    import ctypes
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rad = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(radius))).to(dev)
    t_init = torch.from_numpy(np.ascontiguousarray(d._to_dev_nodes(tags))).to(dev)
    ta = torch.empty_like(t_init)
    # the stage as a device-resident caller runs it: one gtf_tag_propagate call (prepare, the
    # sweeps with their stop test on the device, one flip-count read per batch), wall time
    # from the call to its return with the final tags in place
    ts = []
    for _ in range(reps + 1):
        ta.copy_(t_init)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        flips = d.tag_propagation_dev(ta, rad)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts[1:]))
    # the same with host-order inputs and outputs (upload, download, reordering: the Python API)
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.tag_propagation(tags, radius)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    dt_host = float(np.median(ts[1:]))
    # the prepare and sweep kernels alone: K calls back to back between two events
    keep = torch.zeros(max(g.n_edges, 1), dtype=torch.uint8, device=dev)
    proc = torch.zeros(max(g.n_nodes, 1), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(2, dtype=torch.int32, device=dev)
    tb = torch.empty_like(ta)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    K = 50
    e0.record()
    for i in range(K):
        d.lib.gtf_tag_prepare(ctypes.byref(d.cg), vp(rad), vp(keep), vp(proc), vp(cnt), d.stream)
    e1.record()
    torch.cuda.synchronize()
    prep_ms = e0.elapsed_time(e1) / K
    e0.record()
    for i in range(K):
        d.lib.gtf_tag_sweep(ctypes.byref(d.cg), vp(keep), vp(proc), vp(ta if i % 2 == 0 else tb),
                            vp(tb if i % 2 == 0 else ta), vp(cnt[1:2]), d.stream)
    e1.record()
    torch.cuda.synchronize()
    sweep_ms = e0.elapsed_time(e1) / K
    # the sweep kernel the stage itself runs, per sweep: the marginal time of the product call
    # between S1 and S2 forced sweeps (flip threshold -1: the stop rule never fires), compact
    # kept lists with int32 tags (the default) and the keep-mask sweeps (GTF_TAG_CSR=0)
    S1, S2 = 8, 264
    marg = {}
    prev = os.environ.get("GTF_TAG_CSR")
    try:
        for name, val in (("csr_int32", "1"), ("keep_mask", "0")):
            os.environ["GTF_TAG_CSR"] = val
            w = {}
            for S in (S1, S2):
                ts = []
                for _ in range(reps + 1):
                    ta.copy_(t_init)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    d.tag_propagation_dev(ta, rad, threshold=-1.0, max_sweeps=S)
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t0)
                w[S] = float(np.median(ts[1:]))
            marg[name] = (w[S2] - w[S1]) / (S2 - S1) * 1e3
    finally:
        if prev is None:
            os.environ.pop("GTF_TAG_CSR", None)
        else:
            os.environ["GTF_TAG_CSR"] = prev
    sweeps = len(flips)
    nbytes = 4 * g.n_edges + 8 * g.n_nodes   # SURVEY §8d B_tag, per sweep
    stage_sweep = {k: {"sweep_ms": v, "achieved_GBps": nbytes / (v * 1e-3) / 1e9,
                       "frac_of_peak": nbytes / (v * 1e-3) / 1e9 / rf.HBM_PEAK_GBS} for k, v in marg.items()}
    return {"initial_tags": "N - 1 - node index" if descending else "node index",
            "sweeps": sweeps, "flips": [int(x) for x in flips], "stage_wall_ms": dt * 1e3,
                                  "stage_wall_host_order_ms": dt_host * 1e3,
                                  "prepare_call_ms": prep_ms, "sweep_call_ms": sweep_ms,
                                  "stage_over_kernels": dt * 1e3 / (prep_ms + sweeps * sweep_ms),
                                  "algorithmic_bytes_per_sweep": nbytes,
                                  "achieved_GBps": nbytes / (sweep_ms * 1e-3) / 1e9,
                                  "frac_of_peak": nbytes / (sweep_ms * 1e-3) / 1e9 / rf.HBM_PEAK_GBS,
            "stage_sweep": stage_sweep,
            "stage_sweep_note": "per-sweep time of the sweeps gtf_tag_propagate itself runs: (wall(%d) - "
                                "wall(%d)) / %d of the call with flip threshold -1 (every sweep runs); "
                                "csr_int32 = the stage's default sweep (compact kept lists, int32 tags "
                                "while every tag fits), keep_mask = GTF_TAG_CSR=0 (the sender-schedule "
                                "sweep of gtf_tag_sweep, int64 tags and the keep mask); the *_call_ms / "
                                "achieved_GBps / frac_of_peak fields above time gtf_tag_sweep alone"
                                % (S2, S1, S2 - S1),
                                  "note": "stage_wall_ms: one gtf_tag_propagate call on device-resident tags / radius "
                                          "(prepare, sweeps with the stop rule evaluated on the device, one flip-count "
                                          "read per batch of sweeps), call to return; stage_over_kernels = that wall "
                                          "time / (prepare + sweeps x sweep) kernel time; *_call_ms: K calls back to "
                                          "back between two events; stage_wall_host_order_ms adds the host-order "
                                          "upload, download and reordering of DeviceGraph.tag_propagation"}


def bench_c3_section(dev, steps, warmup, params, layout="tiled", tile=4096):
    """configs[2] beside the C4 headline: 64 C2-like events fused into one CSR (2.0 M hits /
    5.9 M edges), K passes on staged inputs, then the same K with HIP events around the
    kernels -- the fused node kernel's roofline on SURVEY §8(d)'s bytes at the size §8(d)
    quotes roofline fractions on (>= 1 GB of traffic per pass)"""
    import torch
    from gtf import synth, roofline as rf
    from gtf.device import DeviceGraph
    g = synth.workload("c3", seed=0)
    d = DeviceGraph(g, dev, layout=layout, tile=tile)
    snap = d.snapshot(DeviceGraph.PASS_INPUTS)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(steps)]
    for row in evs:
        for e in row:
            e.record()
    handles = [[e.cuda_event for e in row] for row in evs]
    d.clear_errors()
    for _ in range(warmup):
        d.restore(snap)
        d.full_pass(params)
    d.stage_inputs(steps)

    def run(instrumented):
        d.fill_inputs(snap)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            d.use_inputs(i)
            d.full_pass(params, events=handles[i] if instrumented else None)
        torch.cuda.synchronize()
        d.use_inputs(None)
        return (time.perf_counter() - t0) / steps

    t = run(False)
    run(True)
    avg = lambda a, b: float(np.mean([evs[i][a].elapsed_time(evs[i][b]) for i in range(steps)]))  # noqa: E731
    node_ms = avg(2, 3)
    nb = rf.node_bytes(g.n_edges, g.n_nodes)
    pb = rf.pass_bytes(g.n_edges, g.n_nodes)
    res = {"workload": "64 C2-like events fused into one CSR (configs[2])", "nodes": g.n_nodes,
           "directed_edges": g.n_edges, "steps": steps, "ms_per_step": t * 1e3, "edges_per_s": g.n_edges / t,
           "kernel_ms": {"k_sender": avg(0, 1), "k_extrapolate": avg(1, 2), NODE_KERNEL: node_ms},
           "roofline": {"bound": "hbm", "kernel": NODE_KERNEL, "algorithmic_bytes_per_launch": nb,
                        "achieved": nb / (node_ms * 1e-3) / 1e9, "peak": rf.HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": nb / (node_ms * 1e-3) / 1e9 / rf.HBM_PEAK_GBS,
                        "byte_model": "SURVEY §8d (fused node kernel 89 B/edge + 186 B/node)"},
           "pass_roofline": {"algorithmic_bytes_per_step": pb, "frac": pb / t / 1e9 / rf.HBM_PEAK_GBS},
           "device_error_flags": d.errors()}
    # a16 on the fused 5.9 M-edge graph after the pass: several sweeps (where C4 stops after one),
    # the sweep kernel at a size where it can be bandwidth-bound
    try:
        res["a16_tag_propagation"] = bench_tags(d, g, dev, reps=3, descending=True)
    except Exception as ex:   # reported; the section stands
        res["a16_tag_propagation"] = {"error": repr(ex)[:300]}
    del d
    torch.cuda.empty_cache()
    return res


def device_copy_gbps(dev, nbytes=1 << 30, reps=10):
    """measured device-to-device copy bandwidth (bytes read + written per second), the
    practical HBM ceiling SURVEY §8d asks the roofline to be quoted against beside the
    spec peak"""
    import torch
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbps = 2.0 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    return gbps


def reduce_scalar(x, op, dev, backend):
    """all-reduce one number across ranks (device tensor over RCCL, host tensor over gloo)"""
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=op)
    return float(t.item())


def bench_sharded(workload, rank, world, dev, steps, warmup, params, backend="nccl"):
    """Config 4 as the north star states it: ONE pileup-200 event edge-sharded across
    the ranks (azimuthal wedges balanced by slots; gtf/shard.py), one halo exchange per
    pass (all-to-all over RCCL). Total work is fixed as N grows ("strong"). Every rank
    builds the same event (seed 0). Times K steps of restore + pass + exchange, and the
    same K steps without the exchange (pass_ms: the compute share)."""
    import torch
    import torch.distributed as dist
    from gtf import synth
    from gtf.device import DeviceGraph
    from gtf.shard import ShardedDeviceGraph
    from gtf import roofline as rf
    g = synth.workload(workload, seed=0)
    sd = ShardedDeviceGraph(g, rank, world, dev, backend=backend)
    torch_backend = "gloo" if backend == "gloo" else "nccl"
    snap = sd.d.snapshot(DeviceGraph.PASS_INPUTS)
    sd.d.clear_errors()
    for _ in range(warmup):
        sd.d.restore(snap)
        sd.step(params)
    sd.d.stage_inputs(steps)   # step i runs on staged copy i of the pass input (as at N = 1)

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(steps)]
    for row in evs:      # torch creates the HIP event on first record
        for e in row:
            e.record()
    handles = [[e.cuda_event for e in row] for row in evs]

    def run(exchange, instrumented=False, overlap=True):
        sd.overlap = overlap
        sd.d.fill_inputs(snap)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            sd.d.use_inputs(i)
            if exchange:
                sd.step(params)   # (the previous step's halo exchanged beside this pass's phase 1a)
            else:
                sd.pass_(params, events=handles[i] if instrumented else None)
        if exchange:
            sd.flush()     # the last pass's halo, inside the timed region
        t_issue = time.perf_counter() - t0     # host time to enqueue the K steps
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        sd.d.use_inputs(None)
        issue[exchange] = reduce_scalar(t_issue, dist.ReduceOp.MAX, dev, torch_backend)
        return reduce_scalar(time.perf_counter() - t0, dist.ReduceOp.MAX, dev, torch_backend)

    issue = {}
    # the step in both forms: the halo exchange beside the next pass's phase 1a (overlap), and
    # the one-call pass followed by the exchange; the headline takes the faster (the phased
    # pass costs two more launches, the overlap hides the exchange: which wins depends on the
    # exchange's time on the node's xGMI)
    el_ov = run(True, overlap=True)
    issue_ov = issue[True]
    el_seq = run(True, overlap=False)
    el = min(el_ov, el_seq)
    if el == el_ov:
        issue[True] = issue_ov
    el_pass = run(False)
    run(False, instrumented=True)   # this rank's kernels between events (the sharded roofline)
    # the overlapped step with HIP events between its parts on the pass stream (rank 0's in
    # the line): phase 1a, the wait for the halo and its unpack, phase 1b, the node kernels
    pevs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(steps)]
    sd.overlap = True
    sd.d.fill_inputs(snap)
    torch.cuda.synchronize()
    dist.barrier()
    for i in range(steps):
        sd.d.use_inputs(i)
        sd.step(params, phase_events=pevs[i])
    sd.flush()
    torch.cuda.synchronize()
    dist.barrier()
    sd.d.use_inputs(None)

    def pavg(a, b):
        return float(np.mean([pevs[i][a].elapsed_time(pevs[i][b]) for i in range(1, steps)]))   # (step 0: no halo)
    phase_ms = {"phase_1a": pavg(0, 1), "exchange_wait_and_unpack": pavg(1, 2), "phase_1b": pavg(2, 3),
                "node_kernels_and_pack": pavg(3, 4), "step": pavg(0, 4)}
    # the halo all-to-all alone (the collective, no pack / unpack), K times between barriers
    from gtf.shard import alltoall_bytes
    sview, rview = sd._io()[4:6]
    with torch.cuda.stream(sd._tstream()):
        for _ in range(2):
            alltoall_bytes(sview, rview, sd.send_sizes, sd.recv_sizes, torch_backend, None)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            alltoall_bytes(sview, rview, sd.send_sizes, sd.recv_sizes, torch_backend, None)
        torch.cuda.synchronize()
        a2a_s = reduce_scalar(time.perf_counter() - t0, dist.ReduceOp.MAX, dev, torch_backend)
    if backend == "native":   # libgtf's own grouped send / receive pairs: the whole exchange
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            sd.exchange()
        torch.cuda.synchronize()
        a2a_native_s = reduce_scalar(time.perf_counter() - t0, dist.ReduceOp.MAX, dev, torch_backend)
    else:
        a2a_native_s = None
    flags = int(reduce_scalar(sd.d.errors(), dist.ReduceOp.MAX, dev, torch_backend))
    hb = int(reduce_scalar(sd.halo_bytes, dist.ReduceOp.MAX, dev, torch_backend))
    pl = sd.plan

    def avg(a, b):
        return float(np.mean([evs[i][a].elapsed_time(evs[i][b]) for i in range(steps)]))

    # this rank's owned receivers / slots / directed edges (the per-GPU sizes of the headline)
    lo, hi = int(pl.slot_lo[rank]), int(pl.slot_hi[rank])
    own_nodes = int(pl.node_hi[rank] - pl.node_lo[rank])
    own_edges = int(sd.d.t["is_edge"][lo:hi].sum().item())
    k_ms = {"k_sender": avg(0, 1), "k_extrapolate": avg(1, 2), NODE_KERNEL: avg(2, 3)}
    node_b = rf.node_bytes(own_edges, own_nodes)
    ext_b = rf.extrap_bytes(own_edges, own_nodes)
    kr = {NODE_KERNEL: (k_ms[NODE_KERNEL], node_b),
          "k_sender+k_extrapolate": (k_ms["k_sender"] + k_ms["k_extrapolate"], ext_b)}
    kname = max(kr, key=lambda k: kr[k][0])
    own_edges_max = int(reduce_scalar(own_edges, dist.ReduceOp.MAX, dev, torch_backend))
    own_nodes_max = int(reduce_scalar(own_nodes, dist.ReduceOp.MAX, dev, torch_backend))
    roof = {"bound": "hbm", "kernel": kname, "rank": rank, "achieved": kr[kname][1] / (kr[kname][0] * 1e-3) / 1e9,
            "peak": rf.HBM_PEAK_GBS, "unit": "GB/s",
            "frac": kr[kname][1] / (kr[kname][0] * 1e-3) / 1e9 / rf.HBM_PEAK_GBS, "traffic": None,
            "algorithmic_bytes_per_launch": kr[kname][1], "kernel_ms": kr[kname][0],
            "kernel_ms_all": {k: round(v, 5) for k, v in k_ms.items()},
            "owned_directed_edges": own_edges, "owned_nodes": own_nodes,
            "byte_model": "SURVEY §8d on this rank's owned receivers and edges",
            "timing": "HIP events around this rank's kernels (gtf_pass_shard), no exchange"}
    # tag propagation (a16) on the same sharded event: owned-wedge sweeps + one
    # all-reduce(MAX) per sweep; wall time of the whole stage, max over ranks
    try:
        tags = np.arange(g.n_nodes, dtype=np.int64)
        sd.tag_propagation(tags, g.node["xyzr"][:, 3])    # warm
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        _, tflips = sd.tag_propagation(tags, g.node["xyzr"][:, 3])
        torch.cuda.synchronize()
        tag_s = reduce_scalar(time.perf_counter() - t0, dist.ReduceOp.MAX, dev, torch_backend)
        tag = {"ms": tag_s * 1e3, "sweeps": len(tflips), "flips": tflips,
               "collective": "one all_reduce(MAX) of n_nodes + world int64 words per sweep" +
                             (" (libgtf gtf_tag_propagate_shard)" if backend == "native" else "")}
    except Exception as ex:   # reported; the headline stands
        tag = {"error": repr(ex)[:300]}
    return {"scaling": "strong", "n_gpus": world, "edges": g.n_edges, "nodes": g.n_nodes,
            "ms_per_step": el / steps * 1e3, "edges_per_s": g.n_edges * steps / el,
            "step_form": "overlapped (phases)" if el == el_ov else "one-call pass, then the exchange",
            "ms_per_step_overlapped": el_ov / steps * 1e3, "ms_per_step_sequential": el_seq / steps * 1e3,
            "pass_ms_no_exchange": el_pass / steps * 1e3,
            "host_issue_ms_per_step": issue[True] / steps * 1e3,
            "host_issue_ms_per_step_no_exchange": issue[False] / steps * 1e3,
            "host_issue_note": "host time to enqueue the steps (max over ranks); close to ms_per_step = host-bound",
            "halo_bytes_per_rank_max": hb, "owned_slots_max": pl.cap_slots,
            "overlap": ("the halo exchange of pass i beside pass i+1's phase 1a (the senders whose state and "
                        "out-edge activations are all the rank's own, and the slots they send to; gtf_shard.phases)"),
            "rank0_split": sd.split_sizes,
            "rank0_phase_ms": phase_ms,
            "rank0_phase_timing": ("HIP events on rank 0's pass stream inside the overlapped step (steps 1..K-1): "
                                   "phase 1a, the wait for the previous halo + its unpack, phase 1b, the node kernels "
                                   "+ this pass's halo pack"),
            "alltoall_ms": a2a_s / steps * 1e3,
            "alltoall_note": ("the halo all_to_all_single alone (%s, no pack / unpack), wall time per call, max "
                              "over ranks" % torch_backend),
            "native_exchange_ms": a2a_native_s / steps * 1e3 if a2a_native_s is not None else None,
            "owned_slots_min": int((pl.slot_hi - pl.slot_lo).min()),
            "owned_directed_edges_max": own_edges_max, "owned_nodes_max": own_nodes_max,
            "collective": ("gtf_halo_exchange: per-destination halo segments, grouped ncclSend / ncclRecv inside "
                           "libgtf (RCCL over xGMI)" if backend == "native" else
                           "all_to_all_single of per-destination halo segments (RCCL over xGMI)"),
            "roofline": roof,
            "node_order": "azimuthal wedges, tiled slot-count buckets inside each", "device_error_flags": flags, "backend": backend,
            "tag_propagation": tag}


# the fused node kernel: priors, side norm, reweights, update and KL clustering of every
# receiver in one launch (gtf_pass.hip run_pass)
NODE_KERNEL = "k_node_multi<update+cluster> (KL-distance kernel)"
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06", "final5", "c4", "pmc_c4.json")
# per-launch SQ instruction counters of the pass kernels (tools/gpu_sqmix.sh, same event)
SQ_SUMMARY = os.path.join(ROOT, "profiles", "r06", "final5", "sqmix", "sqmix.json")
SQ_NAMES = {"k_sender+k_extrapolate": ("k_sender_sched", "k_extrapolate"),
            NODE_KERNEL: ("k_node_multi<11, 1, 3, 4, 3, 4, 5, 6, 2, 3, 4, 12, 10, 5, 8, 3>",
                          "k_node_multi<11, 1, 3, 4, 3, 4, 5, 6, 2, 3, 4, 10, 5, 8, 3>")}


def committed_valu(kernel, ms, workload, layout, tile):
    """The VALU-issue roofline of `kernel` beside the HBM one: the committed SQ counters'
    VALU instructions per launch at full issue rate on every SIMD (gtf.roofline
    valu_issue_floor_s) against the measured launch time; None off the profiled C4 config."""
    from gtf import roofline as rf
    if (workload, layout, tile) != ("c4", "tiled", 4096) or kernel not in SQ_NAMES:
        return None
    try:
        with open(SQ_SUMMARY) as f:
            allc = json.load(f)
        if kernel == NODE_KERNEL:   # the fused kernel under its current or its earlier op list
            cs = [next(allc[n] for n in SQ_NAMES[kernel] if n in allc)]
        else:
            cs = [allc[n] for n in SQ_NAMES[kernel]]
    except (OSError, KeyError, ValueError, StopIteration):
        return None
    floor = sum(rf.valu_issue_floor_s(c) for c in cs)
    return {"bound": "valu_issue", "valu_insts_per_launch": sum(c["SQ_INSTS_VALU"] for c in cs),
            "f64_insts_per_launch": sum(c.get(k, 0.0) for c in cs for k in rf.F64_COUNTERS),
            "issue_floor_us": floor * 1e6, "frac": floor / (ms * 1e-3),
            "source": os.path.relpath(SQ_SUMMARY, ROOT)}


def committed_traffic(workload, kernel, layout, tile, edges, nodes):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (separate FETCH_SIZE / WRITE_SIZE passes, tools/gpu_profile.sh; corrections in
    DESIGN.md), or None when no summary matches this workload / node layout / tile /
    kernel (traffic depends on the layout: 318 vs 201 MB for the node kernel) / event size."""
    try:
        with open(PMC_SUMMARY) as f:
            s = json.load(f)
    except OSError:
        return None
    if s.get("workload") != workload or s.get("layout") != layout or s.get("tile") != tile:
        return None
    if s.get("edges") != edges or s.get("nodes") != nodes:   # another generator's event
        return None
    k = s.get("kernels", {}).get(kernel)
    return None if k is None else k.get("hbm_bytes_per_launch")


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """One child process per rank (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torchrun
    sets them), each re-running this script with the same arguments; rank 0 prints the
    line. Called before any GPU call in this process. Returns the worst child exit code
    (a failed rank terminates the others)."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0:
                rc = rc or c
                for q in live:      # one rank failed: the others would wait in a collective
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c4", choices=["c2", "c3", "c4"])
    ap.add_argument("--cpu-tracks", type=int, default=4000,
                    help="tracks of the CPU baseline's secondary bounded sample (0: none)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="skip the config-5 parabolic-KL section")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in stage wall time")
    ap.add_argument("--no-c3", action="store_true",
                    help="skip the configs[2] (C3) section beside the C4 headline (its launches have their own grid "
                         "sizes: tools/kstats_by_grid.py separates them in a profiler's kernel trace)")
    ap.add_argument("--layout", default="tiled", choices=["tiled", "padded", "schedule", "natural"],
                    help="device node order (DeviceGraph layout)")
    ap.add_argument("--tile", type=int, default=4096, help="nodes per tile of --layout tiled")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo", "native"],
                    help="collectives for N > 1: nccl = torch.distributed over RCCL (the default), native = "
                         "libgtf's own RCCL communicator (gtf_comm_*, the id handed over torch.distributed; NOTE: "
                         "it has never run with more than one rank -- the test box has one GPU -- so its grouped "
                         "send / receive pairing at world > 1 is unverified on hardware), gloo = rehearsal with "
                         "several ranks on one GPU")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launched as `python bench.py --gpus N`: start the N ranks here, before anything
        # touches the GPU, one child process per GPU (what torchrun would do)
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist
    from gtf import synth
    from gtf.device import DeviceGraph
    from gtf.params import Params
    from gtf import roofline as rf

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if args.backend == "gloo":   # rehearsal: ranks may share the GPU
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = "cuda:%d" % local
    if world != args.gpus:
        raise SystemExit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    if world > 1:
        if args.backend in ("nccl", "native"):
            dist.init_process_group("nccl", device_id=torch.device(dev))
        else:   # rehearsal of the N > 1 path with several ranks on one GPU (RCCL needs one GPU per rank)
            dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)

    def barrier():
        if world > 1:
            dist.barrier()

    p = Params()
    g = synth.workload(args.workload, seed=1000 * rank)
    # nodes renumbered on upload (DeviceGraph layout "tiled", the default): inside every
    # run of 4096 nodes, bucketed by slot count, so each wavefront of the node kernel
    # reads one contiguous run of slots while neighbouring hits stay close for the sender
    # and extrapolation gathers; the results are the same bit for bit
    # (tests/test_gpu_fullsize.py)
    d = DeviceGraph(g, dev, layout=args.layout, tile=args.tile)
    snap = d.snapshot(DeviceGraph.PASS_INPUTS)
    K, W = args.steps, args.warmup
    NE = 5
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(NE)] for _ in range(K)]
    for row in evs:      # torch creates the HIP event on first record
        for e in row:
            e.record()
    handles = [[e.cuda_event for e in row] for row in evs]

    d.clear_errors()
    for _ in range(W):
        d.restore(snap)
        d.full_pass(p)

    d.stage_inputs(K)   # K resident copies of the pass input, one per timed step

    def timed(instrumented, inline_restore=False):
        """K steps bracketed by barrier + synchronize, step i on staged input copy i;
        instrumented: a HIP event before, between and after the pass's kernels on their
        stream (each event record is a few microseconds of GPU timeline, so the headline
        pass is timed without them); inline_restore: one resident input restored by a
        device copy before every pass instead (round-1 method, reported beside)"""
        d.fill_inputs(snap)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            if inline_restore:
                d.restore(snap)
            else:
                d.use_inputs(i)
            d.full_pass(p, events=handles[i] if instrumented else None)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        d.use_inputs(None)
        return time.perf_counter() - t0

    elapsed = timed(False)        # the headline: K passes as a caller runs them
    elapsed_ev = timed(True)      # the same K passes with per-kernel events (kernel_ms, roofline)
    elapsed_rs = timed(False, inline_restore=True)
    flags = d.errors()

    total_edges = float(g.n_edges)
    tb = "gloo" if args.backend == "gloo" else "nccl"   # the torch.distributed group's backend
    if world > 1:
        elapsed = reduce_scalar(elapsed, dist.ReduceOp.MAX, dev, tb)
        total_edges = reduce_scalar(total_edges, dist.ReduceOp.SUM, dev, tb)

    def avg(a, b):
        return float(np.mean([evs[i][a].elapsed_time(evs[i][b]) for i in range(K)]))

    # eligible nodes of the KL clustering (3 <= |updated_track_states| <= 15), from the
    # state after a pass (clustering does not change dict membership)
    gh = d.download(g.copy())   # host order (any device layout)
    sp = g.slot_ptr
    owner = np.repeat(np.arange(g.n_nodes), np.diff(sp))
    nst = np.bincount(owner, weights=(gh.slot["uts_rank"] >= 0), minlength=g.n_nodes)
    elig = (nst >= 3) & (nst <= 15) & (gh.node["has_uts"] == 1)
    e_elig = int(np.diff(sp)[elig].sum())
    # algorithmic bytes per launch on SURVEY §8d's byte model (the roofline's figure): the
    # fused node kernel 89 B per directed edge + 186 B per node, the extrapolation side
    # 94 B per edge + 104 B per node (together the pass's 183 E + 290 N); the builder's
    # finer model (every slot's reweight traffic + B_KL of the eligible nodes) beside it
    builder = {NODE_KERNEL: rf.fused_node_bytes(g.n_slots, g.n_nodes, e_elig, int(elig.sum()))}
    kern = {
        "k_sender": (avg(0, 1), None),
        "k_extrapolate": (avg(1, 2), None),
        NODE_KERNEL: (avg(2, 3), rf.node_bytes(g.n_edges, g.n_nodes)),
    }
    ext_ms = kern["k_sender"][0] + kern["k_extrapolate"][0]
    cands = {"k_sender+k_extrapolate": (ext_ms, rf.extrap_bytes(g.n_edges, g.n_nodes))}
    cands.update({k: v for k, v in kern.items() if v[1] is not None})
    name = max(cands, key=lambda k: cands[k][0])
    ms, nbytes = cands[name]
    # every kernel of the pass against the HBM roofline (algorithmic bytes / its time)
    per_kernel = {k: {"ms": round(v[0], 5), "algorithmic_bytes": v[1],
                      "achieved_GBps": v[1] / (v[0] * 1e-3) / 1e9,
                      "frac": v[1] / (v[0] * 1e-3) / 1e9 / rf.HBM_PEAK_GBS,
                      "builder_model_bytes": builder.get(k),
                      "builder_model_frac": builder[k] / (v[0] * 1e-3) / 1e9 / rf.HBM_PEAK_GBS if k in builder else None,
                      "traffic_bytes": committed_traffic(args.workload, k, args.layout, args.tile, g.n_edges, g.n_nodes),
                      "valu_roofline": committed_valu(k, v[0], args.workload, args.layout, args.tile)}
                  for k, v in cands.items()}
    achieved = nbytes / (ms * 1e-3) / 1e9
    traffic = committed_traffic(args.workload, name, args.layout, args.tile, g.n_edges, g.n_nodes)
    pass_b = rf.pass_bytes(g.n_edges, g.n_nodes)
    copy_gbps = device_copy_gbps(dev) if rank == 0 else None

    sharded = None
    if world > 1:
        try:
            sharded = bench_sharded(args.workload, rank, world, dev, K, W, p, args.backend)
        except Exception as ex:   # reported; the line then carries the replicas only and is marked
            sharded = {"error": repr(ex)[:300]}

    c5 = comps = c5_sharded = None
    if rank == 0 and world == 1 and not args.no_c5:
        c5 = bench_c5(dev, K, W)
        comps = bench_components(g, p, dev)
    if world > 1 and not args.no_c5:
        try:
            c5_sharded = bench_c5_sharded(dev, K, W, rank, world, tb)
        except Exception as ex:   # reported, the headline stands
            c5_sharded = {"error": repr(ex)[:300]}

    c3 = None
    if rank == 0 and world == 1 and args.workload == "c4" and not args.no_c3:
        try:
            c3 = bench_c3_section(dev, max(10, K // 5), 2, p, args.layout, args.tile)
        except Exception as ex:   # reported; the headline stands
            c3 = {"error": repr(ex)[:300]}

    cpu = cpu_cpp = dropin = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(g, p, args.cpu_tracks)
        cpu_cpp = cpu_baseline_cpp(g, p)
    if rank == 0 and world == 1 and not args.no_dropin:
        dropin = dropin_stage_wall(p)

    if rank == 0:
        out = {
            "metric": "edges/sec (extrapolate+update+KL) on TrackML hit graph; 1/2/4/8-GPU scaling",
            "value": total_edges * K / elapsed,
            "unit": "edges/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "instrumented_ms_per_step": elapsed_ev / K * 1e3,
            "ms_per_step_inline_restore": elapsed_rs / K * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded TrackML-shaped generator, gtf/synth.py)",
            "config": {"workload": {"c4": "pileup-200 TrackML-shaped event (configs[3]) per GPU",
                                    "c3": "64 C2-like events fused into one CSR per GPU (configs[2])",
                                    "c2": "single ~30k-hit / ~90k-edge event per GPU (configs[1])"}[args.workload],
                       "nodes_per_gpu": g.n_nodes, "directed_edges_per_gpu": g.n_edges,
                       "parallelism": "event-parallel x%d (no collective)" % world, "layout": args.layout,
                       "pass": "gtf_pass: extrapolate (a6-a8) + update (a3,a9,a10x2,a11) + KL cluster (a12-a14)"},
            "kernel_ms": {k: round(v[0], 5) for k, v in kern.items()},
            "kernels_roofline": per_kernel,
            "roofline": {"bound": "hbm", "kernel": name, "achieved": achieved, "peak": rf.HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / rf.HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_launch": nbytes, "kernel_ms": ms,
                         "device_copy_GBps": copy_gbps, "frac_of_device_copy": achieved / copy_gbps if copy_gbps else None,
                         "kl_eligible_nodes": int(elig.sum()), "kl_eligible_in_edges": e_elig,
                         "byte_model": "SURVEY §8d (fused node kernel 89 B/edge + 186 B/node)",
                         "builder_model_bytes_per_launch": builder.get(name),
                         "builder_model_frac": per_kernel[name]["builder_model_frac"],
                         "valu_roofline": per_kernel[name]["valu_roofline"]},
            "pass_roofline": {"bound": "hbm", "algorithmic_bytes_per_step": pass_b,
                              "byte_model": "SURVEY §8d B_alg = 183 E + 290 N",
                              "achieved": pass_b / (elapsed / K) / 1e9, "peak": rf.HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": pass_b / (elapsed / K) / 1e9 / rf.HBM_PEAK_GBS},
            "cpu_baseline": cpu,
            "cpu_baseline_cpp": cpu_cpp,
            "dropin_stage": dropin,
            "device_error_flags": flags,
            "c5_parabolic_kl": c5,
            "c3_fused_batch": c3,
            "other_path_stages": comps,
        }
        if c5_sharded is not None:
            out["c5_event_sharded"] = c5_sharded
        if world > 1:
            replicas = {"value": out["value"], "ms_per_step": out["ms_per_step"], "scaling": "weak",
                        "parallelism": "event-parallel x%d (each rank its own C4 event, no collective)" % world,
                        "seed_per_rank": "1000 * rank"}
            out["event_replicas"] = replicas
            out["rccl_world_size"] = dist.get_world_size()
            if sharded and "error" not in sharded:
                out["value"] = sharded["edges_per_s"]
                out["ms_per_step"] = sharded["ms_per_step"]
                out["config"]["parallelism"] = "edge-sharded x%d (one event, azimuthal wedges, halo all-to-all)" % world
                out["config"]["workload"] = "one pileup-200 TrackML-shaped event (configs[3]) across all GPUs"
                # per-GPU sizes of the headline: the largest owned range, the event's totals beside them
                out["config"]["nodes_per_gpu"] = sharded["owned_nodes_max"]
                out["config"]["directed_edges_per_gpu"] = sharded["owned_directed_edges_max"]
                out["config"]["event_nodes"] = sharded["nodes"]
                out["config"]["event_directed_edges"] = sharded["edges"]
                # the roofline of the headline: rank 0's kernels of the sharded pass (the replica
                # pass's roofline stays under event_replicas)
                replicas["roofline"] = out["roofline"]
                replicas["kernel_ms"] = out["kernel_ms"]
                out["roofline"] = sharded["roofline"]
                out["kernel_ms"] = sharded["roofline"]["kernel_ms_all"]
                # the N = 1 -> N speed-up of the single event: measured (this GPU's own one-event
                # pass, event_replicas, against the sharded step), compute only (the sharded
                # pass without its exchange), and DESIGN.md §6's projection from rank 0's
                # compute-only pass on one MI355X (profiles/r05/shard/shard_pass_time.log)
                proj = {2: 138.2 / 81.1, 4: 138.2 / 55.5, 8: 138.2 / 37.6}
                sharded["speedup_vs_one_gpu"] = {
                    "measured": replicas["ms_per_step"] / sharded["ms_per_step"],
                    "compute_only_this_run": replicas["ms_per_step"] / sharded["pass_ms_no_exchange"],
                    "projected_design": proj.get(world),
                    "projected_source": "DESIGN.md §6: rank 0's compute-only share of the C4 pass, N = 1 138.2 us, "
                                        "N = 2 / 4 / 8 81.1 / 55.5 / 37.6 us (profiles/r05/shard/)"}
                out["sharded_single_event"] = sharded
                if sharded["device_error_flags"]:
                    out["invalid"] = "sharded pass device_error_flags %d" % sharded["device_error_flags"]
            else:
                out["scaling"] = "weak"
                out["config"]["parallelism"] = replicas["parallelism"]
                out["sharded_error"] = (sharded or {}).get("error")
        if cpu:
            out["speedup_vs_cpu"] = out["value"] / cpu["value"]
        for k in (cpu_cpp or {}):
            if k.startswith("omp_threads_"):
                out["speedup_vs_cpp_" + k] = out["value"] / cpu_cpp[k]["value"]
        if flags:
            # the reference raises on this input (GTF_ERR_*): the timed pass has no reference answer
            out["invalid"] = "device_error_flags %d: the reference raises on this input" % flags
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    if flags and os.environ.get("GTF_BENCH_DIAG_BUILD", "0") != "1":   # (diagnostics builds with wrong results)
        sys.exit(3)


if __name__ == "__main__":
    main()
