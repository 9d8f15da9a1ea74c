"""Tag propagation on an edge-sharded event ("per sweep allReduce(max) of the
tags + the flip count"): every rank sweeps its owned wedge of nodes
(gtf_tag_sweep_shard) and one all-reduce(MAX) per sweep completes every replica. The
ranks share the box's one GPU and reduce over gloo (bench.py's N > 1 path with RCCL
replaced by gloo; the kernels and the buffer protocol are the same).

Bar: the tags and the flip count of every sweep equal the one-GPU stage
(DeviceGraph.tag_propagation) bit for bit on every rank, and on the volume-7 fixture the
reference's own tags and flip vector [6606, 4749, 3194, 1857, 825, 102]
(tag_propagation/tag_propagation.py:97-164, tests/golden/make_golden.py)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _graph(which):
    if which == "vol7":
        from fixtures import load
        g, _, _, _ = load("tags_vol7")
        return g, g.node["tag"].astype(np.int64), g.node["xyzr"][:, 3]
    from gtf import synth
    g = synth.workload("c4", seed=0)
    return g, np.arange(g.n_nodes, dtype=np.int64), g.node["xyzr"][:, 3]


def _worker(rank, world, port, which, outdir, backend="gloo"):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import torch
    import torch.distributed as dist
    from gtf.shard import ShardedDeviceGraph
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda:0"))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    g, tags, radius = _graph(which)
    sd = ShardedDeviceGraph(g, rank, world, "cuda:0", backend=backend, tile=512)
    # C4: sweep to convergence (the reference's 10 % stop ends after one sweep there)
    out, flips = sd.tag_propagation(tags, radius, threshold=0.1 if which == "vol7" else 0.0)
    np.savez(os.path.join(outdir, "%s_w%d_r%d.npz" % (which, world, rank)), tags=out, flips=np.array(flips))
    dist.barrier()
    dist.destroy_process_group()


def _run(which, world, tmp_path, backend="gloo"):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, which, str(tmp_path), backend)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(110 + 25 * world)
    for p in ps:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    return [np.load(os.path.join(tmp_path, "%s_w%d_r%d.npz" % (which, world, r))) for r in range(world)]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_tags_vol7_equal_reference(world, tmp_path):
    from fixtures import load
    from gtf.device import DeviceGraph
    g, _, extra, _ = load("tags_vol7")
    one, one_flips = DeviceGraph(g).tag_propagation(g.node["tag"], g.node["xyzr"][:, 3])
    kept = extra["tags"] >= 0
    for z in _run("vol7", world, tmp_path):
        assert list(z["flips"]) == list(extra["flips"]) == list(one_flips)
        assert np.array_equal(z["tags"], one)
        assert np.array_equal(z["tags"][kept], extra["tags"][kept])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_tags_c4_equal_single_gpu(world, tmp_path):
    from gtf.device import DeviceGraph
    g, tags, radius = _graph("c4")
    one, one_flips = DeviceGraph(g, layout="tiled").tag_propagation(tags, radius, threshold=0.0)
    assert len(one_flips) > 2 and one_flips[-1] == 0
    for z in _run("c4", world, tmp_path):
        assert list(z["flips"]) == list(one_flips)
        assert np.array_equal(z["tags"], one)


def test_sharded_tags_vol7_rccl_world1(tmp_path):
    """the RCCL all-reduce(MAX) path of the sweep exchange (one rank: the box has one GPU)"""
    from fixtures import load
    g, _, extra, _ = load("tags_vol7")
    kept = extra["tags"] >= 0
    (z,) = _run("vol7", 1, tmp_path, backend="nccl")
    assert list(z["flips"]) == list(extra["flips"])
    assert np.array_equal(z["tags"][kept], extra["tags"][kept])
