"""The edge-sharded pass at full C4 size (BASELINE configs[3]): the benchmark
event (179,788 hits / 1,027,548 directed edges) cut into 2, 4 and 8 azimuthal wedges, one
rank per wedge, the ranks sharing the box's one GPU and exchanging the halo over gloo
(the N > 1 path of bench.py with RCCL replaced by gloo; the kernels and the exchange
lists are the same).

Two passes with the halo exchange between them, then sync(). Every rank's owned
receivers and slots must equal the one-GPU pass bit for bit after pass 1 and after
pass 2, and pass 1 (assembled from the ranks) must match the oracle digest
tests/golden/c4_digest.npz. World 8 is configs[3] itself ("edge-sharded across 8 x MI355X"):
the narrowest wedges, where the most senders straddle a cut. That keeps the reference's per-sender cumulative
``merged_cov[1,1] += var_ms`` (src/extrapolate/extrapolate_merged_states.py:127-128)
across wedge boundaries: a sender whose successors sit in several wedges is scanned
by every rank that owns one of them, each from the same halo copy of its state."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

OUT_NODE = ("has_merged", "merged_state", "merged_cov", "merged_prior", "has_uts", "degree")
OUT_SLOT = ("act", "edge_mw", "uts_rank", "uts_sv", "uts_tau", "uts_cov", "uts_xyzr", "uts_lik", "uts_mw",
            "uts_prior", "uts_lr", "uts_side", "tse_rank", "tse_prior", "tse_mw")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _save(path, h, nodes, slots, flags):
    arrs = {"nodes": nodes, "slots": slots, "flags": np.array(flags)}
    arrs.update({"n__" + f: h.node[f][nodes] for f in OUT_NODE})
    arrs.update({"s__" + f: h.slot[f][slots] for f in OUT_SLOT})
    np.savez(path, **arrs)


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    from gtf import synth
    from gtf.params import Params
    from gtf.shard import ShardedDeviceGraph
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = synth.workload("c4", seed=0)
    sd = ShardedDeviceGraph(g, rank, world, "cuda:0", backend="gloo")
    sd.d.clear_errors()
    p = Params()
    nodes, slots = sd.owned_host_nodes(), sd.owned_host_slots()
    for k in (1, 2):
        sd.step(p)
        torch.cuda.synchronize()
        h = sd.d.download(g.copy())
        _save(os.path.join(outdir, "w%d_r%d_p%d.npz" % (world, rank, k)), h, nodes, slots, sd.d.errors())
    sd.sync()
    torch.cuda.synchronize()
    h = sd.d.download(g.copy())
    np.savez(os.path.join(outdir, "w%d_r%d_sync.npz" % (world, rank)), act=h.slot["act"],
             has_merged=h.node["has_merged"], merged_state=h.node["merged_state"], merged_cov=h.node["merged_cov"],
             halo_bytes=np.array(sd.halo_bytes))
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def single_gpu():
    """the one-GPU pass (bench layout) after pass 1 and pass 2, host order"""
    from gtf import synth
    from gtf.device import DeviceGraph
    from gtf.params import Params
    g = synth.workload("c4", seed=0)
    d = DeviceGraph(g, layout="tiled")
    d.clear_errors()
    outs = []
    for _ in range(2):
        d.full_pass(Params())
        outs.append(d.download(g.copy()))
    assert d.errors() == 0
    return g, outs


@pytest.mark.parametrize("world,fused_1b", [(2, "0"), (4, "0"), (8, "0"), (8, "1")])
def test_sharded_c4_equals_single_gpu_and_digest(world, fused_1b, single_gpu, tmp_path, monkeypatch):
    """fused_1b: phase 1b as one sender-major launch (GTF_SHARD_FUSED_1B, gtf_shard.phases bit 4),
    inherited by the spawned ranks"""
    monkeypatch.setenv("GTF_SHARD_FUSED_1B", fused_1b)
    import torch.multiprocessing as mp
    from test_gpu_c4_digest import _digest, digest_errors
    g, ref = single_gpu
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(110 + 25 * world)   # (8 ranks build and upload the event side by side)
    for p in ps:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    for k in (1, 2):
        asm = ref[k - 1].copy()    # pass-k output assembled from the ranks' owned parts
        seen_n = np.zeros(g.n_nodes, bool)
        seen_s = np.zeros(g.n_slots, bool)
        for r in range(world):
            z = np.load(os.path.join(tmp_path, "w%d_r%d_p%d.npz" % (world, r, k)))
            nodes, slots = z["nodes"], z["slots"]
            assert int(z["flags"]) == 0, (r, k)
            assert not seen_n[nodes].any() and not seen_s[slots].any()
            seen_n[nodes] = True
            seen_s[slots] = True
            for f in OUT_NODE:
                a, b = z["n__" + f], ref[k - 1].node[f][nodes]
                assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), (world, r, k, f)
                asm.node[f][nodes] = a
            for f in OUT_SLOT:
                a, b = z["s__" + f], ref[k - 1].slot[f][slots]
                bad = np.nonzero(~((a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else a == b))[0]
                assert bad.size == 0, (world, r, k, f, bad.size)
                asm.slot[f][slots] = a
        assert seen_n.all() and seen_s.all()
        if k == 1:
            errs, diff_und = digest_errors(asm, _digest())
            assert errs == [], "\n".join(errs)
    # after sync() every replica holds every rank's published state
    for r in range(world):
        z = np.load(os.path.join(tmp_path, "w%d_r%d_sync.npz" % (world, r)))
        assert int(z["halo_bytes"]) > 0
        assert np.array_equal(z["act"], ref[1].slot["act"]), r
        for f in ("has_merged", "merged_state", "merged_cov"):
            assert np.array_equal(z[f], ref[1].node[f], equal_nan=True), (r, f)
