"""libgtf's own RCCL communicator (gtf_comm_*, csrc/gtf_comm.hip; SURVEY §8b gtf_comm_init):
the sharded event driven through libgtf's collectives with no torch.distributed process
group -- the halo exchange (gtf_halo_exchange), the all-gather of owned states
(gtf_allgather_bytes) and the sharded tag propagation (gtf_tag_propagate_shard, one
all-reduce(MAX) per sweep). The box has one GPU, so the world is one rank; every collective
still runs through RCCL.

Bar: bit-equal to the one-GPU pass after two passes (and the tags / flip vector to the
reference's vol-7 run, tag_propagation/tag_propagation.py:97-164)."""
import numpy as np
import pytest

from compare import compare
from fixtures import load

pytestmark = pytest.mark.gpu


def test_native_comm_world1_pass_equals_single_gpu():
    import torch.distributed as dist
    from gtf import synth
    from gtf.comm import NativeComm
    from gtf.device import DeviceGraph
    from gtf.params import Params
    from gtf.shard import ShardedDeviceGraph
    assert not (dist.is_available() and dist.is_initialized())
    g = synth.workload("c2", seed=3)
    p = Params()
    comm = NativeComm.single()
    assert comm.world == 1 and comm.rank == 0
    sd = ShardedDeviceGraph(g, 0, 1, "cuda:0", backend="native", comm=comm)
    one = DeviceGraph(g, layout="tiled")
    for d in (sd.d, one):
        d.clear_errors()
    for _ in range(2):
        sd.step(p)                 # pass + gtf_halo_exchange (pack, RCCL group, unpack)
        one.full_pass(p)
    sd.sync()                      # gtf_shard_pack + gtf_allgather_bytes + unpack
    a, b = sd.d.download(g.copy()), one.download(g.copy())
    assert sd.d.errors() == 0 and one.errors() == 0
    errs = compare(a, b, rtol=0.0, atol=0.0)
    assert errs == [], "\n".join(errs)
    comm.close()


def test_native_comm_world1_tags_equal_reference():
    from gtf.comm import NativeComm
    from gtf.shard import ShardedDeviceGraph
    g, _, extra, _ = load("tags_vol7")
    comm = NativeComm.single()
    sd = ShardedDeviceGraph(g, 0, 1, "cuda:0", backend="native", comm=comm, tile=512)
    tags, flips = sd.tag_propagation(g.node["tag"].astype(np.int64), g.node["xyzr"][:, 3])
    assert list(flips) == list(extra["flips"])
    kept = extra["tags"] >= 0
    assert np.array_equal(tags[kept], extra["tags"][kept])
    comm.close()


def test_native_comm_id_through_a_file(tmp_path):
    """the framework-free id hand-off (rank 0 writes, the others read): one rank here"""
    from gtf.comm import NativeComm
    from gtf.comm import read_id_file
    comm = NativeComm.from_file(str(tmp_path / "uid"), 0, 1, job="test-job")
    assert len(read_id_file(str(tmp_path / "uid"), "test-job", timeout=1.0)) == 128
    comm.close()
