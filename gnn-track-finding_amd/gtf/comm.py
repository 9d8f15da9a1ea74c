"""libgtf's own RCCL communicator (gtf_comm_*, csrc/gtf_comm.hip): the sharded event's
collectives without torch.distributed (SURVEY §8b ``gtf_comm_init``, §8e).

One communicator per rank, created with the rank's GPU current. Rank 0 makes the
GTF_COMM_ID_BYTES unique id (gtf_comm_unique_id) and hands it to the other ranks: through a
file on the node (:meth:`NativeComm.from_file`, no framework at all) or, in a process that
already runs torch.distributed, by a broadcast on that group (:meth:`NativeComm.from_torch`).
The halo all-to-all, the all-gather of owned states and the tag all-reduce(MAX) then run
inside libgtf on the caller's HIP stream (gtf.shard.ShardedDeviceGraph(backend="native")).
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

from . import _native as nat


def _prefer_loaded_rccl():
    """a process that holds PyTorch shares its RCCL with libgtf (one RCCL per process)"""
    if "GTF_RCCL" in os.environ or "torch" not in sys.modules:
        return
    import torch
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    if os.path.exists(p):
        os.environ["GTF_RCCL"] = p


def unique_id(lib=None) -> bytes:
    lib = lib or nat.lib(lean="torch" not in sys.modules)
    _prefer_loaded_rccl()
    buf = ctypes.create_string_buffer(nat.COMM_ID_BYTES)
    nat.check(lib.gtf_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
    return buf.raw


class NativeComm:
    def __init__(self, rank: int, world: int, uid: bytes, lib=None):
        if len(uid) != nat.COMM_ID_BYTES:
            raise ValueError("the RCCL unique id is %d bytes" % nat.COMM_ID_BYTES)
        self.lib = lib or nat.lib(lean="torch" not in sys.modules)
        _prefer_loaded_rccl()
        self.rank, self.world = int(rank), int(world)
        self.ptr = ctypes.c_void_p()
        idb = ctypes.create_string_buffer(uid, nat.COMM_ID_BYTES)
        nat.check(self.lib.gtf_comm_init(ctypes.byref(self.ptr), self.rank, self.world, ctypes.cast(idb, ctypes.c_void_p)))

    @classmethod
    def single(cls, lib=None) -> "NativeComm":
        """a world of one (the one-GPU box): every collective goes through RCCL all the same"""
        return cls(0, 1, unique_id(lib), lib)

    @classmethod
    def from_file(cls, path: str, rank: int, world: int, timeout: float = 120.0, lib=None) -> "NativeComm":
        """rank 0 writes the unique id to `path` (atomically: a temporary file renamed), the
        other ranks wait for it; every rank then joins"""
        if rank == 0:
            uid = unique_id(lib)
            tmp = "%s.%d.tmp" % (path, os.getpid())
            with open(tmp, "wb") as fh:
                fh.write(uid)
            os.replace(tmp, path)
        else:
            t0 = time.monotonic()
            while not os.path.exists(path):
                if time.monotonic() - t0 > timeout:
                    raise TimeoutError("no RCCL unique id at %s after %.0f s" % (path, timeout))
                time.sleep(0.01)
            with open(path, "rb") as fh:
                uid = fh.read()
        return cls(rank, world, uid, lib)

    @classmethod
    def from_torch(cls, group=None, lib=None) -> "NativeComm":
        """the id broadcast from rank 0 over an existing torch.distributed group"""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [unique_id(lib) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return cls(rank, world, obj[0], lib)

    def close(self):
        if self.ptr:
            nat.check(self.lib.gtf_comm_destroy(self.ptr))
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- collectives
    def allreduce_max_i64(self, buf, stream):
        nat.check(self.lib.gtf_allreduce_max_i64(self.ptr, ctypes.c_void_p(buf.data_ptr()), int(buf.numel()), stream))

    def allgather_bytes(self, chunk, out, stream):
        nat.check(self.lib.gtf_allgather_bytes(self.ptr, ctypes.c_void_p(chunk.data_ptr()),
                                               ctypes.c_void_p(out.data_ptr()), int(chunk.numel()), stream))
