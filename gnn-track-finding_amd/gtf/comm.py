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


_ID_MAGIC = b"GTFCOMM1"


def _parent_identity() -> str:
    """the launching parent process: its pid and its start time (field 22 of /proc/<pid>/stat,
    clock ticks since boot), so a recycled pid of a later launcher gives another identity"""
    ppid = os.getppid()
    try:
        with open("/proc/%d/stat" % ppid, "rb") as fh:
            stat = fh.read().decode(errors="replace")
        start = stat[stat.rindex(")") + 2:].split()[19]
    except (OSError, ValueError, IndexError):
        start = "?"
    return "%d@%s" % (ppid, start)


def job_token() -> str:
    """a token that names this launch of the job: GTF_COMM_JOB, else the launcher's run id
    (torchrun's TORCHELASTIC_RUN_ID when it is a real id -- torchrun's default static
    rendezvous sets the literal "none" --, Slurm's SLURM_JOB_ID.SLURM_STEP_ID), else the
    rendezvous address MASTER_ADDR:MASTER_PORT together with the identity of the launching
    parent process (pid and start time). The address alone does not tell two runs apart
    (consecutive runs reuse the default port 29500); the ranks of one launch on a node share
    their parent (torchrun's agent, bench.spawn_ranks), and a later launch has another one."""
    e = os.environ
    if e.get("GTF_COMM_JOB"):
        return e["GTF_COMM_JOB"]
    rid = e.get("TORCHELASTIC_RUN_ID", "")
    if rid and rid.lower() != "none":
        return "torchelastic:" + rid
    if e.get("SLURM_JOB_ID"):
        return "slurm:%s.%s" % (e["SLURM_JOB_ID"], e.get("SLURM_STEP_ID", ""))
    if e.get("MASTER_PORT"):
        return "rdzv:%s:%s:parent:%s" % (e.get("MASTER_ADDR", ""), e["MASTER_PORT"], _parent_identity())
    raise ValueError("NativeComm.from_file needs a job token: pass job=... or set GTF_COMM_JOB "
                     "(or run under a launcher that sets MASTER_PORT / TORCHELASTIC_RUN_ID)")


def write_id_file(path: str, uid: bytes, job: str) -> None:
    """the id file of this job: magic, the job token (length-prefixed), the unique id;
    written to a temporary name and renamed over `path`"""
    tok = job.encode()
    tmp = "%s.%d.tmp" % (path, os.getpid())
    with open(tmp, "wb") as fh:
        fh.write(_ID_MAGIC + len(tok).to_bytes(4, "little") + tok + uid)
    os.replace(tmp, path)


def read_id_file(path: str, job: str, timeout: float = 120.0) -> bytes:
    """wait until `path` holds THIS job's id (a stale file of another run -- other token --
    or a missing one is waited past), then return the unique id"""
    tok = job.encode()
    head = _ID_MAGIC + len(tok).to_bytes(4, "little") + tok
    t0 = time.monotonic()
    while True:
        try:
            with open(path, "rb") as fh:
                data = fh.read()
            if data.startswith(head) and len(data) == len(head) + nat.COMM_ID_BYTES:
                return data[len(head):]
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise TimeoutError("no RCCL unique id of job %r at %s after %.0f s (ranks launched by different "
                               "parents need a common GTF_COMM_JOB)" % (job, path, timeout))
        time.sleep(0.01)


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
    def from_file(cls, path: str, rank: int, world: int, timeout: float = 120.0, lib=None,
                  job: str | None = None) -> "NativeComm":
        """rank 0 writes the unique id to `path` (atomically: a temporary file renamed), the
        other ranks wait for it; every rank then joins. The file carries a job token
        (`job`, else :func:`job_token` from the launcher's environment) and a rank accepts
        only a file whose token is its own, so an id file left by an earlier run is never
        read as this run's"""
        job = job_token() if job is None else job
        if rank == 0:
            uid = unique_id(lib)
            write_id_file(path, uid, job)
        else:
            uid = read_id_file(path, job, timeout)
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
