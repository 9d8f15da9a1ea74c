"""The RCCL id hand-off through a file (gtf.comm.NativeComm.from_file): a rank
other than 0 must never take an id file left by an earlier run. Two processes, no GPU:
rank 0's writer and a reader of the same path, with a stale file of another job present
when the reader starts."""
import multiprocessing as mp
import os
import time

import pytest


def _reader(path, job, q):
    from gtf.comm import read_id_file
    try:
        q.put(read_id_file(path, job, timeout=30.0))
    except Exception as ex:   # reported to the parent
        q.put(repr(ex))


def test_stale_id_file_is_not_read(tmp_path):
    from gtf.comm import write_id_file
    path = str(tmp_path / "uid")
    old, new = b"\x01" * 128, b"\x02" * 128
    write_id_file(path, old, "rdzv:127.0.0.1:1111")          # an earlier run's file
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_reader, args=(path, "rdzv:127.0.0.1:2222", q))
    p.start()
    time.sleep(1.0)            # the reader is polling, the stale file in place
    assert q.empty()
    write_id_file(path, new, "rdzv:127.0.0.1:2222")          # rank 0 of this run
    got = q.get(timeout=30)
    p.join(30)
    assert got == new


def test_job_token_from_environment(monkeypatch):
    from gtf.comm import _parent_identity, job_token
    for k in ("GTF_COMM_JOB", "TORCHELASTIC_RUN_ID", "SLURM_JOB_ID", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    with pytest.raises(ValueError):
        job_token()
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29500")
    assert job_token() == "rdzv:127.0.0.1:29500:parent:" + _parent_identity()
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")   # torchrun's static rendezvous: not an id
    assert job_token().startswith("rdzv:127.0.0.1:29500:parent:")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "abc")
    assert job_token() == "torchelastic:abc"
    monkeypatch.setenv("GTF_COMM_JOB", "mine")
    assert job_token() == "mine"


def _token_of_child(q):
    from gtf.comm import job_token
    q.put(job_token())


def _launch(q):
    """a launcher: its own ranks (children) share its identity"""
    ctx = mp.get_context("spawn")
    q2 = ctx.Queue()
    kids = [ctx.Process(target=_token_of_child, args=(q2,)) for _ in range(2)]
    for k in kids:
        k.start()
    toks = [q2.get(timeout=60) for _ in kids]
    for k in kids:
        k.join(30)
    q.put(toks)


def test_default_token_differs_between_launches(monkeypatch):
    """two launches with the same default rendezvous (torchrun's TORCHELASTIC_RUN_ID "none",
    the same MASTER_ADDR:MASTER_PORT): the ranks of one launch agree on the token, the next
    launch's ranks get another one, so they never take the earlier launch's id file"""
    for k in ("GTF_COMM_JOB", "SLURM_JOB_ID"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29500")
    ctx = mp.get_context("spawn")
    runs = []
    for _ in range(2):
        q = ctx.Queue()
        p = ctx.Process(target=_launch, args=(q,))
        p.start()
        runs.append(q.get(timeout=120))
        p.join(30)
    assert runs[0][0] == runs[0][1] and runs[1][0] == runs[1][1]
    assert runs[0][0] != runs[1][0]


def test_reader_times_out_on_wrong_job(tmp_path):
    from gtf.comm import read_id_file, write_id_file
    path = str(tmp_path / "uid")
    write_id_file(path, b"\x03" * 128, "other")
    with pytest.raises(TimeoutError):
        read_id_file(path, "mine", timeout=0.3)
    assert os.path.exists(path)
