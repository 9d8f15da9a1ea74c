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
    from gtf.comm import job_token
    for k in ("GTF_COMM_JOB", "TORCHELASTIC_RUN_ID", "SLURM_JOB_ID", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    with pytest.raises(ValueError):
        job_token()
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29500")
    assert job_token() == "rdzv:127.0.0.1:29500"
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "abc")
    assert job_token() == "torchelastic:abc"
    monkeypatch.setenv("GTF_COMM_JOB", "mine")
    assert job_token() == "mine"


def test_reader_times_out_on_wrong_job(tmp_path):
    from gtf.comm import read_id_file, write_id_file
    path = str(tmp_path / "uid")
    write_id_file(path, b"\x03" * 128, "other")
    with pytest.raises(TimeoutError):
        read_id_file(path, "mine", timeout=0.3)
    assert os.path.exists(path)
