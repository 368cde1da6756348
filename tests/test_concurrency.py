"""Concurrency: the namespace RW lock, journal group commit, and concurrent namespace mutations
whose journal replays to the same tree.

Reference tests: core/server/worker/src/test/java/alluxio/worker/block/ClientRWLockTest.java,
tests/src/test/java/alluxio/client/fs/concurrent/Concurrent{Create,Rename,Delete}IntegrationTest,
core/server/common/src/test/java/alluxio/master/journal/AsyncJournalWriterTest.java.
"""
import random
import threading
import time

import pytest

from alluxio_amd.conf import Configuration
from alluxio_amd.journal.system import AsyncJournalWriter
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.utils.exceptions import AlluxioStatusException
from alluxio_amd.utils.locks import RWLock


def test_rwlock_excludes_writers_from_readers():
    lock = RWLock()
    state = {"readers": 0, "writers": 0, "violations": 0, "reads": 0, "writes": 0}
    guard = threading.Lock()
    stop = time.monotonic() + 1.5

    def reader():
        while time.monotonic() < stop:
            with lock.read():
                with guard:
                    state["readers"] += 1
                    state["violations"] += state["writers"] != 0
                with lock.read():            # reentrant read, even with a writer queued
                    pass
                with guard:
                    state["readers"] -= 1
                    state["reads"] += 1

    def writer():
        while time.monotonic() < stop:
            with lock.write():
                with guard:
                    state["writers"] += 1
                    state["violations"] += state["readers"] != 0 or state["writers"] != 1
                with lock.read():            # the write holder may read
                    pass
                time.sleep(0.0002)
                with guard:
                    state["writers"] -= 1
                    state["writes"] += 1
            time.sleep(0.0005)
    ts = [threading.Thread(target=reader) for _ in range(6)] + [threading.Thread(target=writer) for _ in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(10)
    assert not any(t.is_alive() for t in ts), "deadlock"
    assert state["violations"] == 0
    assert state["reads"] > 100 and state["writes"] > 20
    assert lock.reader_count == 0 and not lock.is_write_locked


def test_rwlock_timeouts_and_writer_preference():
    lock = RWLock()
    lock.acquire_read()
    got = []
    t = threading.Thread(target=lambda: got.append(lock.acquire_write(timeout=0.1)))
    t.start()
    t.join()
    assert got == [False]                      # timed out behind the reader
    assert lock.acquire_read(timeout=0.1)      # gate reopened after the writer gave up
    lock.release_read()
    # a waiting writer blocks new readers (writer preference)
    w = threading.Thread(target=lambda: (lock.acquire_write(), time.sleep(0.2), lock.release_write()))
    w.start()
    time.sleep(0.05)
    other = []
    r = threading.Thread(target=lambda: other.append(lock.acquire_read(timeout=0.05)))
    r.start()
    r.join()
    assert other == [False]
    lock.release_read()
    w.join()
    assert lock.acquire_read(timeout=1)
    lock.release_read()


class _SlowWriter:
    def __init__(self):
        self.entries, self.flushes, self.closed = [], 0, False

    def write(self, e):
        self.entries.append(e)

    def flush(self):
        time.sleep(0.002)
        self.flushes += 1

    def close(self):
        self.closed = True


def test_journal_group_commit():
    w = _SlowWriter()
    aj = AsyncJournalWriter(w, batch_ms=5.0)
    n_threads, per = 16, 50

    def client(k):
        for i in range(per):
            c = aj.append((k, i))
            aj.flush(c)
    ts = [threading.Thread(target=client, args=(k,)) for k in range(n_threads)]
    t0 = time.monotonic()
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    elapsed = time.monotonic() - t0
    aj.close()
    assert len(w.entries) == n_threads * per
    for k in range(n_threads):                 # per-client order preserved
        assert [i for kk, i in w.entries if kk == k] == list(range(per))
    # batched: far fewer flushes than flush requests, and no fixed batch-window per request
    assert w.flushes < n_threads * per / 3
    assert elapsed < n_threads * per * 0.005 / 4


def test_concurrent_namespace_ops_replay(tmp_path):
    c = Configuration(load_site=False)
    c.set("alluxio.master.journal.type", "UFS")
    c.set("alluxio.master.journal.folder", str(tmp_path / "j"))
    c.set("alluxio.web.server.enabled", "false")
    m = AlluxioMasterProcess(c, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    fs = m.fs_master
    fs.create_directory("/c", write_type="MUST_CACHE")
    errors = []

    def worker(k):
        rnd = random.Random(k)
        for i in range(60):
            p = f"/c/t{k}_{i}"
            try:
                fs.create_file(p, write_type="MUST_CACHE")
                fs.complete_file(p)
                r = rnd.random()
                if r < 0.3:
                    fs.rename(p, p + ".r")
                elif r < 0.5:
                    fs.delete(p)
                elif r < 0.6:
                    fs.create_directory(f"/c/d{k}_{i}/x", recursive=True, write_type="MUST_CACHE")
            except AlluxioStatusException as e:
                errors.append(e)
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errors, errors[:3]
    live = sorted(i.name for i in fs.list_status("/c", recursive=True))
    m.stop()
    m = AlluxioMasterProcess(c, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    try:
        replayed = sorted(i.name for i in m.fs_master.list_status("/c", recursive=True, load_metadata="NEVER"))
        assert replayed == live and len(live) > 8 * 30
    finally:
        m.stop()
