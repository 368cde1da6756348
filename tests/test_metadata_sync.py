"""Parallel metadata sync (master/sync.py: InodeSyncStream + UfsStatusCache).

Parity: core/server/master/src/test/java/alluxio/master/file/FileSystemMasterSyncMetadataTest.java
(sync adds / removes / reloads changed files, recursive and not) and UfsStatusCacheTest (listing
prefetch, statuses from the parent listing, joined in-flight fetches).  The latency test stands in
for an object store: every UFS list/status call sleeps, and a wide tree must sync in far less than
the serial sum of its round trips.
"""
import os
import threading
import time

import pytest

from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.master.sync import UfsStatusCache
from alluxio_amd.underfs.local import LocalUnderFileSystem


@pytest.fixture
def master(tmp_path):
    conf = Configuration({"alluxio.master.journal.folder": str(tmp_path / "journal"),
                          "alluxio.security.authorization.permission.enabled": "false",
                          "alluxio.master.metadata.sync.concurrency.level": "16",
                          "alluxio.master.metadata.sync.ufs.prefetch.pool.size": "16",
                          "alluxio.master.metadata.sync.executor.pool.size": "8"})
    m = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    m._ufs = str(tmp_path / "ufs")
    yield m
    m.stop()


def _mk(root, rel, data=b"x"):
    p = os.path.join(root, rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "wb") as f:
        f.write(data)


def _paths(fs, path):
    return sorted(i.path for i in fs.list_status(path, recursive=True, load_metadata="NEVER"))


def test_sync_adds_removes_and_reloads(master):
    fs, ufs = master.fs_master, master._ufs
    for rel in ("s/a", "s/d1/b", "s/d1/d2/c", "s/d3/e"):
        _mk(ufs, rel)
    st = fs.sync_metadata("/s")
    assert st["added"] >= 1
    assert _paths(fs, "/s") == ["/s/a", "/s/d1", "/s/d1/b", "/s/d1/d2", "/s/d1/d2/c", "/s/d3", "/s/d3/e"]
    # external changes: delete a file and a directory, add nested entries, rewrite a file
    os.remove(os.path.join(ufs, "s/a"))
    import shutil
    shutil.rmtree(os.path.join(ufs, "s/d3"))
    _mk(ufs, "s/d1/d2/new/deep")
    time.sleep(0.01)
    _mk(ufs, "s/d1/b", b"changed-content")
    st = fs.sync_metadata("/s")
    assert st["removed"] == 2 and st["updated"] == 1 and st["added"] >= 1
    assert _paths(fs, "/s") == ["/s/d1", "/s/d1/b", "/s/d1/d2", "/s/d1/d2/c", "/s/d1/d2/new",
                                "/s/d1/d2/new/deep"]
    assert fs.get_status("/s/d1/b", load_metadata="NEVER").length == len(b"changed-content")
    assert fs.check_consistency("/s") == []
    # nothing changed: a second sync is a no-op and takes its child statuses from the listings
    st = fs.sync_metadata("/s")
    assert (st["added"], st["removed"], st["updated"]) == (0, 0, 0)
    assert st["ufs_status_calls"] == 1          # only the sync root; children come from listings


def test_non_recursive_sync_stays_at_one_level(master):
    fs, ufs = master.fs_master, master._ufs
    _mk(ufs, "n/top")
    _mk(ufs, "n/sub/inner")
    fs.sync_metadata("/n", recursive=True)
    _mk(ufs, "n/top2")
    _mk(ufs, "n/sub/inner2")
    st = fs.sync_metadata("/n", recursive=False)
    assert st["added"] == 1
    names = _paths(fs, "/n")
    assert "/n/top2" in names and "/n/sub/inner2" not in names


def test_wide_tree_sync_overlaps_ufs_latency(master, monkeypatch):
    fs, ufs = master.fs_master, master._ufs
    width = 24
    for i in range(width):
        _mk(ufs, f"w/d{i}/f")
    delay = 0.03
    inflight, peak = [0], [0]
    lock = threading.Lock()
    tls = threading.local()                     # local list_status calls get_status per entry:
    orig_list, orig_status = LocalUnderFileSystem.list_status, LocalUnderFileSystem.get_status

    def slow(fn):
        def wrapper(self, *a, **k):
            if getattr(tls, "inside", False):   # only the outer call is one "round trip"
                return fn(self, *a, **k)
            tls.inside = True
            with lock:
                inflight[0] += 1
                peak[0] = max(peak[0], inflight[0])
            try:
                time.sleep(delay)
                return fn(self, *a, **k)
            finally:
                tls.inside = False
                with lock:
                    inflight[0] -= 1
        return wrapper
    monkeypatch.setattr(LocalUnderFileSystem, "list_status", slow(orig_list))
    monkeypatch.setattr(LocalUnderFileSystem, "get_status", slow(orig_status))
    t0 = time.perf_counter()
    st = fs.sync_metadata("/w")
    dt = time.perf_counter() - t0
    assert len(_paths(fs, "/w")) == 2 * width
    calls = st["ufs_list_calls"] + st["ufs_status_calls"]
    assert calls >= width                        # one listing per directory at least
    assert peak[0] >= 4                          # listings really overlapped
    assert dt < 0.5 * calls * delay, (dt, calls)


def test_recursive_load_metadata_prefetches(master, monkeypatch):
    fs, ufs = master.fs_master, master._ufs
    for i in range(8):
        _mk(ufs, f"r/d{i}/x/f")
    fs.load_metadata("/r", recursive=True)
    assert len(_paths(fs, "/r")) == 8 * 3


def test_status_cache_joins_prefetch_and_fills_child_statuses():
    import concurrent.futures as cf
    from alluxio_amd.underfs.base import UfsDirectoryStatus, UfsFileStatus
    calls = {"list": 0, "status": 0}
    gate = threading.Event()

    def fetch_list(p):
        calls["list"] += 1
        gate.wait(5)
        return [UfsFileStatus("a", 3), UfsDirectoryStatus("b")]

    def fetch_status(p):
        calls["status"] += 1
        return None
    with cf.ThreadPoolExecutor(2) as pool:
        c = UfsStatusCache(fetch_list, fetch_status, pool)
        c.prefetch_children("/d")
        c.prefetch_children("/d")                 # deduplicated while in flight
        gate.set()
        got = c.fetch_children("/d")              # joins the in-flight listing
        assert [s.name for s in got] == ["a", "b"] and calls["list"] == 1
        assert c.get_status("/d/a").content_length == 3 and c.get_status("/d/b").is_directory
        assert calls["status"] == 0
        assert c.get_status("/d/zz") is None and calls["status"] == 1
