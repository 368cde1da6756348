"""UFS absent-path cache (reference AsyncUfsAbsentPathCacheTest / UfsAbsentPathCache): repeated
lookups of missing paths stop touching the UFS; creation, loads, syncs and remounts invalidate."""
import os
import time

import pytest

from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.underfs.local import LocalUnderFileSystem
from alluxio_amd.utils import exceptions as ex


@pytest.fixture
def master(tmp_path):
    conf = Configuration({"alluxio.master.journal.folder": str(tmp_path / "journal"),
                          "alluxio.security.authorization.permission.enabled": "false"})
    m = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    m._ufs = str(tmp_path / "ufs")
    yield m
    m.stop()


def _count_ufs_status(monkeypatch):
    calls = [0]
    orig = LocalUnderFileSystem.get_status

    def counting(self, path):
        calls[0] += 1
        return orig(self, path)
    monkeypatch.setattr(LocalUnderFileSystem, "get_status", counting)
    return calls


def test_missing_paths_served_from_cache(master, monkeypatch):
    fs = master.fs_master
    calls = _count_ufs_status(monkeypatch)
    with pytest.raises(ex.FileDoesNotExistException):
        fs.get_status("/nope/deep/file")
    first = calls[0]
    assert first >= 1
    for _ in range(50):
        with pytest.raises(ex.FileDoesNotExistException):
            fs.get_status("/nope/deep/file")
        with pytest.raises(ex.FileDoesNotExistException):
            fs.list_status("/nope/deep/file")
    assert calls[0] == first                        # no further UFS round trips
    deadline = time.time() + 5                      # the async walk records the missing ancestor
    while fs.absent_cache.is_absent("/nope/other") is False and time.time() < deadline:
        time.sleep(0.01)
    assert fs.absent_cache.is_absent("/nope/other")  # a sibling under the missing directory
    # LoadMetadataType ALWAYS still asks the UFS
    with pytest.raises(ex.FileDoesNotExistException):
        fs.get_status("/nope/deep/file", load_metadata="ALWAYS")
    assert calls[0] > first


def test_creation_load_and_sync_invalidate(master):
    fs = master.fs_master
    for p in ("/a/x", "/b/y"):
        with pytest.raises(ex.FileDoesNotExistException):
            fs.get_status(p)
    assert fs.absent_cache.is_absent("/a/x")
    fs.create_file("/a/x", recursive=True, write_type="MUST_CACHE")   # creating drops the entry (and ancestors)
    assert not fs.absent_cache.is_absent("/a/x") and fs.get_status("/a/x").length == 0
    # the file appears in the UFS behind Alluxio's back: ONCE keeps answering from the cache,
    # a metadata sync of the parent re-reads it
    os.makedirs(os.path.join(master._ufs, "b"), exist_ok=True)
    with open(os.path.join(master._ufs, "b", "y"), "wb") as f:
        f.write(b"123")
    with pytest.raises(ex.FileDoesNotExistException):
        fs.get_status("/b/y")
    fs.sync_metadata("/b")
    assert fs.get_status("/b/y").length == 3


def test_remount_invalidates(master, tmp_path):
    fs = master.fs_master
    other = tmp_path / "other"
    (other / "d").mkdir(parents=True)
    with pytest.raises(ex.FileDoesNotExistException):
        fs.get_status("/mnt/d")
    assert fs.absent_cache.is_absent("/mnt/d")
    fs.mount("/mnt", str(other))
    assert not fs.absent_cache.is_absent("/mnt/d")           # another mount id now
    assert fs.get_status("/mnt/d").folder


def test_lru_capacity():
    from alluxio_amd.master.absent_cache import AsyncUfsAbsentPathCache

    class _Res:
        mount_id = 1

    class _MT:
        def resolve(self, p):
            return _Res()

    c = AsyncUfsAbsentPathCache(_MT(), capacity=3)
    for i in range(5):
        c.add_single_path(f"/p{i}")
    assert c.size() == 3 and not c.is_absent("/p0") and c.is_absent("/p4/child")
