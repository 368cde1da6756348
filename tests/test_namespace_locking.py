"""Namespace locking: UFS I/O runs under path-scoped locks, never under the tree-wide lock.

Parity: core/server/master/src/main/java/alluxio/master/file/meta/InodeLockManager.java,
LockedInodePath.java, InodeTree.java:99-111 (lock patterns), and the fault-injection fake
tests/src/test/java/alluxio/testutils/underfs/sleeping/SleepingUnderFileSystem.java: a slow UFS
operation on one subtree must not stall metadata operations on other subtrees.
"""
import os
import statistics
import threading
import time

import pytest

from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.conf import Configuration
from alluxio_amd.master.inode_lock import (IR, IW, R, W, PathLockManager, WouldBlock, check_may_block,
                                           nonblocking_lane)
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.utils.exceptions import DeadlineExceededException, FileDoesNotExistException


# ---- lock manager ----------------------------------------------------------------------------
def _try(mgr, reqs, timeout=0.05):
    """True when ``reqs`` can be acquired by ANOTHER thread within ``timeout``."""
    out = {}

    def run():
        try:
            mgr.lock(reqs, timeout_s=timeout).close()
            out["ok"] = True
        except DeadlineExceededException:
            out["ok"] = False
    t = threading.Thread(target=run)
    t.start()
    t.join()
    return out["ok"]


def test_lock_compatibility_matrix():
    m = PathLockManager()
    with m.lock([("/a/b", W)]):
        assert m.held_paths() == {"/": [IW], "/a": [IW], "/a/b": [W]}
        assert _try(m, [("/a/c", W)])           # sibling: IW/IW on /a
        assert not _try(m, [("/a/b/x", W)])     # below the W
        assert not _try(m, [("/a", W)])         # W above vs IW
        assert not _try(m, [("/a/b", R)])
        assert not _try(m, [("/a", R)])         # R vs IW
        assert _try(m, [("/z", R)])
    with m.lock([("/a", R)]):
        assert _try(m, [("/a/b", R)])           # readers share
        assert not _try(m, [("/a/b", W)])       # IW on /a vs R
    assert m.held_paths() == {}


def test_lock_list_is_atomic_and_reentrant():
    m = PathLockManager()
    with m.lock([("/s", W), ("/d/x", W)]):
        # the same thread may lock inside its own subtree (a mutation calling another)
        with m.lock([("/s/child", W)]):
            pass
        assert not _try(m, [("/d", W)])
        assert not _try(m, [("/s/q", W)])
    # all-or-nothing: a list that conflicts on one path acquires none of them
    with m.lock([("/x", W)]):
        res = {}

        def other():
            try:
                m.lock([("/y", W), ("/x/k", W)], timeout_s=0.05)
            except DeadlineExceededException:
                res["held"] = m.held_paths()
        t = threading.Thread(target=other)
        t.start()
        t.join()
        assert "/y" not in res["held"]


def test_nonblocking_lane_raises_instead_of_waiting():
    m = PathLockManager()
    with m.lock([("/a", W)]):
        out = {}

        def lane():
            with nonblocking_lane():
                try:
                    m.lock([("/a/b", W)])
                except WouldBlock:
                    out["spilled"] = True
                try:
                    check_may_block("ufs")
                except WouldBlock:
                    out["ufs"] = True
            check_may_block("ufs")                   # off the lane: fine
            out["after"] = True
        t = threading.Thread(target=lane)
        t.start()
        t.join()
    assert out == {"spilled": True, "ufs": True, "after": True}


# ---- master with a slow UFS ------------------------------------------------------------------
@pytest.fixture
def master(tmp_path):
    conf = Configuration({"alluxio.master.journal.folder": str(tmp_path / "journal"),
                          "alluxio.master.journal.type": "UFS",
                          "alluxio.security.authorization.permission.enabled": "false",
                          "alluxio.user.metadata.cache.enabled": "false"})
    m = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    yield m
    m.stop()


def _mount_slow(m, tmp_path, ms=1000):
    slow = tmp_path / "slow_ufs"
    (slow / "dir").mkdir(parents=True)
    for i in range(2):
        (slow / "dir" / f"f{i}").write_bytes(b"x" * 10)
    (slow / "mv").mkdir()
    (slow / "mv" / "g").write_bytes(b"y")
    m.fs_master.mount("/slow", f"sleepfs://{slow}", properties={
        "alluxio.underfs.sleep.delete_file.ms": str(ms), "alluxio.underfs.sleep.delete_directory.ms": str(ms),
        "alluxio.underfs.sleep.rename_directory.ms": str(ms), "alluxio.underfs.sleep.rename_file.ms": str(ms),
        "alluxio.underfs.sleep.mkdirs.ms": str(ms)})
    m.fs_master.load_metadata("/slow", recursive=True)
    return slow


def _timed(fn):
    t = time.perf_counter()
    fn()
    return time.perf_counter() - t


def test_slow_ufs_delete_and_rename_do_not_stall_other_paths(master, tmp_path):
    """A 3 s UFS delete (2 files + dir, 1 s each) and a 1 s UFS rename run while clients create,
    stat and list unrelated paths through the native RPC front end: those stay fast.  Operations
    inside the deleting subtree see the namespace as of before the delete (reads) or wait for it
    (a create below it), and fail cleanly once it is gone."""
    fsm = master.fs_master
    slow = _mount_slow(master, tmp_path)
    fs = FileSystem(conf=Configuration({"alluxio.user.metadata.cache.enabled": "false",
                                        "alluxio.user.network.inprocess.transport.enabled": "false"}),
                    master_address=master.address)
    fs.create_directory("/other", allow_exists=True)
    errors = []

    def bg(fn):
        def run():
            try:
                fn()
            except Exception as e:  # noqa: BLE001
                errors.append(e)
        t = threading.Thread(target=run)
        t.start()
        return t

    t_del = bg(lambda: fs.delete("/slow/dir", recursive=True))
    t_mv = bg(lambda: fs.rename("/slow/mv", "/slow/mv2"))
    time.sleep(0.2)                      # both are now inside their UFS calls
    lat = []
    t_end = time.perf_counter() + 1.5
    i = 0
    while time.perf_counter() < t_end:
        lat.append(_timed(lambda: fs.create_file(f"/other/f{i}").close()))
        lat.append(_timed(lambda: fs.get_status(f"/other/f{i}")))
        lat.append(_timed(lambda: fs.list_status("/other")))
        lat.append(_timed(lambda: fs.get_status("/slow/dir/f0")))    # pre-delete state, no wait
        i += 1
    assert t_del.is_alive(), "the slow delete should still be running"
    # a blocked op would take the full 3 s of UFS sleeps; allow scheduler noise on a busy box
    p95 = sorted(lat)[int(0.95 * (len(lat) - 1))]
    assert max(lat) < 1.0 and p95 < 0.05 and statistics.median(lat) < 0.02, (max(lat), p95, statistics.median(lat))
    # a create inside the subtree being deleted waits for the delete and then fails
    t0 = time.perf_counter()
    with pytest.raises(FileDoesNotExistException):
        fsm.create_file("/slow/dir/new")
    assert time.perf_counter() - t0 > 0.3
    t_del.join(timeout=10)
    t_mv.join()
    assert not errors, errors
    assert not os.path.exists(slow / "dir") and os.path.exists(slow / "mv2" / "g")
    assert fs.exists("/slow/mv2/g") and not fs.exists("/slow/dir", load_metadata="NEVER")
    assert master.native_rpc is not None and master.native_rpc.spilled >= 2   # Remove/Rename left the lane
    fs.close()


def test_recursive_delete_of_10k_persisted_files_does_not_block(master, tmp_path):
    fsm = master.fs_master
    root = tmp_path / "ufs" / "big"
    for d in range(10):
        sub = root / f"d{d}"
        sub.mkdir(parents=True)
        for i in range(1000):
            (sub / f"f{i}").write_bytes(b"")
    fsm.load_metadata("/big", recursive=True)
    assert fsm.total_paths() >= 10_011
    fsm.create_directory("/live")
    lat = []
    done = threading.Event()

    def deleter():
        fsm.delete("/big", recursive=True)
        done.set()
    t = threading.Thread(target=deleter)
    t0 = time.perf_counter()
    t.start()
    i = 0
    while not done.is_set():
        lat.append(_timed(lambda: fsm.create_file(f"/live/f{i}")))
        lat.append(_timed(lambda: fsm.get_status(f"/live/f{i}")))
        i += 1
    t.join()
    took = time.perf_counter() - t0
    assert not os.path.exists(root)
    p95 = sorted(lat)[int(0.95 * (len(lat) - 1))]
    assert max(lat) < 1.0 and p95 < 0.1, (max(lat), p95, took, len(lat))
    assert len(lat) >= 20, (len(lat), took)        # the namespace kept serving during the delete
    with pytest.raises(FileDoesNotExistException):
        fsm.get_status("/big", load_metadata="NEVER")


def test_failed_ufs_delete_keeps_failed_path_and_ancestors(master, tmp_path):
    """A UFS delete failure deletes what it could and keeps the failed inode and its ancestors
    (reference DeleteContext / UfsDeleter: 'failed to delete' paths stay)."""
    from alluxio_amd.underfs import testing
    from alluxio_amd.utils.exceptions import UnavailableException
    fsm = master.fs_master
    ufs = tmp_path / "ufs"
    (ufs / "p" / "ok").mkdir(parents=True)
    (ufs / "p" / "ok" / "a").write_bytes(b"1")
    (ufs / "p" / "bad").mkdir()
    (ufs / "p" / "bad" / "b").write_bytes(b"2")
    fsm.load_metadata("/p", recursive=True)
    res = fsm._resolve_ufs("/p/bad/b")
    orig = res.ufs.delete_file

    def delete_file(path):
        if path.endswith("/bad/b"):
            raise OSError("injected")
        return orig(path)
    res.ufs.delete_file = delete_file
    try:
        with pytest.raises(UnavailableException):
            fsm.delete("/p", recursive=True)
    finally:
        res.ufs.delete_file = orig
    names = sorted(i.path for i in fsm.list_status("/p", recursive=True, load_metadata="NEVER"))
    assert names == ["/p/bad", "/p/bad/b"]
    assert not (ufs / "p" / "ok").exists() and (ufs / "p" / "bad" / "b").exists()
    del testing


def test_block_removal_waits_for_durable_delete(master):
    """Group-committed (deferred) RPC: the blocks of a deleted file are queued for worker
    removal only after the DeleteFile entry is durable, and never when the flush fails
    (RpcContext.close ordering)."""
    from alluxio_amd.journal.system import deferred_flush
    fsm = master.fs_master
    calls = []
    orig = fsm.block_master.remove_blocks
    fsm.block_master.remove_blocks = lambda ids, delete: calls.append((list(ids), delete))
    try:
        fsm.create_file("/x")
        fsm.get_new_block_id_for_file("/x")
        with deferred_flush() as d:
            fsm.delete("/x")
            assert d.pending and len(d.after) == 1 and calls == []    # nothing queued yet
        # the front end runs the callbacks once the flush landed
        for cb in d.after:
            cb()
        assert len(calls) == 1 and calls[0][1] is True
    finally:
        fsm.block_master.remove_blocks = orig
