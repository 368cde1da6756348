"""File-system / block / meta master behaviour (reference FileSystemMasterTest, InodeTreeTest,
BlockMasterTest, MountTableTest): in-process masters over a temp UFS journal, no workers."""
import os
import time

import pytest

from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.proto import pb
from alluxio_amd.utils import exceptions as ex
from alluxio_amd.utils import ids


@pytest.fixture
def master(tmp_path):
    conf = Configuration({"alluxio.master.journal.folder": str(tmp_path / "journal"),
                          "alluxio.security.authorization.permission.enabled": "false"})
    m = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    m._tmp = tmp_path
    yield m
    m.stop()


def test_create_list_delete(master):
    fs = master.fs_master
    fs.create_directory("/a/b/c", recursive=True)
    with pytest.raises(ex.FileAlreadyExistsException):
        fs.create_directory("/a/b")
    fs.create_directory("/a/b", allow_exists=True)
    with pytest.raises(ex.FileDoesNotExistException):
        fs.create_directory("/x/y")
    fi = fs.create_file("/a/f1", block_size=1024, write_type="MUST_CACHE")
    assert ids.get_sequence_number(fi.fileId) == (1 << 24) - 1
    assert [i.path for i in fs.list_status("/a")] == ["/a/b", "/a/f1"]
    assert sorted(i.path for i in fs.list_status("/", recursive=True)) == ["/a", "/a/b", "/a/b/c", "/a/f1"]
    with pytest.raises(ex.DirectoryNotEmptyException):
        fs.delete("/a")
    fs.delete("/a", recursive=True)
    assert fs.list_status("/") == []


def test_block_ids_and_complete(master):
    fs, bm = master.fs_master, master.block_master
    fi = fs.create_file("/f", block_size=100, write_type="MUST_CACHE")
    b0 = fs.get_new_block_id_for_file("/f")
    b1 = fs.get_new_block_id_for_file("/f")
    assert ids.get_file_id(b0) == fi.fileId and ids.get_sequence_number(b1) == 1
    with pytest.raises(ex.FailedPreconditionException):
        fs.complete_file("/f")  # blocks not committed
    wid = bm.get_worker_id(pb.grpc.WorkerNetAddress(host="w1", rpcPort=1, dataPort=1))
    bm.worker_register(wid, ["MEM"], {"MEM": 10_000}, {"MEM": 0}, {})
    bm.commit_block(wid, 100, "MEM", "HBM", b0, 100)
    bm.commit_block(wid, 150, "MEM", "HBM", b1, 50)
    fs.complete_file("/f")
    st = fs.get_status("/f")
    assert st.completed and st.length == 150 and list(st.blockIds) == [b0, b1]
    assert st.inAlluxioPercentage == 100 and st.inMemoryPercentage == 100
    assert st.fileBlockInfos[1].offset == 100
    assert st.fileBlockInfos[0].blockInfo.locations[0].workerAddress.host == "w1"
    with pytest.raises(ex.FailedPreconditionException):
        fs.complete_file("/f")


def test_rename_semantics(master, tmp_path):
    fs = master.fs_master
    fs.create_directory("/d1/sub", recursive=True, write_type="CACHE_THROUGH")
    fs.create_file("/d1/sub/f", write_type="THROUGH")
    with open(os.path.join(master._tmp, "ufs", "d1", "sub", "f"), "wb") as f:
        f.write(b"abc")
    fs.complete_file("/d1/sub/f", ufs_length=3)
    fs.create_directory("/d2", write_type="CACHE_THROUGH")
    fs.rename("/d1/sub", "/d2/moved")
    assert fs.get_status("/d2/moved/f", load_metadata="NEVER").length == 3
    assert os.path.exists(os.path.join(master._tmp, "ufs", "d2", "moved", "f"))
    with pytest.raises(ex.InvalidPathException):
        fs.rename("/d2", "/d2/moved/x")
    fs.create_directory("/d3")
    with pytest.raises(ex.FileAlreadyExistsException):
        fs.rename("/d2", "/d3")


def test_load_metadata_and_sync(master):
    ufs = os.path.join(master._tmp, "ufs")
    os.makedirs(os.path.join(ufs, "ext", "deep"))
    for n in ("a", "deep/b"):
        with open(os.path.join(ufs, "ext", n), "wb") as f:
            f.write(b"x" * 10)
    fs = master.fs_master
    assert fs.get_status("/ext/deep/b").length == 10  # loaded on demand (ONCE)
    names = [i.path for i in fs.list_status("/ext")]
    assert names == ["/ext/a", "/ext/deep"]
    with pytest.raises(ex.FileDoesNotExistException):
        fs.get_status("/ext/zz", load_metadata="NEVER")
    os.remove(os.path.join(ufs, "ext", "a"))
    with open(os.path.join(ufs, "ext", "new"), "wb") as f:
        f.write(b"yy")
    stats = fs.sync_metadata("/ext")
    assert stats["removed"] >= 1 and stats["added"] >= 1
    assert sorted(i.name for i in fs.list_status("/ext", load_metadata="NEVER")) == ["deep", "new"]
    assert fs.check_consistency("/ext") == []


def test_mount_unmount_and_reverse_resolve(master, tmp_path):
    other = tmp_path / "other_ufs"
    (other / "d").mkdir(parents=True)
    (other / "d" / "f").write_bytes(b"12345")
    fs = master.fs_master
    fs.mount("/mnt", str(other), read_only=True)
    assert fs.get_status("/mnt/d/f").length == 5
    assert fs.reverse_resolve(str(other / "d" / "f")) == "/mnt/d/f"
    with pytest.raises(ex.AccessControlException):
        fs.create_file("/mnt/new", write_type="THROUGH")
    with pytest.raises(ex.InvalidPathException):
        fs.mount("/mnt/inner", str(other / "d"))
    assert "/mnt" in fs.get_mount_table()
    fs.unmount("/mnt")
    assert not fs.tree.exists("/mnt") and "/mnt" not in fs.get_mount_table()


def test_set_attribute_pin_ttl_and_free(master):
    fs, bm = master.fs_master, master.block_master
    fs.create_directory("/p")
    fs.create_file("/p/f", block_size=10, write_type="CACHE_THROUGH")
    fs.complete_file("/p/f", ufs_length=0)
    fs.set_attribute("/p", pinned=True, recursive=True)
    assert fs.pinned_file_ids() == [fs.get_status("/p/f").fileId]
    with pytest.raises(ex.FailedPreconditionException):
        fs.free("/p", recursive=True)
    fs.free("/p", recursive=True, forced=True)
    assert fs.pinned_file_ids() == []
    fs.set_attribute("/p/f", ttl=1, ttl_action="DELETE")
    time.sleep(0.01)
    fs.tree.ttl_buckets.interval = 1
    fs.tree.ttl_buckets.clear()
    fs.tree.ttl_buckets.insert(fs.tree.get("/p/f"))
    assert fs.ttl_check() == ["/p/f"]
    assert not fs.tree.exists("/p/f")
    del bm


def test_acl_and_permissions(tmp_path):
    conf = Configuration({"alluxio.master.journal.folder": str(tmp_path / "j"),
                          "alluxio.security.authorization.permission.enabled": "true"})
    m = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    try:
        from alluxio_amd.security import as_user
        fs = m.fs_master
        fs.permission.superuser = "root_admin"
        with as_user("root_admin"):
            fs.create_directory("/priv", mode=0o700)
            fs.set_attribute("/priv", owner="alice")
        with as_user("bob"):
            with pytest.raises(ex.AccessControlException):
                fs.create_file("/priv/x", write_type="MUST_CACHE")
        with as_user("alice"):
            fs.create_file("/priv/x", write_type="MUST_CACHE")
            fs.set_acl("/priv", "MODIFY", [__import__("alluxio_amd.security.acl", fromlist=["AclEntry"]).AclEntry.parse(
                "user:bob:rwx")])
        with as_user("bob"):
            fs.create_file("/priv/y", write_type="MUST_CACHE")
            info = fs.get_status("/priv")
            assert any(e.subject == "bob" for e in info.acl.entries)
    finally:
        m.stop()


def test_journal_replay_restores_namespace(tmp_path):
    conf = Configuration({"alluxio.master.journal.folder": str(tmp_path / "j")})
    m = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    m.fs_master.create_directory("/r/s", recursive=True)
    m.fs_master.create_file("/r/s/f", write_type="MUST_CACHE")
    m.fs_master.rename("/r/s/f", "/r/g")
    m.meta_master.set_path_configuration("/r", {"alluxio.user.file.writetype.default": "THROUGH"})
    cid = m.meta_master.cluster_id
    m.stop()
    m2 = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m2.start(start_heartbeats=False)
    try:
        assert sorted(i.path for i in m2.fs_master.list_status("/", recursive=True, load_metadata="NEVER")) == \
            ["/r", "/r/g", "/r/s"]
        assert m2.meta_master.path_conf.get_all()["/r"]["alluxio.user.file.writetype.default"] == "THROUGH"
        assert m2.meta_master.cluster_id == cid
        f = m2.fs_master.create_file("/r/h", write_type="MUST_CACHE")
        assert f.fileId not in (m2.fs_master.get_status("/r/g").fileId,)
    finally:
        m2.stop()


def test_block_master_worker_lifecycle(master):
    bm = master.block_master
    addr = pb.grpc.WorkerNetAddress(host="h", rpcPort=5, dataPort=5)
    wid = bm.get_worker_id(addr)
    assert bm.get_worker_id(addr) == wid
    assert bm.worker_heartbeat(wid, {}, [], {})[0] == "Register"
    bm.commit_block_in_ufs(77, 10)
    bm.worker_register(wid, ["MEM"], {"MEM": 100}, {"MEM": 10}, {("MEM", "HBM"): [77, 88]})
    cmd, data = bm.worker_heartbeat(wid, {"MEM": 10}, [], {})
    assert cmd == "Free" and data == [88]  # unknown block -> free it
    assert [l.workerId for l in bm.block_info(77).locations] == [wid]
    bm.remove_blocks([77], delete=False)
    assert bm.worker_heartbeat(wid, {"MEM": 0}, [], {}) == ("Free", [77, 88])
    bm.worker_timeout_ms = 0
    time.sleep(0.002)
    assert bm.detect_lost_workers() == [wid]
    assert bm.worker_count() == 0 and bm.lost_worker_count() == 1
    assert 77 in bm.lost_blocks()
    assert bm.get_worker_id(addr) == wid  # re-registration keeps the id


def _atime(m, path):
    return m.fs_master.get_status(path, update_timestamps=False).lastAccessTimeMs


def test_access_time_updates_journaled_and_replayed(tmp_path):
    """AccessTimeUpdater: an open (getStatus with READ access) and a listing advance
    lastAccessTimeMs past the precision; batched updates are journaled at the flush (or stop) and
    survive a restart (reference AccessTimeUpdater.java, DefaultFileSystemMaster.java:882,1103)."""
    for flush in ("0", "1h"):
        jdir = tmp_path / f"journal{flush}"
        conf = Configuration({"alluxio.master.journal.folder": str(jdir),
                              "alluxio.security.authorization.permission.enabled": "false",
                              "alluxio.master.file.access.time.update.precision": "0",
                              "alluxio.master.file.access.time.journal.flush.interval": flush})
        m = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / f"ufs{flush}"))
        m.start(start_heartbeats=False)
        fs = m.fs_master
        fs.create_directory("/d")
        fs.create_file("/d/f", write_type="MUST_CACHE")
        fs.complete_file("/d/f")
        t0, d0 = _atime(m, "/d/f"), _atime(m, "/d")
        time.sleep(0.02)
        fs.get_status("/d/f", access_mode=0)                 # no access mode: not an access
        assert _atime(m, "/d/f") == t0
        fs.get_status("/d/f")                                # READ access (an open)
        t1 = _atime(m, "/d/f")
        assert t1 > t0
        fs.list_status("/d")
        assert _atime(m, "/d") > d0
        upd = fs.access_time
        assert upd.updates >= 2
        assert bool(upd._pending) == (flush != "0")          # batched: journaled at the flush / stop
        m.stop()                                             # flushes the batch
        m2 = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / f"ufs{flush}"))
        m2.start(start_heartbeats=False)
        assert _atime(m2, "/d/f") == t1
        m2.stop()


def test_access_time_precision_skips_updates(master):
    fs = master.fs_master
    fs.create_file("/p", write_type="MUST_CACHE")
    fs.complete_file("/p")
    n = fs.access_time.updates
    fs.get_status("/p")                                      # default precision: 1 day
    assert fs.access_time.updates == n


def test_time_series_recorder(master):
    ts = master.time_series
    ts.heartbeat()
    master.metrics_master._cluster["Cluster.BytesReadUfsAll"] = 6 << 20
    ts._last = (ts._last[0] - 60.0, ts._last[1])             # one minute later
    ts.heartbeat()
    series = {s["name"]: s["dataPoints"] for s in ts.store.series()}
    assert {"% Alluxio Space Used", "% UFS Space Used", "Cluster.BytesReadUfsThroughput",
            "Cluster.BytesWrittenAlluxioThroughput"} <= set(series)
    assert len(series["% Alluxio Space Used"]) == 2
    assert series["Cluster.BytesReadUfsThroughput"][-1]["value"] == pytest.approx(6 << 20, rel=0.01)
    assert 0 <= series["% UFS Space Used"][-1]["value"] <= 100
    assert {"timeStamp", "value"} == set(series["% UFS Space Used"][0])
