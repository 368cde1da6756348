"""End-to-end integration over an in-process cluster (reference LocalAlluxioClusterResource-based
integration tests: FileInStreamIntegrationTest, RemoteReadIntegrationTest, FreeIntegrationTest,
and TestRunner's ReadType x WriteType matrix from ``bin/alluxio runTests``)."""
import os

import numpy as np
import pytest

from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.utils import exceptions as ex

MB = 1 << 20


@pytest.fixture(scope="module")
def cluster():
    c = LocalAlluxioCluster(num_workers=2, grpc=True, conf={
        "alluxio.worker.tieredstore.level0.dirs.path": "dram",
        "alluxio.worker.tieredstore.level0.dirs.quota": "64MB",
        "alluxio.user.block.size.bytes.default": "4MB"}).start()
    yield c
    c.stop()


@pytest.mark.parametrize("write_type", ["MUST_CACHE", "CACHE_THROUGH", "THROUGH", "ASYNC_THROUGH"])
@pytest.mark.parametrize("read_type", ["NO_CACHE", "CACHE", "CACHE_PROMOTE"])
def test_read_write_type_matrix(cluster, write_type, read_type):
    fs = cluster.client()
    path = f"/matrix/{write_type}-{read_type}"
    data = os.urandom(9 * MB + 123)
    fs.write_file(path, data, write_type=write_type)
    st = fs.get_status(path)
    assert st.length == len(data) and st.completed
    assert st.persisted == (write_type in ("CACHE_THROUGH", "THROUGH"))
    assert fs.read_file(path, read_type=read_type) == data
    with fs.open_file(path, read_type=read_type) as f:
        f.seek(5 * MB - 7)
        assert f.read(100) == data[5 * MB - 7:5 * MB + 93]
        buf = bytearray(1000)
        assert f.pread(4 * MB - 500, buf) == 1000 and bytes(buf) == data[4 * MB - 500:4 * MB + 500]
    fs.close()


def test_through_then_cache_read_populates_workers(cluster):
    fs = cluster.client()
    data = os.urandom(6 * MB)
    fs.write_file("/t/through", data, write_type="THROUGH")
    assert fs.get_status("/t/through").in_alluxio_percentage == 0
    assert fs.read_file("/t/through", read_type="CACHE") == data
    assert fs.get_status("/t/through").in_alluxio_percentage == 100
    fs.free("/t/through")
    cluster.heartbeat_workers()
    assert fs.get_status("/t/through").in_alluxio_percentage == 0
    assert fs.read_file("/t/through", read_type="NO_CACHE") == data
    assert fs.get_status("/t/through").in_alluxio_percentage == 0


def test_remote_grpc_read_path(cluster):
    """Force the gRPC ReadBlock path by dropping the in-process worker shortcut."""
    from alluxio_amd.client import context as cctx
    fs = cluster.client()
    data = os.urandom(5 * MB + 9)
    fs.write_file("/r/remote", data, write_type="MUST_CACHE")
    saved = dict(cctx._LOCAL_WORKERS)
    cctx._LOCAL_WORKERS.clear()
    try:
        assert fs.read_file("/r/remote") == data
    finally:
        cctx._LOCAL_WORKERS.update(saved)
    fs.close()


def test_grpc_cold_read_streams_while_caching(cluster):
    """A cold block read over gRPC from offset 0 is cached while it streams (read-through,
    UnderFileSystemBlockReader.java:205-243); a mid-block cold read streams without caching."""
    from alluxio_amd.client import context as cctx
    fs = cluster.client()
    data = os.urandom(9 * MB + 5)
    fs.write_file("/rt/f", data, write_type="THROUGH")
    fs.write_file("/rt/g", data, write_type="THROUGH")
    saved = dict(cctx._LOCAL_WORKERS)
    cctx._LOCAL_WORKERS.clear()
    before = sum(w.worker.metrics.counter("BytesReadUfsThrough").count for w in cluster.workers)
    try:
        assert fs.read_file("/rt/f", read_type="CACHE") == data
        with fs.open_file("/rt/g", read_type="CACHE") as f:
            f.seek(MB + 3)
            assert f.read(1000) == data[MB + 3:MB + 1003]
    finally:
        cctx._LOCAL_WORKERS.update(saved)
    assert fs.get_status("/rt/f").in_alluxio_percentage == 100
    through = sum(w.worker.metrics.counter("BytesReadUfsThrough").count for w in cluster.workers)
    assert through - before >= len(data)
    fs.close()


def test_device_read_into_tensor(cluster):
    import torch
    fs = cluster.client()
    data = np.random.default_rng(3).integers(0, 256, 3 * MB + 11, dtype=np.uint8)
    fs.write_file("/dev/x", data, write_type="MUST_CACHE")
    out = torch.empty(len(data), dtype=torch.uint8)
    with fs.open_file("/dev/x") as f:
        assert f.read_into(out) == len(data)
    assert np.array_equal(out.numpy(), data)


def test_namespace_ops_through_client(cluster):
    fs = cluster.client()
    fs.create_directory("/ns/a/b", recursive=True, write_type="CACHE_THROUGH")
    fs.write_file("/ns/a/b/f", b"hello", write_type="CACHE_THROUGH")
    assert [s.name for s in fs.list_status("/ns/a")] == ["b"]
    fs.rename("/ns/a/b/f", "/ns/a/g")
    assert fs.read_file("/ns/a/g") == b"hello"
    assert os.path.exists(os.path.join(cluster.ufs_root, "ns", "a", "g"))
    with pytest.raises(ex.NotFoundException):
        fs.get_status("/ns/nope")
    fs.set_attribute("/ns/a/g", pinned=True)
    assert fs.get_status("/ns/a/g").pinned
    with pytest.raises(ex.AlluxioStatusException):
        fs.free("/ns/a/g")
    fs.set_attribute("/ns/a/g", pinned=False)
    fs.delete("/ns", recursive=True)
    assert not fs.exists("/ns")
    assert not os.path.exists(os.path.join(cluster.ufs_root, "ns"))


def test_mount_external_ufs(cluster, tmp_path):
    ext = tmp_path / "ext"
    ext.mkdir()
    (ext / "data.bin").write_bytes(b"z" * 4096)
    fs = cluster.client()
    fs.mount("/ext", str(ext))
    assert fs.read_file("/ext/data.bin") == b"z" * 4096
    assert "/ext" in fs.get_mount_table()
    fs.unmount("/ext")
    assert not fs.exists("/ext", load_metadata="NEVER")


def test_worker_heartbeat_reports_eviction(tmp_path):
    with LocalAlluxioCluster(num_workers=1, conf={
            "alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": "8MB",
            "alluxio.user.block.size.bytes.default": "2MB"}) as c:
        fs = c.client()
        for i in range(6):
            fs.write_file(f"/ev/f{i}", os.urandom(2 * MB), write_type="CACHE_THROUGH")
        c.heartbeat_workers()
        cached = [fs.get_status(f"/ev/f{i}").in_alluxio_percentage for i in range(6)]
        assert cached[:2] == [0, 0] and cached[2:] == [100] * 4
        assert fs.read_file("/ev/f0")  # re-cached from the UFS
        fs.close()


def test_async_persist(tmp_path):
    with LocalAlluxioCluster(num_workers=1, conf={
            "alluxio.worker.tieredstore.level0.dirs.path": "dram"}) as c:
        fs = c.client()
        fs.write_file("/ap/f", b"persist me", write_type="ASYNC_THROUGH")
        st = fs.get_status("/ap/f")
        assert st.persistence_state if False else st.info.persistenceState == "TO_BE_PERSISTED"
        from alluxio_amd.job.persist import inline_persist_handler
        c.master.fs_master.persist_handler = inline_persist_handler(c.master.fs_master, fs)
        c.master.fs_master.persistence_scheduler_heartbeat()
        st = fs.get_status("/ap/f")
        assert st.persisted
        with open(os.path.join(c.ufs_root, "ap", "f"), "rb") as f:
            assert f.read() == b"persist me"


def test_client_metrics_sync():
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"}) as c:
        fs = c.client()
        fs.write_file("/m/f", b"x" * 1000, write_type="MUST_CACHE")
        fs.read_file("/m/f")
        assert fs.ctx.sync_metrics() > 0
        ms = c.master.metrics_master.get_metrics()
        assert any("BytesReadClient" in k for k in ms), sorted(ms)[:20]
        fs.close()


def test_domain_socket_data_server(tmp_path):
    """A same-node client reaches the worker's data server over its Unix domain socket
    (AlluxioWorkerProcess domain-socket server; BytesReadDomain metric)."""
    import os
    from alluxio_amd.client.context import unregister_local_worker, worker_address_str
    from alluxio_amd.rpc import domain_socket_for
    import tempfile
    uds_dir = tempfile.mkdtemp(prefix="uds", dir="/tmp")   # sun_path is limited to 108 bytes
    with LocalAlluxioCluster(num_workers=1, grpc=True, work_dir=str(tmp_path / "c"), conf={
            "alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.worker.data.server.domain.socket.address": str(uds_dir),
            "alluxio.worker.data.server.domain.socket.as.uuid": "true"}) as c:
        w = c.workers[0]
        path = w.worker.address.domainSocketPath
        assert path.startswith(uds_dir) and os.path.exists(path)
        data = os.urandom(3 << 20)
        fs = c.client()
        fs.write_file("/uds/f", data, write_type="MUST_CACHE")
        addr = worker_address_str(w.worker.address)
        unregister_local_worker(addr)            # no in-process shortcut: go through the data server
        from alluxio_amd.client.file_system import FileSystem
        conf2 = c.conf.copy()
        conf2.set("alluxio.user.network.inprocess.transport.enabled", "false")
        conf2.set("alluxio.user.short.circuit.enabled", "false")   # else the shared-DRAM short circuit wins
        fs2 = FileSystem(conf=conf2, master_address=c.master.address)
        assert fs2.read_file("/uds/f") == data
        assert domain_socket_for(addr) == path
        assert w.worker.metrics.counter("BytesReadDomain").count >= len(data)
        fs.close()
        fs2.close()
    import shutil
    shutil.rmtree(uds_dir, ignore_errors=True)


def test_ufs_fallback_block_write(tmp_path):
    """UFS_FALLBACK_BLOCK (UfsFallbackBlockWriteHandler): an ASYNC_THROUGH write with the UFS tier
    enabled to a worker too small for the block spills the block -- bytes already written
    included -- to a UFS block file, commits it to the master as in-UFS, reads come back from
    that file, and persisting the file removes the staging block files.  Both the gRPC handler
    and the in-process writer are exercised."""
    from alluxio_amd.client import context as cctx
    from alluxio_amd.worker.ufs_fallback import UFS_BLOCKS_DIR
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": "3MB",
            "alluxio.worker.hbm.page.size": "256KB",
            "alluxio.user.block.size.bytes.default": "4MB",
            "alluxio.user.file.buffer.bytes": "1MB",
            "alluxio.user.file.ufs.tier.enabled": "true"}
    with LocalAlluxioCluster(num_workers=1, grpc=True, conf=conf, work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        from alluxio_amd.job.persist import inline_persist_handler
        c.master.fs_master.persist_handler = inline_persist_handler(c.master.fs_master, fs)
        blocks_dir = os.path.join(c.ufs_root, UFS_BLOCKS_DIR)
        w = c.workers[0].worker
        for name, via_grpc in (("inproc", False), ("grpc", True)):
            data = os.urandom(9 * MB + 77)
            before = w.metrics.counter("UfsFallbackBlocks").count
            saved = dict(cctx._LOCAL_WORKERS)
            if via_grpc:
                cctx._LOCAL_WORKERS.clear()
            try:
                fs.write_file(f"/fb/{name}", data, write_type="ASYNC_THROUGH")
            finally:
                cctx._LOCAL_WORKERS.update(saved)
            st = fs.get_status(f"/fb/{name}")
            assert st.length == len(data) and not st.persisted
            assert os.listdir(blocks_dir), "no block went to the UFS tier"
            assert w.metrics.counter("UfsFallbackBlocks").count > before
            assert fs.read_file(f"/fb/{name}", read_type="NO_CACHE") == data
            # persisting (UFS-tier blocks read back from their block files) clears the staging files
            c.master.fs_master.persistence_scheduler_heartbeat()
            assert fs.get_status(f"/fb/{name}").persisted
            with open(os.path.join(c.ufs_root, "fb", name), "rb") as f:
                assert f.read() == data
            assert os.listdir(blocks_dir) == []
        fs.close()


def test_cache_through_ufs_copy_matches_after_free(cluster):
    """CACHE_THROUGH writes the UFS copy beside the cache copy (zero-copy view of the caller's
    buffer); after freeing the cached blocks the bytes come back from the UFS intact."""
    fs = cluster.client()
    data = np.random.default_rng(5).integers(0, 256, 13 * MB + 17, dtype=np.uint8)
    fs.write_file("/ct/big", data, write_type="CACHE_THROUGH")
    fs.free("/ct/big")
    cluster.heartbeat_workers()
    assert fs.read_file("/ct/big", read_type="NO_CACHE") == data.tobytes()
    fs.close()


def test_remote_fetcher_flow_control_and_master_length(tmp_path):
    """Worker-to-worker gRPC block fetch (GrpcDataReader.java:123-160 semantics): the block length
    comes from the master, every chunk is acknowledged, and the source's flow-control window
    (alluxio.worker.network.reader.buffer.size) really throttles a reader that stops acking."""
    import queue
    import threading

    from alluxio_amd.proto import pb
    from alluxio_amd.rpc import Channel
    from alluxio_amd.worker.remote import remote_block_fetcher
    c = LocalAlluxioCluster(num_workers=2, grpc=True, work_dir=str(tmp_path), conf={
        "alluxio.worker.tieredstore.level0.dirs.path": "dram",
        "alluxio.worker.tieredstore.level0.dirs.quota": "64MB",
        "alluxio.worker.network.reader.buffer.size": "1MB",
        "alluxio.user.block.size.bytes.default": "8MB"}).start()
    try:
        fs = c.client()
        data = os.urandom(6 * MB + 5)
        fs.write_file("/rf", data, write_type="MUST_CACHE")
        bi = fs.get_status("/rf").fileBlockInfos[0].blockInfo
        src = next(w for w in c.workers if w.worker.has_block(bi.blockId))
        dst = next(w for w in c.workers if w is not src)
        host, port = src.address.rsplit(":", 1)
        # 1) a reader that never acks gets at most window + one chunk, then the source pauses
        got, reqs = [], queue.Queue()

        def it():
            yield pb.block.ReadRequest(block_id=bi.blockId, offset=0, length=bi.length, chunk_size=256 << 10)
            while reqs.get() is not None:
                pass
        stream = Channel(src.address, force_grpc=True).raw_stream("alluxio.grpc.block.BlockWorker", "ReadBlock")(it())

        def drain():
            try:
                for r in stream:
                    got.append(len(r.chunk.data))
            except Exception:  # noqa: BLE001 - cancelled below
                pass
        t = threading.Thread(target=drain, daemon=True)
        t.start()
        t.join(1.5)
        assert t.is_alive() and sum(got) <= (1 << 20) + (256 << 10), sum(got)
        reqs.put(None)
        stream.cancel()
        # 2) the fetcher (no length given: asked from the master) acks and completes the block
        remote_block_fetcher(dst.worker, host, int(port))(bi.blockId)
        assert dst.worker.read_bytes(bi.blockId, 0, bi.length) == data
    finally:
        c.stop()
