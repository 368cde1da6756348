"""The worker's native gRPC data port (csrc/data_server.cpp + the H2 front end's streaming bridge)
and the native host reader (csrc/block_source.cpp).

Reference behaviour pinned here: GrpcDataServer.java:50-198 serves the whole BlockWorker service on
the data port; BlockReadHandler.java:111-152 / AbstractReadHandler.java stream a locked block in
chunks and pause while more than the window is un-acked by ``offset_received``;
ReadResponseMarshaller.java:38-80 (header + raw chunk bytes) is what a stock gRPC client decodes.
"""
import os
import time

import grpc
import numpy as np
import pytest

from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.ops.native import lib
from alluxio_amd.proto import SERVICES, pb
from alluxio_amd.rpc import marshal

pytestmark = pytest.mark.skipif(not lib().FrameRpcServer.grpc_available(), reason="libnghttp2 not present")

BW = "alluxio.grpc.block.BlockWorker"
REMOTE = {"alluxio.user.network.inprocess.transport.enabled": "false",
          "alluxio.user.short.circuit.enabled": "false"}


def _cluster(tmp_path, extra=None, auth="NOSASL"):
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": "512MB",
            "alluxio.user.block.size.bytes.default": "4MB",
            "alluxio.security.authentication.type": auth,
            "alluxio.security.authorization.permission.enabled": "false"}
    conf.update(extra or {})
    return LocalAlluxioCluster(num_workers=1, conf=conf, grpc=True, work_dir=str(tmp_path / "c"))


def _remote_fs(cluster, **props):
    from alluxio_amd.client.file_system import FileSystem
    from alluxio_amd.conf import Configuration
    p = dict(REMOTE)
    p.update(props)
    if cluster.conf.get("alluxio.security.authentication.type") == "NOSASL":
        p["alluxio.security.authentication.type"] = "NOSASL"
    return FileSystem(conf=Configuration(p), master_address=cluster.master.address)


def _blocks(fs, path):
    st = fs.get_status(path)
    return [(fbi.blockInfo.blockId, fbi.blockInfo.length) for fbi in st.fileBlockInfos]


def test_native_reader_over_data_port(tmp_path):
    with _cluster(tmp_path) as c:
        fs = c.client()
        data = np.random.default_rng(0).integers(0, 256, (10 << 20) + 321, dtype=np.uint8)
        fs.write_file("/f", data, write_type="MUST_CACHE")
        w = c.workers[0]
        assert w.data_server is not None and w.worker.address.dataPort == w.data_server.port
        assert w.data_server.port != w.worker.address.rpcPort
        rfs = _remote_fs(c)
        try:
            with rfs.open_file("/f") as f:                      # 4 KiB read(buf) loop
                assert f._nat is not None
                buf = bytearray(4096)
                out = bytearray()
                while True:
                    n = f.readinto(buf)
                    if not n:
                        break
                    out += buf[:n]
            assert bytes(out) == data.tobytes()
            with rfs.open_file("/f") as f:                      # seeks, across and within blocks
                for pos, n in [(9 << 20, 5000), (7, 100), ((4 << 20) - 10, 40), (len(data) - 3, 10)]:
                    f.seek(pos)
                    assert f.read(n) == data[pos:pos + n].tobytes()
                    assert f.tell() == min(len(data), pos + n)
            st = w.data_server.stats
            assert st.streams >= 3 and st.bytes >= len(data) and st.declined == 0
        finally:
            rfs.close()
            fs.close()


def test_stock_grpc_client_on_data_port_flow_control(tmp_path):
    """A grpcio ReadBlock call against the native port: frames decode as ReadResponse, the server
    stops at the window until offset_received arrives, and the stream completes after acks."""
    with _cluster(tmp_path, {"alluxio.worker.network.reader.buffer.size": "1MB"}) as c:
        fs = c.client()
        data = np.random.default_rng(1).integers(0, 256, 4 << 20, dtype=np.uint8)
        fs.write_file("/g", data, write_type="MUST_CACHE")
        (bid, blen), = _blocks(fs, "/g")
        port = c.workers[0].data_server.port
        ch = grpc.insecure_channel(f"127.0.0.1:{port}")
        try:
            spec = SERVICES[BW]["ReadBlock"]
            call = ch.stream_stream(spec.path, spec.request.SerializeToString, marshal.decode_read_response)
            import queue
            q: queue.Queue = queue.Queue()
            q.put(pb.block.ReadRequest(block_id=bid, offset=0, length=blen, chunk_size=64 << 10))

            def reqs():
                while True:
                    r = q.get()
                    if r is None:
                        return
                    yield r
            it = call(reqs())
            got = bytearray()
            # without acks the server sends at most window (+ one chunk)
            deadline = time.time() + 5
            while len(got) < (1 << 20):
                got += bytes(next(it).chunk.data)
                assert time.time() < deadline
            time.sleep(0.3)
            sent = c.workers[0].data_server.stats.bytes
            assert sent <= (1 << 20) + (64 << 10), sent
            while len(got) < blen:
                q.put(pb.block.ReadRequest(offset_received=len(got)))
                got += bytes(next(it).chunk.data)
            q.put(None)
            assert bytes(got) == data.tobytes()
            with pytest.raises(StopIteration):
                next(it)
            # a block the worker does not hold: bridged to the Python servicer -> NOT_FOUND
            call2 = ch.stream_stream(spec.path, spec.request.SerializeToString, spec.response.FromString)
            with pytest.raises(grpc.RpcError) as ei:
                list(call2(iter([pb.block.ReadRequest(block_id=12345, offset=0, length=10)])))
            assert ei.value.code() == grpc.StatusCode.NOT_FOUND
            assert c.workers[0].data_server.stats.declined >= 1
        finally:
            ch.close()
            fs.close()


def test_stock_grpc_write_block_then_native_read(tmp_path):
    """A stock gRPC client's WriteBlock on the data port (chunks written into the block by the C++
    server, commit through the internal NativeWriteCommit call), read back natively."""
    with _cluster(tmp_path) as c:
        fs = c.client()
        rfs = _remote_fs(c)
        w = c.workers[0]
        try:
            ch = grpc.insecure_channel(f"127.0.0.1:{w.data_server.port}")
            spec = SERVICES[BW]["WriteBlock"]
            call = ch.stream_stream(spec.path, marshal.serialize, spec.response.FromString)
            payload = np.random.default_rng(2).integers(0, 256, (3 << 20) + 17, dtype=np.uint8).tobytes()
            bid = 777
            msgs = [pb.block.WriteRequest(command=pb.block.WriteRequestCommand(type=0, id=bid, offset=0,
                                                                                 space_to_reserve=1 << 20))]
            for i in range(0, len(payload), 1 << 20):
                msgs.append(marshal.write_request_frame(payload[i:i + (1 << 20)]))
            resps = list(call(iter(msgs)))
            assert resps[-1].offset == len(payload)
            ch.close()
            assert w.worker.has_block(bid)
            assert w.data_server.stats.write_streams >= 1 and w.data_server.stats.write_bytes >= len(payload)
            src = lib().GrpcBlockSource("127.0.0.1", w.data_server.port, bid, len(payload), 1 << 20)
            out = np.empty(len(payload), dtype=np.uint8)
            src.read_into(0, len(payload), out.ctypes.data)
            assert out.tobytes() == payload
            src.close()
            # the client library's WriteBlock (rpc port) and native read back (data port)
            data = np.random.default_rng(3).integers(0, 256, (5 << 20) + 1, dtype=np.uint8)
            rfs.write_file("/w", data, write_type="MUST_CACHE")
            assert rfs.read_file("/w") == data.tobytes()
        finally:
            rfs.close()
            fs.close()


def test_ufs_read_through_bridged(tmp_path):
    """A block that is not cached, with native UFS reads off: ReadBlock with UFS options is served
    by the Python servicer through the bridge (read-through caching), then natively once cached."""
    with _cluster(tmp_path, {"alluxio.worker.data.server.native.ufs.read.enabled": "false"}) as c:
        fs = c.client()
        data = np.random.default_rng(4).integers(0, 256, (6 << 20) + 9, dtype=np.uint8)
        fs.write_file("/u", data, write_type="CACHE_THROUGH")
        fs.free("/u")
        w = c.workers[0]
        c.heartbeat_workers()          # the Free command runs on the worker heartbeat
        assert not w.worker.native.block_ids(-1)
        rfs = _remote_fs(c)
        try:
            before = w.data_server.stats.declined
            assert rfs.read_file("/u") == data.tobytes()
            assert w.data_server.stats.declined > before
            assert rfs.read_file("/u") == data.tobytes()
        finally:
            rfs.close()
            fs.close()


def test_native_read_requires_authenticated_channel(tmp_path):
    with _cluster(tmp_path, auth="SIMPLE") as c:
        fs = c.client()
        data = np.arange(1 << 20, dtype=np.uint32).view(np.uint8)
        fs.write_file("/s", data, write_type="MUST_CACHE")
        (bid, blen), = _blocks(fs, "/s")
        port = c.workers[0].data_server.port
        with pytest.raises(lib().StoreError) as ei:       # no channel-id: refused in C++
            src = lib().GrpcBlockSource("127.0.0.1", port, bid, blen, 1 << 20)
            src.read_into(0, 100, np.empty(100, dtype=np.uint8).ctypes.data)
        assert "authenticated" in str(ei.value)
        rfs = _remote_fs(c)                                # SASL channel: its id authorizes the call
        try:
            assert rfs.read_file("/s") == data.tobytes()
        finally:
            rfs.close()
            fs.close()


def test_native_client_against_grpcio_server(tmp_path):
    """The native gRPC client interoperates with the pure-grpcio BlockWorker server (rpc port)."""
    with _cluster(tmp_path) as c:
        fs = c.client()
        data = np.random.default_rng(5).integers(0, 256, 3 << 20, dtype=np.uint8)
        fs.write_file("/i", data, write_type="MUST_CACHE")
        (bid, blen), = _blocks(fs, "/i")
        rpc_port = c.workers[0].worker.address.rpcPort
        src = lib().GrpcBlockSource("127.0.0.1", rpc_port, bid, blen, 256 << 10)
        out = np.empty(blen, dtype=np.uint8)
        src.read_into(0, blen, out.ctypes.data)
        assert np.array_equal(out, data)
        src.read_into(1000, 50, out.ctypes.data)          # backward: a new call at the offset
        assert np.array_equal(out[:50], data[1000:1050])
        src.close()
        fs.close()


def test_cancelled_stream_releases_the_block_lock(tmp_path):
    with _cluster(tmp_path) as c:
        fs = c.client()
        data = np.random.default_rng(6).integers(0, 256, 4 << 20, dtype=np.uint8)
        fs.write_file("/x", data, write_type="MUST_CACHE")
        (bid, blen), = _blocks(fs, "/x")
        w = c.workers[0]
        src = lib().GrpcBlockSource("127.0.0.1", w.data_server.port, bid, blen, 64 << 10)
        out = np.empty(4096, dtype=np.uint8)
        src.read_into(0, 4096, out.ctypes.data)
        src.close()                                        # mid-stream
        deadline = time.time() + 5
        while True:                                        # the read lock is gone: removable
            try:
                w.worker.remove_block(1, bid)
                break
            except Exception:  # noqa: BLE001
                assert time.time() < deadline
                time.sleep(0.05)
        assert not w.worker.has_block(bid)
        fs.close()


def test_in_process_host_reads_use_store_source(tmp_path):
    """An in-process worker: host read(buf) goes through the chunk buffer filled from the store."""
    with _cluster(tmp_path) as c:
        from alluxio_amd.client.file_system import FileSystem
        from alluxio_amd.conf import Configuration
        # 1 MiB chunks: several refills per block, so read-ahead inside a block is visible
        fs = FileSystem(conf=Configuration({"alluxio.user.native.reader.buffer.size": "1MB"}),
                        master_address=c.master.address)
        data = np.random.default_rng(7).integers(0, 256, (9 << 20) + 5, dtype=np.uint8)
        fs.write_file("/p", data, write_type="MUST_CACHE")
        with fs.open_file("/p") as f:
            b = bytearray(4096)
            parts = []
            while True:
                n = f.readinto(b)
                if not n:
                    break
                parts.append(bytes(b[:n]))
            assert f._nat.refills >= 9
            assert f._nat.prefetch_hits >= 5          # the next chunk was read ahead
        assert b"".join(parts) == data.tobytes()
        # prefetch off: same bytes through synchronous refills only
        from alluxio_amd.client.file_system import FileSystem
        from alluxio_amd.conf import Configuration
        nfs = FileSystem(conf=Configuration({"alluxio.user.native.reader.prefetch.enabled": "false"}),
                         master_address=c.master.address)
        with nfs.open_file("/p") as f:
            assert f.read() == data.tobytes() and f._nat.prefetch_hits == 0
        nfs.close()
        fs.close()


def test_native_writer_over_data_port(tmp_path):
    """FileOutStream to a remote worker: every block goes through the native client
    (GrpcBlockSink) and the native WriteBlock server; the master sees the committed blocks."""
    with _cluster(tmp_path) as c:
        w = c.workers[0]
        rfs = _remote_fs(c, **{"alluxio.user.block.size.bytes.default": "4MB"})
        try:
            st0 = (w.data_server.stats.write_streams, w.data_server.stats.write_bytes)
            data = np.random.default_rng(7).integers(0, 256, (13 << 20) + 5, dtype=np.uint8)
            with rfs.create_file("/nw", write_type="MUST_CACHE") as f:
                for i in range(0, len(data), 3 << 20):           # writes that straddle blocks
                    f.write(data[i:i + (3 << 20)])
            blocks = _blocks(rfs, "/nw")
            assert len(blocks) == 4
            assert w.data_server.stats.write_streams - st0[0] == 4
            assert w.data_server.stats.write_bytes - st0[1] == len(data)
            assert rfs.get_status("/nw").in_alluxio_percentage == 100
            assert all(w.worker.has_block(b) for b, _ in blocks)
            assert rfs.read_file("/nw") == data.tobytes()
            # CRC recorded at commit, as for any committed block
            assert all(b in w.worker.crc for b, _ in blocks) or not w.worker.crc_enabled
        finally:
            rfs.close()


def test_native_ufs_file_writes(tmp_path):
    """THROUGH / CACHE_THROUGH from a remote client: the first UFS_FILE stream of a mount runs in
    Python, which registers the local-directory mount; later streams are written by the native
    server (temp file renamed over the target).  Paths outside the mount stay in Python."""
    import os
    with _cluster(tmp_path) as c:
        w = c.workers[0]
        st = w.data_server.stats
        rfs = _remote_fs(c)
        try:
            rng = np.random.default_rng(11)
            first = rng.integers(0, 256, (3 << 20) + 1, dtype=np.uint8)
            rfs.write_file("/t/first", first, write_type="THROUGH")
            assert st.ufs_write_streams == 0                 # Python servicer, mount registered
            assert len(w.data_server.ufs_roots) == 1
            data = rng.integers(0, 256, (9 << 20) + 7, dtype=np.uint8)
            rfs.write_file("/t/second", data, write_type="THROUGH")
            rfs.write_file("/t/deep/third", data[:12345], write_type="CACHE_THROUGH")
            assert st.ufs_write_streams == 2
            assert st.ufs_write_bytes == data.nbytes + 12345
            with open(os.path.join(c.ufs_root, "t", "second"), "rb") as f:
                assert f.read() == data.tobytes()
            assert rfs.read_file("/t/deep/third") == data[:12345].tobytes()
            assert rfs.read_file("/t/first") == first.tobytes()
            assert not [n for n in os.listdir(os.path.join(c.ufs_root, "t")) if n.endswith(".tmp")]
            assert rfs.get_status("/t/second").is_persisted
            # the root confinement of the native path
            roots = w.data_server.ufs_roots
            mid = rfs.get_status("/t/second").mountId
            assert roots.resolve(mid, os.path.join(c.ufs_root, "t", "x")) is not None
            assert roots.resolve(mid, "file://" + os.path.join(c.ufs_root, "t", "x")) is not None
            assert roots.resolve(mid, os.path.join(c.ufs_root, "..", "x")) is None
            assert roots.resolve(mid, "/etc/passwd") is None
            assert roots.resolve(mid + 1000, os.path.join(c.ufs_root, "x")) is None
        finally:
            rfs.close()


def test_parallel_block_reads_into_host_buffers(tmp_path):
    """A host read spanning several remote blocks reads them at once, one native ReadBlock
    stream each; the stream position moves past the read, and a positioned read does not."""
    with _cluster(tmp_path) as c:
        fs = c.client()
        data = np.random.default_rng(14).integers(0, 256, (19 << 20) + 77, dtype=np.uint8)
        fs.write_file("/pr", data, write_type="MUST_CACHE")
        w = c.workers[0]
        for par in ("4", "1"):
            rfs = _remote_fs(c, **{"alluxio.user.device.read.parallelism": par})
            try:
                n0 = w.data_server.stats.streams
                buf = np.zeros((13 << 20) + 5, dtype=np.uint8)
                with rfs.open_file("/pr") as f:
                    f.seek((2 << 20) + 3)
                    assert f.read_into(buf) == len(buf)
                    assert f.tell() == (2 << 20) + 3 + len(buf)
                    assert f.read(10) == data[f.tell() - 10:f.tell()].tobytes()
                    assert f.pread(1, buf[:(9 << 20)]) == 9 << 20
                    assert f.tell() == (15 << 20) + 18
                assert np.array_equal(buf[:(9 << 20)], data[1:(9 << 20) + 1])
                assert np.array_equal(buf[(9 << 20):], data[(11 << 20) + 3:(15 << 20) + 8])
                if par == "4":
                    # 4 blocks for the read_into, 3 for the pread, plus the position-keeping reader
                    assert w.data_server.stats.streams - n0 >= 7
            finally:
                rfs.close()


def test_cache_through_ufs_error_surfaces_from_helper_thread(tmp_path):
    """CACHE_THROUGH runs the UFS write beside the cache write on a helper thread: its failure
    is raised by write(), after both have finished with the caller's buffer."""
    with _cluster(tmp_path) as c:
        rfs = _remote_fs(c)
        try:
            data = np.random.default_rng(13).integers(0, 256, 1 << 20, dtype=np.uint8)
            f = rfs.create_file("/ct", write_type="CACHE_THROUGH")
            f.write(data)
            calls = []

            def boom(host):
                calls.append(len(host))
                raise OSError("UFS is gone")
            f._ufs.write = boom
            f._pair_write = lambda ptr, n: False     # the helper-thread path, not the native pair
            f._tee = False                           # ... nor the worker-side tee
            with pytest.raises(OSError, match="UFS is gone"):
                f.write(data)
            assert calls == [data.nbytes]
            f.cancel()
            assert f._beside is None
        finally:
            rfs.close()


def test_native_ufs_file_write_cancel_leaves_no_file(tmp_path):
    import os
    from alluxio_amd.proto import pb as _pb
    with _cluster(tmp_path) as c:
        w = c.workers[0]
        root = c.ufs_root
        w.data_server.ufs_roots.set(77, root)
        C = lib()
        target = os.path.join(root, "x", "cancelled")
        cmd = _pb.block.WriteRequestCommand(type=1, id=5, create_ufs_file_options=_pb.dataserver.CreateUfsFileOptions(
            ufs_path=target, mount_id=77, mode=0o600))
        data = np.random.default_rng(12).integers(0, 256, 2 << 20, dtype=np.uint8)
        s = C.GrpcBlockSink("127.0.0.1", w.data_server.port, 5, command=cmd.SerializeToString())
        s.write_ptr(data.ctypes.data, data.nbytes)
        s.cancel()
        deadline = time.time() + 5
        xdir = os.path.join(root, "x")
        # the parent is made by the pool task that opens the temp file: a cancel that wins the race
        # leaves no directory at all
        while os.path.isdir(xdir) and os.listdir(xdir):
            assert time.time() < deadline
            time.sleep(0.05)
        assert not os.path.exists(target)
        s = C.GrpcBlockSink("127.0.0.1", w.data_server.port, 5, command=cmd.SerializeToString())
        s.write_ptr(data.ctypes.data, data.nbytes)
        assert s.commit() == data.nbytes
        assert os.stat(target).st_mode & 0o777 == 0o600
        with open(target, "rb") as f:
            assert f.read() == data.tobytes()
        # a path outside the registered root is not written natively: the Python servicer
        # (UfsFileWriteHandler's behavior) takes the call
        bad = cmd.__class__.FromString(cmd.SerializeToString())
        bad.create_ufs_file_options.ufs_path = os.path.join(str(tmp_path), "outside")
        n0, d0 = w.data_server.stats.ufs_write_streams, w.data_server.stats.write_declined
        s = C.GrpcBlockSink("127.0.0.1", w.data_server.port, 6, command=bad.SerializeToString())
        s.write_ptr(data.ctypes.data, 1024)
        s.commit()
        assert w.data_server.stats.ufs_write_streams == n0
        assert w.data_server.stats.write_declined == d0 + 1


def test_parallel_block_writes_of_one_large_write(tmp_path):
    """One host write() spanning several blocks to a remote worker streams whole blocks at once
    (one WriteBlock each, ids taken in file order); the partial head and tail go sequentially."""
    with _cluster(tmp_path) as c:
        w = c.workers[0]
        for par in ("4", "1"):
            rfs = _remote_fs(c, **{"alluxio.user.block.size.bytes.default": "4MB",
                                   "alluxio.user.device.read.parallelism": par})
            try:
                data = np.random.default_rng(15).integers(0, 256, (29 << 20) + 11, dtype=np.uint8)
                n0 = w.data_server.stats.write_streams
                with rfs.create_file(f"/pw{par}", write_type="MUST_CACHE") as f:
                    f.write(data[:(1 << 20) + 3])          # a partial first block
                    f.write(data[(1 << 20) + 3:])          # fills it, then 6 whole blocks + a tail
                blocks = _blocks(rfs, f"/pw{par}")
                assert [n for _, n in blocks] == [4 << 20] * 7 + [(1 << 20) + 11]
                assert w.data_server.stats.write_streams - n0 == 8
                assert rfs.read_file(f"/pw{par}") == data.tobytes()
                assert rfs.get_status(f"/pw{par}").in_alluxio_percentage == 100
            finally:
                rfs.close()


def test_parallel_block_write_failure_fails_stream(tmp_path, monkeypatch):
    """A failure in one block of a parallel multi-block write commits none of the blocks, and the
    stream stays failed: a later write() raises and close() cancels the file instead of completing
    it with a hole."""
    import threading

    from alluxio_amd.client import streams
    with _cluster(tmp_path) as c:
        w = c.workers[0]
        rfs = _remote_fs(c, **{"alluxio.user.block.size.bytes.default": "4MB",
                               "alluxio.user.device.read.parallelism": "4"})
        orig = streams.GrpcBlockWriter.write_ptr
        calls = [0]
        lock = threading.Lock()

        def flaky(self, offset, ptr, length, kind):
            with lock:
                calls[0] += 1
                k = calls[0]
            if k == 2:
                raise IOError("injected block write failure")
            return orig(self, offset, ptr, length, kind)
        monkeypatch.setattr(streams.GrpcBlockWriter, "write_ptr", flaky)
        try:
            data = np.random.default_rng(16).integers(0, 256, 16 << 20, dtype=np.uint8)
            free0 = w.worker.native.dir_available(0)
            f = rfs.create_file("/pwfail", write_type="MUST_CACHE")
            with pytest.raises(IOError, match="injected"):
                f.write(data)
            assert calls[0] >= 2
            with pytest.raises(IOError, match="failed earlier"):
                f.write(data[:10])
            with pytest.raises(IOError, match="cancelled"):
                f.close()
            assert not rfs.exists("/pwfail")
            deadline = time.time() + 10                  # no block of it stays committed or open
            while w.worker.native.dir_available(0) != free0:
                assert time.time() < deadline
                time.sleep(0.05)
        finally:
            rfs.close()


def test_native_write_errors_and_cancel(tmp_path):
    with _cluster(tmp_path) as c:
        w = c.workers[0]
        port = w.data_server.port
        C = lib()
        data = np.random.default_rng(8).integers(0, 256, 2 << 20, dtype=np.uint8)
        s = C.GrpcBlockSink("127.0.0.1", port, 4242)
        s.write_ptr(data.ctypes.data, data.nbytes)
        assert s.commit() == data.nbytes
        assert w.worker.has_block(4242)
        # the same block again: ALREADY_EXISTS from the native server
        with pytest.raises(C.StoreError) as ei:
            s2 = C.GrpcBlockSink("127.0.0.1", port, 4242)
            s2.write_ptr(data.ctypes.data, data.nbytes)
            s2.commit()
        assert ei.value.args[0] == 2
        # cancelled mid-block: the temp block and its space go away
        free0 = w.worker.native.dir_available(0)
        s3 = C.GrpcBlockSink("127.0.0.1", port, 4343, reserve=4 << 20)
        s3.write_ptr(data.ctypes.data, data.nbytes)
        s3.cancel()
        deadline = time.time() + 5
        while w.worker.native.has_temp_block(4343) or w.worker.native.dir_available(0) != free0:
            assert time.time() < deadline
            time.sleep(0.05)
        assert not w.worker.has_block(4343)
        # the commit call is internal to the server: a client calling it is refused
        ch = grpc.insecure_channel(f"127.0.0.1:{port}")
        spec = SERVICES[BW]["NativeWriteCommit"]
        call = ch.unary_unary(spec.path, spec.request.SerializeToString, spec.response.FromString)
        with pytest.raises(grpc.RpcError) as ge:
            call(pb.block.NativeWriteCommitRequest(session_id=1, block_id=4242, length=1))
        assert ge.value.code() == grpc.StatusCode.PERMISSION_DENIED
        ch.close()


def test_short_circuit_write_into_shared_arena(tmp_path):
    """A same-node writer in another process (here: a client with in-process transport off)
    writes into the worker's shared DRAM arena directly (OpenDeviceWrite -> ArenaSink ->
    CommitDeviceWrite); the last block's over-reserved pages are returned at commit."""
    with _cluster(tmp_path) as c:
        w = c.workers[0]
        rfs = _remote_fs(c, **{"alluxio.user.short.circuit.enabled": "true",
                               "alluxio.user.block.size.bytes.default": "4MB"})
        try:
            free0 = w.worker.native.dir_available(0)
            ws0 = w.data_server.stats.write_streams
            data = np.random.default_rng(9).integers(0, 256, (9 << 20) + 77, dtype=np.uint8)
            with rfs.create_file("/sc", write_type="MUST_CACHE") as f:
                for i in range(0, len(data), 1 << 20):
                    f.write(data[i:i + (1 << 20)])
            blocks = _blocks(rfs, "/sc")
            assert [n for _, n in blocks] == [4 << 20, 4 << 20, (1 << 20) + 77]
            assert w.data_server.stats.write_streams == ws0        # nothing went over WriteBlock
            assert rfs.get_status("/sc").in_alluxio_percentage == 100
            assert rfs.read_file("/sc") == data.tobytes()
            page = 1 << 20
            used = sum(-(-n // page) * page for _, n in blocks)
            assert free0 - w.worker.native.dir_available(0) == used
            # an aborted short-circuit write leaves nothing behind
            from alluxio_amd.client.streams import IpcBlockWriter
            from alluxio_amd.client.context import worker_address_str
            wr = IpcBlockWriter(rfs.ctx, worker_address_str(w.worker.address), 999_999, 4 << 20)
            wr.write_ptr(0, data.ctypes.data, 1 << 20, 0)
            wr.cancel()
            assert not w.worker.native.has_temp_block(999_999) and not w.worker.has_block(999_999)
            assert free0 - w.worker.native.dir_available(0) == used
        finally:
            rfs.close()


def test_short_circuit_write_survives_session_timeout(tmp_path):
    """An open short-circuit write outlives alluxio.worker.session.timeout: the client's session
    keeper renews it (SessionHeartbeat), so the cleaner does not hand its reserved pages to another
    block while the writer still copies into them.  A handle nobody renews still expires."""
    from alluxio_amd.client.context import worker_address_str
    from alluxio_amd.client.streams import IpcBlockWriter
    with _cluster(tmp_path, {"alluxio.worker.session.timeout": "600ms"}) as c:
        w = c.workers[0]
        rfs = _remote_fs(c, **{"alluxio.user.short.circuit.enabled": "true",
                               "alluxio.worker.session.timeout": "600ms"})
        try:
            addr = worker_address_str(w.worker.address)
            rng = np.random.default_rng(11)
            data = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
            wr = IpcBlockWriter(rfs.ctx, addr, 777_001, 3 << 20)
            wr.write_ptr(0, data.ctypes.data, 1 << 20, 0)
            for _ in range(3):                               # cleaner passes, each past the timeout
                time.sleep(0.7)
                assert wr.session not in w.worker.cleanup_expired_sessions()
            assert w.worker.native.has_temp_block(777_001)
            other = rng.integers(0, 256, 4 << 20, dtype=np.uint8)
            rfs.write_file("/other", other, write_type="MUST_CACHE")   # takes free pages now
            wr.write_ptr(1 << 20, data.ctypes.data + (1 << 20), 2 << 20, 0)
            wr.commit()
            assert w.worker.has_block(777_001)
            assert rfs.read_file("/other") == other.tobytes()
            assert rfs.ctx.session_keeper().renewals >= 2
            assert not rfs.ctx.session_keeper().open_sessions()
            # nobody renews this one: the cleaner reclaims it as before
            wr2 = IpcBlockWriter(rfs.ctx, addr, 777_002, 1 << 20)
            rfs.ctx.session_keeper().remove(addr, wr2.session)
            time.sleep(0.7)
            assert wr2.session in w.worker.cleanup_expired_sessions()
            assert not w.worker.native.has_temp_block(777_002)
            wr2.h = None
        finally:
            rfs.close()


def _read_request_call(port):
    ch = grpc.insecure_channel(f"127.0.0.1:{port}")
    spec = SERVICES[BW]["ReadBlock"]
    return ch, ch.stream_stream(spec.path, spec.request.SerializeToString, spec.response.FromString)


def test_native_cold_read_through(tmp_path):
    """Cold blocks of a local-directory mount are read through by the native data server once the
    mount is registered: each block streams to the client as its UFS slots land, is cached in the
    store and committed (master sees it) before the call ends.  A partial read streams without
    caching; a cancelled read-through leaves no temp block (UnderFileSystemBlockReader.java:251-274)."""
    with _cluster(tmp_path, {"alluxio.worker.ufs.ingest.chunk.size": "1MB", "alluxio.worker.ufs.ingest.depth": "2",
                             "alluxio.worker.network.reader.buffer.size": "1MB"}) as c:
        fs = c.client()
        rng = np.random.default_rng(21)
        files = {f"/cold/{k}": rng.integers(0, 256, (9 << 20) + 17 * (i + 1), dtype=np.uint8)
                 for i, k in enumerate("abcd")}
        for p, d in files.items():
            fs.write_file(p, d, write_type="CACHE_THROUGH")
        fs.free("/cold", recursive=True)
        w = c.workers[0]
        c.heartbeat_workers()
        assert not w.worker.native.block_ids(-1)
        st = w.data_server.stats
        rfs = _remote_fs(c)
        try:
            # the first cold read of the mount: resolved on demand (ResolveUfsMount), read natively
            d0, s0 = st.declined, st.cold_streams
            assert rfs.read_file("/cold/a") == files["/cold/a"].tobytes()
            assert len(w.data_server.ufs_roots) == 1
            assert st.declined == d0 and st.cold_streams - s0 == len(_blocks(rfs, "/cold/a"))
            d0, s0, c0 = st.declined, st.cold_streams, st.cold_cached
            z0 = st.zero_copy_frames
            free0 = w.worker.native.dir_available(0)
            assert rfs.read_file("/cold/b") == files["/cold/b"].tobytes()
            assert st.zero_copy_frames > z0            # UFS slots went to the socket without a copy
            nb = len(_blocks(rfs, "/cold/b"))
            # the timing the benches report per block: the readers' and the senders' side
            snd = st.send_timing["cold"]
            assert snd["streams"] >= nb and 0 < snd["first_ns"] <= snd["life_ns"]
            ct = st.cold_timing_ns
            assert ct["ufs_read"] > 0 and ct["first_slot"] > 0
            assert st.declined == d0                       # nothing went to Python
            assert st.cold_streams - s0 == nb
            deadline = time.time() + 10                    # the client may see its last byte before the
            while st.cold_cached - c0 < nb:                # commit that ends the call
                assert time.time() < deadline
                time.sleep(0.02)
            assert st.cold_cached - c0 == nb
            assert all(w.worker.has_block(b) for b, _ in _blocks(rfs, "/cold/b"))
            assert rfs.get_status("/cold/b").in_alluxio_percentage == 100
            assert free0 - w.worker.native.dir_available(0) >= files["/cold/b"].nbytes
            assert rfs.read_file("/cold/b") == files["/cold/b"].tobytes()   # now from the store
            # a positioned read inside a cold block: streamed, not cached
            (bid, blen), = _blocks(rfs, "/cold/c")[1:2]
            with rfs.open_file("/cold/c") as f:
                f.seek(blen + 1000)
                assert f.read(5000) == files["/cold/c"][blen + 1000:blen + 6000].tobytes()
            assert not w.worker.has_block(bid)
            # a read-through cancelled after its first chunk: the temp block is aborted
            st_d = rfs.get_status("/cold/d")
            (bid, blen) = _blocks(rfs, "/cold/d")[0]
            opts = pb.dataserver.OpenUfsBlockOptions(
                ufs_path=st_d.ufsPath, offset_in_file=0, block_size=blen, mountId=st_d.mountId)
            ch, call = _read_request_call(w.data_server.port)
            it = call(iter([pb.block.ReadRequest(block_id=bid, offset=0, length=blen, chunk_size=1 << 20,
                                                 open_ufs_block_options=opts)]))
            first = next(it)
            assert first.chunk.data == files["/cold/d"][:1 << 20].tobytes()
            it.cancel()
            ch.close()
            deadline = time.time() + 10
            while st.cold_active or w.worker.native.has_temp_block(bid):
                assert time.time() < deadline
                time.sleep(0.05)
            assert not w.worker.has_block(bid)
            # a client that goes away right after the last byte still leaves the block cached
            # (UnderFileSystemBlockReader.close commits a fully read block)
            import queue
            ch, call = _read_request_call(w.data_server.port)
            q = queue.Queue()
            q.put(pb.block.ReadRequest(block_id=bid, offset=0, length=blen, chunk_size=1 << 20,
                                       open_ufs_block_options=opts))
            it = call(iter(q.get, None))
            got = b""
            for _ in range(blen >> 20):                     # ack each chunk as it arrives
                got += next(it).chunk.data
                q.put(pb.block.ReadRequest(offset_received=len(got)))
            it.cancel()
            q.put(None)
            ch.close()
            assert got == files["/cold/d"][:blen].tobytes()
            deadline = time.time() + 10
            while not w.worker.has_block(bid):
                assert time.time() < deadline
                time.sleep(0.05)
            assert rfs.read_file("/cold/d") == files["/cold/d"].tobytes()
        finally:
            rfs.close()
            fs.close()


def test_native_cold_read_ahead_of_next_block(tmp_path):
    """A whole-block read-through reads the file's next block's first two UFS reads ahead once its
    own reads are done; the next block's cold stream sends those bytes (byte-exact) instead of
    reading the UFS.  A block the store already holds is not read ahead; the last block's read-ahead
    (past the end of the file) leaves nothing; with the key off nothing is read ahead."""
    extra = {"alluxio.worker.ufs.ingest.chunk.size": "1MB", "alluxio.worker.ufs.ingest.depth": "2",
             "alluxio.worker.network.reader.buffer.size": "1MB"}
    for enabled in (True, False):
        with _cluster(tmp_path / str(enabled), dict(
                extra, **{"alluxio.worker.data.server.native.ufs.readahead.enabled": str(enabled).lower()})) as c:
            fs = c.client()
            data = np.random.default_rng(31).integers(0, 256, (4 << 22) + 777, dtype=np.uint8)
            fs.write_file("/ra/f", data, write_type="CACHE_THROUGH")
            fs.free("/ra", recursive=True)
            w = c.workers[0]
            c.heartbeat_workers()
            st = w.data_server.stats
            rfs = _remote_fs(c)
            try:
                blocks = _blocks(rfs, "/ra/f")
                assert len(blocks) == 5
                # block 2 is cached already: block 1's stream does not read it ahead
                with rfs.open_file("/ra/f") as f:
                    f.seek(2 << 22)
                    assert f.read(4 << 20) == data[2 << 22:3 << 22].tobytes()
                deadline = time.time() + 10
                while not w.worker.has_block(blocks[2][0]) or st.cold_active:   # its read-ahead done too
                    assert time.time() < deadline
                    time.sleep(0.02)
                h0, b0, c0 = st.cold_readahead_hits, st.cold_readahead_bytes, st.cold_bytes
                assert b0 == (2 << 20 if enabled else 0)        # block 2 read block 3's first two reads
                got = b""
                with rfs.open_file("/ra/f") as f:
                    for _ in blocks:                  # one block at a time, the read-ahead lands between
                        got += f.read(4 << 20)
                        while st.cold_active:
                            time.sleep(0.01)
                        time.sleep(0.1)
                assert got == data.tobytes()
                hits, ahead = st.cold_readahead_hits - h0, st.cold_readahead_bytes - b0
                if enabled:
                    # blocks 1 and 3 start from read-ahead bytes: block 0 reads block 1's first two
                    # reads ahead, block 3 block 4's (777 bytes: shorter than one chunk, nothing);
                    # block 1 skips the cached block 2
                    assert hits == 4 and ahead == 2 << 20
                else:
                    assert hits == 0 and ahead == 0
                assert st.cold_bytes - c0 == data.nbytes - (4 << 20)   # every streamed byte counted once
                deadline = time.time() + 10
                while not all(w.worker.has_block(b) for b, _ in blocks):
                    assert time.time() < deadline
                    time.sleep(0.02)
                assert rfs.read_file("/ra/f") == data.tobytes()
                if enabled:
                    # a file rewritten under the same path has new block ids: the old file's
                    # read-ahead bytes are never sent for it
                    old = np.random.default_rng(32).integers(0, 256, 3 << 22, dtype=np.uint8)
                    fs.write_file("/ra/g", old, write_type="CACHE_THROUGH")
                    fs.free("/ra/g")
                    c.heartbeat_workers()
                    with rfs.open_file("/ra/g") as f:
                        assert f.read(4 << 20) == old[:4 << 20].tobytes()
                    while st.cold_active:
                        time.sleep(0.01)
                    b1, h1 = st.cold_readahead_bytes, st.cold_readahead_hits
                    assert b1 > b0 + (2 << 20)          # block 1 of the old file was read ahead
                    fs.delete("/ra/g")
                    new = np.random.default_rng(33).integers(0, 256, 3 << 22, dtype=np.uint8)
                    fs.write_file("/ra/g", new, write_type="CACHE_THROUGH")
                    fs.free("/ra/g")
                    c.heartbeat_workers()
                    rfs.close()
                    rfs = _remote_fs(c)
                    with rfs.open_file("/ra/g") as f:
                        f.seek(4 << 20)
                        assert f.read(4 << 20) == new[4 << 20:8 << 20].tobytes()
                    assert st.cold_readahead_hits == h1
            finally:
                rfs.close()
                fs.close()


def test_native_cold_read_through_s3(tmp_path):
    """Cold blocks of an S3 mount (native BlobServer endpoint) are read through by the data server's
    own signed ranged GETs once the first read in Python registered the mount."""
    srv = lib().BlobServer(str(tmp_path / "blobs"), "127.0.0.1", 0)
    srv.start()
    try:
        base = f"http://127.0.0.1:{srv.port}"
        import requests
        assert requests.put(base + "/bkt").status_code == 200
        rng = np.random.default_rng(22)
        objs = {k: rng.integers(0, 256, (6 << 20) + 5 * i, dtype=np.uint8) for i, k in enumerate(("x", "y"))}
        for k, d in objs.items():
            assert requests.put(f"{base}/bkt/ds/{k}", data=d.tobytes()).status_code == 200
        with _cluster(tmp_path) as c:
            fs = c.client()
            fs.mount("/s3", "s3://bkt/ds", properties={"alluxio.underfs.s3.endpoint": base,
                                                       "s3a.accessKeyId": "AKID", "s3a.secretKey": "sk"})
            w = c.workers[0]
            st = w.data_server.stats
            rfs = _remote_fs(c)
            try:
                assert rfs.read_file("/s3/x") == objs["x"].tobytes()          # Python, registers the mount
                mid = rfs.get_status("/s3/y").mountId
                assert w.data_server.ufs_roots.resolve_s3(mid, "s3://bkt/ds/y") == ("bkt", "ds/y")
                d0, s0, b0 = st.declined, st.cold_streams, st.cold_bytes
                assert rfs.read_file("/s3/y") == objs["y"].tobytes()
                nb = len(_blocks(rfs, "/s3/y"))
                assert st.declined == d0 and st.cold_streams - s0 == nb
                assert st.cold_bytes - b0 == objs["y"].nbytes
                deadline = time.time() + 10
                while not all(w.worker.has_block(b) for b, _ in _blocks(rfs, "/s3/y")):
                    assert time.time() < deadline
                    time.sleep(0.02)
            finally:
                rfs.close()
                fs.close()
    finally:
        srv.stop()


def test_sigv4_matches_python_signer():
    import datetime

    from alluxio_amd.underfs import s3
    cl = s3.S3Client("http://127.0.0.1:9000", "AKID", "SECRET/KEY+x", "eu-west-1")
    when = datetime.datetime(2024, 5, 6, 7, 8, 9, tzinfo=datetime.timezone.utc)

    class Fixed(datetime.datetime):
        @classmethod
        def now(cls, tz=None):
            return when
    real = s3.datetime.datetime
    s3.datetime.datetime = Fixed
    try:
        for path in ("/bkt/a b/c+d.bin", "/bkt/plain/key", "/bkt/ü/x"):
            h = cl._headers("GET", path, {}, s3._EMPTY_SHA)
            lines = lib().sigv4_headers("127.0.0.1:9000", "AKID", "SECRET/KEY+x", "eu-west-1", "GET", path, "",
                                        s3._EMPTY_SHA, "20240506T070809Z")
            got = dict(line.split(": ", 1) for line in lines.strip().split("\r\n"))
            assert got["authorization"] == h["authorization"]
    finally:
        s3.datetime.datetime = real
    import hashlib
    for data in (b"", b"abc", bytes(range(256)) * 300):
        assert lib().sha256_hex(data) == hashlib.sha256(data).hexdigest()


def test_ack_beyond_sent_bytes_does_not_stall(tmp_path):
    """An offset_received past what was sent is clamped (it used to wrap the unsigned window test
    and park the call, read lock held, forever)."""
    import threading
    with _cluster(tmp_path, {"alluxio.worker.network.reader.buffer.size": "1MB"}) as c:
        fs = c.client()
        data = np.random.default_rng(23).integers(0, 256, 4 << 20, dtype=np.uint8)
        fs.write_file("/ack", data, write_type="MUST_CACHE")
        (bid, blen), = _blocks(fs, "/ack")
        got_first = threading.Event()

        def reqs():
            yield pb.block.ReadRequest(block_id=bid, offset=0, length=blen, chunk_size=256 << 10)
            got_first.wait(10)
            yield pb.block.ReadRequest(offset_received=1 << 40)
            for k in range(1, 40):                          # then honest acks, chunk by chunk
                time.sleep(0.02)
                yield pb.block.ReadRequest(offset_received=min(blen, k * (256 << 10)))
        ch, call = _read_request_call(c.workers[0].data_server.port)
        out = bytearray()
        for r in call(reqs(), timeout=20):
            out += r.chunk.data
            got_first.set()
        ch.close()
        assert bytes(out) == data.tobytes()
        fs.close()


def test_native_s3_through_writes(tmp_path):
    """THROUGH writes of a remote client into an S3 mount: once the mount is registered, the data
    server streams each file as a multipart upload itself (parts of the mount's partition size on
    upload threads, at most buffer.size / part in flight, request window held back meanwhile),
    completes it at the client's half-close and aborts it when the client goes away."""
    import requests
    srv = lib().BlobServer(str(tmp_path / "blobs"), "127.0.0.1", 0)
    srv.start()
    try:
        base = f"http://127.0.0.1:{srv.port}"
        assert requests.put(base + "/bkt").status_code == 200
        assert requests.put(base + "/bkt/out/").status_code == 200
        with _cluster(tmp_path) as c:
            fs = c.client()
            fs.mount("/s3", "s3://bkt/out", properties={
                "alluxio.underfs.s3.endpoint": base,
                "alluxio.underfs.s3.streaming.upload.partition.size": "1MB",
                "alluxio.underfs.object.store.upload.buffer.size": "2MB"})
            w = c.workers[0]
            st = w.data_server.stats
            rfs = _remote_fs(c)
            try:
                rng = np.random.default_rng(31)
                first = rng.integers(0, 256, (3 << 20) + 5, dtype=np.uint8)
                rfs.write_file("/s3/first", first, write_type="THROUGH")      # Python; registers the mount
                assert requests.get(base + "/bkt/out/first").content == first.tobytes()
                n0, b0 = st.ufs_write_streams, st.ufs_write_bytes
                big = rng.integers(0, 256, (13 << 20) + 77, dtype=np.uint8)
                rfs.write_file("/s3/big", big, write_type="THROUGH")
                small = rng.integers(0, 256, 1000, dtype=np.uint8)
                rfs.write_file("/s3/small", small, write_type="CACHE_THROUGH")
                assert st.ufs_write_streams - n0 == 2
                assert st.ufs_write_bytes - b0 == big.nbytes + small.nbytes
                assert requests.get(base + "/bkt/out/big").content == big.tobytes()
                assert requests.get(base + "/bkt/out/small").content == small.tobytes()
                assert rfs.read_file("/s3/big") == big.tobytes()
                assert requests.get(base + "/bkt", params={"uploads": ""}).text.count("<Upload>") == 0
                # a writer that goes away mid-file: its upload is aborted, no object appears
                f = rfs.create_file("/s3/gone", write_type="THROUGH")
                f.write(rng.integers(0, 256, 5 << 20, dtype=np.uint8))
                f.cancel()
                deadline = time.time() + 10
                while requests.get(base + "/bkt", params={"uploads": ""}).text.count("<Upload>"):
                    assert time.time() < deadline
                    time.sleep(0.05)
                assert requests.head(base + "/bkt/out/gone").status_code == 404
                # CACHE_THROUGH into S3 with the tee: the bytes go once, to the block stream; the
                # worker's S3 stream fills its multipart parts from the store (AppendBlock), here
                # across block boundaries (4 MiB blocks, 1 MiB parts) and a partial last block
                tee0, b1 = st.ufs_tee_bytes, st.ufs_write_bytes
                ct = rng.integers(0, 256, (9 << 20) + 333, dtype=np.uint8)
                # auto (the default): teed only with enough CACHE_THROUGH streams open in the process
                auto = rng.integers(0, 256, (5 << 20) + 3, dtype=np.uint8)
                t_a = st.ufs_tee_bytes
                rfs.write_file("/s3/auto1", auto, write_type="CACHE_THROUGH", block_size=4 << 20)
                assert st.ufs_tee_bytes == t_a                       # 1 open stream < 8
                rfs.ctx.conf.set("alluxio.user.file.cache.through.tee.object.store.min.streams", "1")
                rfs.write_file("/s3/auto2", auto, write_type="CACHE_THROUGH", block_size=4 << 20)
                assert st.ufs_tee_bytes - t_a == auto.nbytes
                for k in ("auto1", "auto2"):
                    assert requests.get(base + "/bkt/out/" + k).content == auto.tobytes()
                rfs.ctx.conf.set("alluxio.user.file.cache.through.tee.object.store.enabled", "true")
                tee0, b1 = st.ufs_tee_bytes, st.ufs_write_bytes
                with rfs.create_file("/s3/ct", write_type="CACHE_THROUGH", block_size=4 << 20) as f:
                    for i in range(0, len(ct), 1 << 20):
                        f.write(ct[i:i + (1 << 20)])
                assert st.ufs_tee_bytes - tee0 == ct.nbytes and st.ufs_write_bytes - b1 == ct.nbytes
                assert requests.get(base + "/bkt/out/ct").content == ct.tobytes()
                # a persist job of a cached file into S3: the holding worker appends its blocks
                from alluxio_amd.job.persist import persist_file
                pz = rng.integers(0, 256, (6 << 20) + 7, dtype=np.uint8)
                rfs.write_file("/s3/pz", pz, write_type="MUST_CACHE", block_size=4 << 20)
                tee1 = st.ufs_tee_bytes
                assert persist_file(rfs, "/s3/pz") == pz.nbytes
                assert st.ufs_tee_bytes - tee1 == pz.nbytes
                assert requests.get(base + "/bkt/out/pz").content == pz.tobytes()
                # the client-copy fallback reaches the same bucket through the mount's options
                from alluxio_amd.conf import Configuration
                rfs.write_file("/s3/pz2", pz, write_type="MUST_CACHE", block_size=4 << 20)
                off = Configuration({"alluxio.job.persist.worker.append.enabled": "false"})
                tee2 = st.ufs_tee_bytes
                assert persist_file(rfs, "/s3/pz2", conf=off) == pz.nbytes
                assert st.ufs_tee_bytes == tee2
                assert requests.get(base + "/bkt/out/pz2").content == pz.tobytes()
                # bytes, a block, bytes on one S3 stream: the stream keeps file order across the
                # append (a half-filled part continues after the block; parts are 1 MiB)
                b1 = rng.integers(0, 256, (3 << 19), dtype=np.uint8)
                b2 = rng.integers(0, 256, 700_000, dtype=np.uint8)
                blk = rfs.get_status("/s3/pz").info.fileBlockInfos[0].blockInfo
                mix = rfs.create_file("/s3/mix", write_type="THROUGH")
                mix._ufs.write(b1)
                mix._ufs.append_block(blk.blockId, blk.length)
                mix._ufs.write(b2)
                mix._ufs.close()
                mix.cancel()                                   # drop the Alluxio entry, keep the object
                want = b1.tobytes() + pz.tobytes()[:blk.length] + b2.tobytes()
                assert requests.get(base + "/bkt/out/mix").content == want
                # the block vanished before the worker appended it: the upload is aborted, close fails
                g = rfs.create_file("/s3/ct2", write_type="CACHE_THROUGH", block_size=4 << 20)
                g.write(ct[:(5 << 20)])                     # block 0 appended, block 1 in progress
                orig = g._ufs.append_block

                def append_after_removal(block_id, length):
                    c.workers[0].native.remove_block(block_id)
                    orig(block_id, length)
                g._ufs.append_block = append_after_removal
                with pytest.raises(Exception):
                    g.close()
                deadline = time.time() + 10
                while requests.get(base + "/bkt", params={"uploads": ""}).text.count("<Upload>"):
                    assert time.time() < deadline
                    time.sleep(0.05)
                assert requests.head(base + "/bkt/out/ct2").status_code == 404
                assert st.store_tasks == 0          # no AppendBlock copy left using the store
            finally:
                rfs.close()
                fs.close()
    finally:
        srv.stop()


def test_bounded_ipc_open_times_out_and_client_falls_back(tmp_path, monkeypatch):
    """A HIP IPC import that does not return makes the arena unavailable after the deadline
    instead of hanging the reader (csrc/ipc.cpp ipc_open_bounded, stalled here by its test hook);
    the handle is not retried, and the map layer turns the timeout into UnavailableException so
    the block readers / writers fall back to the data port."""
    import subprocess
    import sys
    code = (
        "import os, sys, time\n"
        f"sys.path.insert(0, {str(__import__('os').path.dirname(__import__('os').path.dirname(__file__)))!r})\n"
        "from alluxio_amd.ops.native import lib\n"
        "h = bytes(range(64))\n"
        "lib()\n"
        "t0 = time.time()\n"
        "try:\n"
        "    lib().ipc_open_bounded(h, 0, 300)\n"
        "    print('opened')\n"
        "except TimeoutError as e:\n"
        "    print('timeout', round(time.time() - t0, 2))\n"
        "try:\n"
        "    lib().ipc_open_bounded(h, 0, 300)\n"
        "except TimeoutError as e:\n"
        "    print('again', 'before' in str(e))\n")
    env = dict(__import__('os').environ, ALLUXIO_AMD_IPC_OPEN_DELAY_MS="3000")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, env=env)
    lines = p.stdout.split()
    assert lines[0] == "timeout" and float(lines[1]) < 2.0, p.stdout + p.stderr[-2000:]
    assert lines[2:] == ["again", "True"]
    # the map layer: a timed-out import is an UnavailableException (callers use the data port)
    from alluxio_amd.parallel import ipc
    from alluxio_amd.utils.exceptions import UnavailableException

    class Stub:
        def ipc_open_bounded(self, handle, device, timeout_ms):
            raise TimeoutError("stuck")
    monkeypatch.setattr(ipc, "lib", lambda: Stub())
    with pytest.raises(UnavailableException):
        ipc.IpcMappings().open(b"x" * 64, 0)


def test_cache_through_pair_write_lands_in_cache_and_ufs(tmp_path):
    """CACHE_THROUGH from a remote client with native streams on both sides: each write goes to the
    cache block stream and the UFS_FILE stream in one native call (sink_write_pair); the bytes land
    in both, across block boundaries, and a failed UFS stream fails the write."""
    import os
    with _cluster(tmp_path) as c:
        rfs = _remote_fs(c)
        try:
            data = np.random.default_rng(21).integers(0, 256, (9 << 20) + 4097, dtype=np.uint8)
            with rfs.create_file("/pair", write_type="CACHE_THROUGH", block_size=4 << 20) as f:
                f._tee = False                       # the paired path (the tee has its own test)
                used = []
                orig = f._pair_write
                f._pair_write = lambda ptr, n: used.append(orig(ptr, n)) or used[-1]
                for i in range(0, len(data), 1 << 20):
                    f.write(data[i:i + (1 << 20)])
            assert any(used)
            assert rfs.read_file("/pair") == data.tobytes()
            st = rfs.get_status("/pair")
            assert st.info.inAlluxioPercentage == 100
            ufs_path = st.info.ufsPath
            with open(ufs_path.replace("file://", ""), "rb") as fh:
                assert fh.read() == data.tobytes()
            # the UFS stream dies: the next paired write raises
            f2 = rfs.create_file("/pair2", write_type="CACHE_THROUGH", block_size=4 << 20)
            f2._tee = False
            f2.write(data[:1 << 20])
            f2._ufs._sink.cancel()
            with pytest.raises(Exception):
                for _ in range(8):
                    f2.write(data[:1 << 20])
            f2.cancel()
        finally:
            rfs.close()


def test_cache_through_tee_sends_bytes_once(tmp_path):
    """CACHE_THROUGH with the cache block and the UFS stream on one worker: the bytes go only to the
    block stream; after each block commits, the UFS stream appends it from the worker's store
    (AppendBlock).  The file is byte-exact in the cache and in the UFS, across block boundaries and
    a partial last block; a block that vanished before its append fails the file's UFS stream."""
    with _cluster(tmp_path) as c:
        rfs = _remote_fs(c)
        try:
            data = np.random.default_rng(23).integers(0, 256, (9 << 20) + 777, dtype=np.uint8)
            # the mount's first UFS_FILE stream runs in the Python servicer (which registers the
            # mount natively): it handles AppendBlock too
            with rfs.create_file("/tee0", write_type="CACHE_THROUGH", block_size=4 << 20) as f:
                for i in range(0, len(data), 1 << 20):
                    f.write(data[i:i + (1 << 20)])
            st0 = rfs.get_status("/tee0")
            with open(st0.info.ufsPath.replace("file://", ""), "rb") as fh:
                assert fh.read() == data.tobytes()
            st0 = c.workers[0].data_server.stats
            tee0, ufs0 = st0.ufs_tee_bytes, st0.ufs_write_bytes
            with rfs.create_file("/tee", write_type="CACHE_THROUGH", block_size=4 << 20) as f:
                pairs = []
                f._pair_write = lambda ptr, n: pairs.append(n) or False
                for i in range(0, len(data), 1 << 20):
                    f.write(data[i:i + (1 << 20)])
            assert not pairs                                    # never the two-stream path
            st = c.workers[0].data_server.stats
            assert st.ufs_tee_bytes - tee0 == len(data)
            assert st.ufs_write_bytes - ufs0 == len(data)
            assert rfs.read_file("/tee") == data.tobytes()
            status = rfs.get_status("/tee")
            assert status.info.inAlluxioPercentage == 100
            with open(status.info.ufsPath.replace("file://", ""), "rb") as fh:
                assert fh.read() == data.tobytes()
            # the block is gone before the worker appends it: the UFS stream (and close) fail
            g = rfs.create_file("/tee2", write_type="CACHE_THROUGH", block_size=4 << 20)
            g.write(data[:1 << 20])
            bid = g._block_id
            orig = g._ufs.append_block

            def append_after_removal(block_id, length):
                c.workers[0].native.remove_block(block_id)
                orig(block_id, length)
            g._ufs.append_block = append_after_removal
            with pytest.raises(Exception):
                g.close()
            assert bid is not None
        finally:
            rfs.close()


@pytest.mark.gpu
def test_cache_through_tee_from_hbm_is_byte_exact(tmp_path):
    """The CACHE_THROUGH tee with the cache in HBM: each committed block is copied out of device
    memory in pipelined 8 MiB pieces (two pinned buffers, the pool thread's own stream) and appended
    to the UFS file; several writers at once, partial last blocks, bytes checked in the UFS and the
    cache."""
    import concurrent.futures as cf
    with _cluster(tmp_path, {"alluxio.worker.tieredstore.level0.dirs.path": "hbm:0",
                             "alluxio.worker.tieredstore.level0.dirs.quota": "1GB",
                             "alluxio.worker.hbm.page.size": "2MB"}) as c:
        rfs = _remote_fs(c)
        try:
            # the mount's first UFS stream runs in the Python servicer (which then registers the
            # mount natively): its AppendBlock reads the block out of HBM through the store
            warm = np.random.default_rng(4).integers(0, 256, (9 << 20) + 5, dtype=np.uint8)
            rfs.write_file("/warm", warm, write_type="CACHE_THROUGH", block_size=4 << 20)
            with open(rfs.get_status("/warm").info.ufsPath.replace("file://", ""), "rb") as fh:
                assert fh.read() == warm.tobytes()
            st = c.workers[0].data_server.stats
            tee0 = st.ufs_tee_bytes
            rng = np.random.default_rng(5)
            datas = [rng.integers(0, 256, (37 << 20) + 4097 * i, dtype=np.uint8) for i in range(4)]

            def put(i):
                with rfs.create_file(f"/hbm{i}", write_type="CACHE_THROUGH", block_size=16 << 20) as f:
                    for o in range(0, len(datas[i]), 1 << 20):
                        f.write(datas[i][o:o + (1 << 20)])
            with cf.ThreadPoolExecutor(4) as ex:
                list(ex.map(put, range(4)))
            assert st.ufs_tee_bytes - tee0 == sum(len(d) for d in datas)
            for i, d in enumerate(datas):
                status = rfs.get_status(f"/hbm{i}")
                with open(status.info.ufsPath.replace("file://", ""), "rb") as fh:
                    assert fh.read() == d.tobytes()
                assert rfs.read_file(f"/hbm{i}") == d.tobytes()
        finally:
            rfs.close()


def test_persist_appends_blocks_on_the_holding_worker(tmp_path):
    """A persist job of a file cached on one worker moves no bytes through the job process: the
    worker appends each block from its store to the file's UFS stream (AppendBlock) and renames
    the temp file into place; byte-exact, and counted as tee bytes by the native data server."""
    from alluxio_amd.job.persist import persist_file
    with _cluster(tmp_path) as c:
        rfs = _remote_fs(c)
        try:
            rfs.write_file("/warm", b"w" * 100, write_type="CACHE_THROUGH")   # registers the mount natively
            data = np.random.default_rng(8).integers(0, 256, (10 << 20) + 321, dtype=np.uint8)
            rfs.write_file("/ap/f", data, write_type="ASYNC_THROUGH", block_size=4 << 20)
            st = c.workers[0].data_server.stats
            tee0 = st.ufs_tee_bytes
            assert persist_file(rfs, "/ap/f") == len(data)
            assert st.ufs_tee_bytes - tee0 == len(data)
            ufs_path = rfs.get_status("/ap/f").info.ufsPath.replace("file://", "")
            with open(ufs_path, "rb") as fh:
                assert fh.read() == data.tobytes()
            assert not [n for n in os.listdir(os.path.dirname(ufs_path)) if ".tmp" in n]
        finally:
            rfs.close()


@pytest.mark.gpu
def test_persist_from_hbm_to_local_and_s3_is_byte_exact(tmp_path):
    """Worker-side persist with the blocks in HBM: the local UFS stream and the S3 multipart
    stream both copy every block out of device memory (pinned pieces on the pool thread's own
    stream) into the persisted file / object, byte-exact, while 3 persists run at once."""
    import concurrent.futures as cf

    import requests

    from alluxio_amd.job.persist import persist_file
    srv = lib().BlobServer(str(tmp_path / "blobs"), "127.0.0.1", 0)
    srv.start()
    try:
        base = f"http://127.0.0.1:{srv.port}"
        assert requests.put(base + "/bkt").status_code == 200
        assert requests.put(base + "/bkt/out/").status_code == 200
        with _cluster(tmp_path, {"alluxio.worker.tieredstore.level0.dirs.path": "hbm:0",
                                 "alluxio.worker.tieredstore.level0.dirs.quota": "1GB",
                                 "alluxio.worker.hbm.page.size": "2MB"}) as c:
            fs = c.client()
            fs.mount("/s3", "s3://bkt/out", properties={
                "alluxio.underfs.s3.endpoint": base,
                "alluxio.underfs.s3.streaming.upload.partition.size": "8MB",
                "alluxio.underfs.object.store.upload.buffer.size": "32MB"})
            rfs = _remote_fs(c)
            try:
                rfs.write_file("/warm", b"w" * 100, write_type="CACHE_THROUGH")
                rfs.write_file("/s3/warm", b"w" * 100, write_type="THROUGH")     # registers both mounts natively
                st = c.workers[0].data_server.stats
                rng = np.random.default_rng(12)
                datas = {f"/p{i}": rng.integers(0, 256, (21 << 20) + 999 * i, dtype=np.uint8) for i in range(3)}
                datas.update({f"/s3/o{i}": rng.integers(0, 256, (19 << 20) + 77 * i, dtype=np.uint8) for i in range(3)})
                for p, d in datas.items():
                    rfs.write_file(p, d, write_type="MUST_CACHE", block_size=8 << 20)
                tee0 = st.ufs_tee_bytes
                with cf.ThreadPoolExecutor(3) as ex:
                    assert list(ex.map(lambda p: persist_file(rfs, p), datas)) == [d.nbytes for d in datas.values()]
                assert st.ufs_tee_bytes - tee0 == sum(d.nbytes for d in datas.values())
                for p, d in datas.items():
                    if p.startswith("/s3/"):
                        got = requests.get(base + "/bkt/out/" + p[4:]).content
                    else:
                        with open(rfs.get_status(p).info.ufsPath.replace("file://", ""), "rb") as fh:
                            got = fh.read()
                    assert got == d.tobytes(), p
            finally:
                rfs.close()
                fs.close()
    finally:
        srv.stop()
