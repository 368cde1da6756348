"""Timeouts, retries and cancellation of the object-store data path, driven by the native
BlobServer's fault injection (503 SlowDown, connection reset, silent server, body stall).

Reference behaviour pinned here: S3AUnderFileSystem.java:150-191 gives the AWS client
``alluxio.underfs.s3.socket.timeout`` / ``request.timeout`` / ``max.error.retry`` (AWS SDK default 3
retries of 5xx, throttling and I/O errors); ObjectUnderFileSystem.java:654,1153 retries
open / status calls with the eventual-consistency back-off; UnderFileSystemBlockReader aborts the
temp block of a read-through that fails (BlockReadHandler / UfsInputStreamCache).
"""
import os
import time

import numpy as np
import pytest
import requests

from alluxio_amd.ops.native import lib

from test_data_server import _blocks, _cluster, _remote_fs

pytestmark = pytest.mark.skipif(not lib().FrameRpcServer.grpc_available(), reason="libnghttp2 not present")

MB = 1 << 20


@pytest.fixture
def blob(tmp_path):
    srv = lib().BlobServer(str(tmp_path / "blobs"), "127.0.0.1", 0)
    srv.start()
    base = f"http://127.0.0.1:{srv.port}"
    assert requests.put(base + "/bkt").status_code == 200
    yield srv, base
    srv.stop()


def _put(base, key, data):
    assert requests.put(f"{base}/bkt/{key}", data=bytes(data)).status_code == 200


def _reader(srv, **kw):
    opts = dict(socket_timeout_ms=400, request_timeout_ms=3000, max_retries=3, backoff_base_ms=5, backoff_max_ms=20)
    opts.update(kw)
    return lib().HttpRangeReader("127.0.0.1", srv.port, 8, **opts)


def _get(rd, key, off, n, parallel=1):
    buf = np.zeros(n, dtype=np.uint8)
    got = rd.get_into(f"/bkt/{key}", f"Host: 127.0.0.1\r\n", off, n, buf.ctypes.data, parallel, 64 << 10)
    return got, buf


@pytest.mark.parametrize("kind", [1, 2])
def test_native_get_retries_503_and_reset_byte_exact(blob, kind):
    srv, base = blob
    data = np.random.default_rng(kind).integers(0, 256, 3 * MB + 17, dtype=np.uint8)
    _put(base, "obj", data)
    rd = _reader(srv)
    srv.inject(kind, "GET", 1, 2)                 # the next two GETs fail, the third succeeds
    got, buf = _get(rd, "obj", 5, len(data) - 5)
    assert got == len(data) - 5 and np.array_equal(buf, data[5:])
    assert srv.injected == 2 and rd.retries == 2
    # every sub-range of a parallel read retries by itself
    srv.inject(kind, "GET", 2, 1)
    got, buf = _get(rd, "obj", 0, len(data), parallel=4)
    assert got == len(data) and np.array_equal(buf, data)


def test_native_get_gives_up_after_max_retries(blob):
    srv, base = blob
    _put(base, "obj", b"x" * 1000)
    rd = _reader(srv, max_retries=2)
    srv.inject(1, "GET", 1, 10)
    got, _ = _get(rd, "obj", 0, 1000)
    assert got == -503 and rd.retries == 2 and srv.injected == 3


@pytest.mark.parametrize("kind", [3, 4])
def test_native_get_stall_times_out_within_the_limit(blob, kind):
    """A silent server (no response / half a body then nothing) ends the call with the timeout code
    after the socket timeout of each attempt, never later than the request timeout."""
    srv, base = blob
    data = np.random.default_rng(9).integers(0, 256, 4 * MB, dtype=np.uint8)
    _put(base, "obj", data)
    rd = _reader(srv, socket_timeout_ms=300, request_timeout_ms=1500, max_retries=10)
    srv.inject(kind, "GET", 1, 100, stall_ms=20000)
    t0 = time.monotonic()
    got, _ = _get(rd, "obj", 0, len(data))
    el = time.monotonic() - t0
    assert got == -2, got                          # kHttpTimeout
    assert 0.25 < el < 2.5, el
    assert rd.timeouts >= 1
    srv.clear_faults()
    got, buf = _get(rd, "obj", 0, len(data))       # the client is still usable
    assert got == len(data) and np.array_equal(buf, data)


def test_native_connect_timeout_to_a_blackhole():
    """A connect that never completes is bounded by the connect timeout (10.255.255.1 drops SYNs on
    most networks; a refused / unreachable address fails at once -- both end well inside the limit)."""
    rd = lib().HttpRangeReader("10.255.255.1", 9, 2, connect_timeout_ms=300, socket_timeout_ms=300,
                               request_timeout_ms=1000, max_retries=1, backoff_base_ms=5, backoff_max_ms=10)
    buf = np.zeros(10, dtype=np.uint8)
    t0 = time.monotonic()
    got = rd.get_into("/b/k", "Host: x\r\n", 0, 10, buf.ctypes.data, 1, 64 << 10)
    assert got in (-1, -2)
    assert time.monotonic() - t0 < 2.0


def test_python_s3_client_retries_and_times_out(blob, tmp_path):
    from alluxio_amd.underfs.s3 import S3UnderFileSystem
    srv, base = blob
    ufs = S3UnderFileSystem("s3://bkt/p", properties={
        "alluxio.underfs.s3.endpoint": base, "alluxio.underfs.s3.socket.timeout": "400ms",
        "alluxio.underfs.s3.request.timeout": "2s", "alluxio.underfs.s3.max.error.retry": "2",
        "alluxio.underfs.s3.native.reader.enabled": "false",
        "alluxio.underfs.eventual.consistency.retry.max.num": "1"})
    assert ufs.max_retries == 2 and ufs.socket_timeout_ms == 400 and ufs.request_timeout_ms == 2000
    data = os.urandom(300_000)
    srv.inject(1, "PUT", 1, 1)                    # SlowDown once: retried
    with ufs.create("s3://bkt/p/a") as w:
        w.write(data)
    srv.inject(2, "HEAD", 1, 1)                   # reset once: retried
    assert ufs.get_status("s3://bkt/p/a").content_length == len(data)
    with ufs.open("s3://bkt/p/a") as f:
        assert f.read() == data
    assert ufs.client.retries == 2
    srv.inject(3, "HEAD", 1, 100, stall_ms=10000)
    t0 = time.monotonic()
    with pytest.raises(TimeoutError):
        ufs.get_status("s3://bkt/p/a")
    assert time.monotonic() - t0 < 3.0            # request timeout (2 s) + one socket timeout
    srv.clear_faults()
    # retryOnException of the object store base: an I/O error of a status call is tried again
    ufs2 = S3UnderFileSystem("s3://bkt/p", properties={
        "alluxio.underfs.s3.endpoint": base, "alluxio.underfs.s3.max.error.retry": "0",
        "alluxio.underfs.eventual.consistency.retry.base.sleep": "5ms",
        "alluxio.underfs.eventual.consistency.retry.max.num": "3"})
    srv.inject(1, "HEAD", 1, 2)
    assert ufs2.get_status("s3://bkt/p/a").content_length == len(data)


def _s3_cluster(tmp_path, base, cluster_conf=None, **mount_props):
    props = {"alluxio.underfs.s3.endpoint": base, "s3a.accessKeyId": "AKID", "s3a.secretKey": "sk",
             "alluxio.underfs.s3.socket.timeout": "400ms", "alluxio.underfs.s3.request.timeout": "2s",
             "alluxio.underfs.s3.max.error.retry": "2", "alluxio.underfs.eventual.consistency.retry.max.num": "1"}
    props.update(mount_props)
    c = _cluster(tmp_path, cluster_conf)
    c.__enter__()
    fs = c.client()
    fs.mount("/s3", "s3://bkt/ds", properties=props)
    return c, fs


def test_native_cold_read_retries_and_stalls(blob, tmp_path):
    """Cold blocks read through natively: a 503 or a reset of one GET is retried byte-exact (no
    Python detour); a stalled store fails the stream with UNAVAILABLE within the configured
    timeout and leaves no temp block; the worker then serves the next read normally."""
    srv, base = blob
    rng = np.random.default_rng(3)
    objs = {k: rng.integers(0, 256, 6 * MB + 11 * i, dtype=np.uint8) for i, k in enumerate("wxyz")}
    objs["z"] = rng.integers(0, 256, 24 * MB + 5, dtype=np.uint8)   # reads of 1, 8, 8, 7 MiB
    for k, d in objs.items():
        _put(base, "ds/" + k, d)
    # one block per object and one GET per read (no sub-range split): the Nth GET is the Nth read
    # (no next-block read-ahead, which would add GETs past each object's end)
    c, fs = _s3_cluster(tmp_path, base, cluster_conf={"alluxio.user.block.size.bytes.default": "32MB",
                                                      "alluxio.worker.data.server.native.ufs.readahead.enabled": "false",
                                                      # the temp block exists once two reads landed
                                                      "alluxio.worker.data.server.native.ufs.create.after.reads": "2"},
                        **{"alluxio.underfs.s3.threads.max": "1"})
    rfs = _remote_fs(c)
    try:
        w = c.workers[0]
        st = w.data_server.stats
        assert rfs.read_file("/s3/w") == objs["w"].tobytes()        # Python: registers the mount
        for kind, key in ((1, "x"), (2, "y")):
            d0, s0 = st.declined, st.cold_streams
            srv.inject(kind, "GET", 1, 1)
            assert rfs.read_file("/s3/" + key) == objs[key].tobytes()
            assert st.declined == d0 and st.cold_streams > s0
        assert srv.injected == 2
        # a silent store: the stream fails within socket/request timeout (2 s + slack), UNAVAILABLE
        a0 = st.cold_aborted
        # from the 3rd GET on: the first two reads (one chunk, then a slot) land, the temp block
        # is created behind them, then the reads stall -- the block must be aborted, not left
        # behind
        srv.inject(3, "GET", 3, 1000, stall_ms=30000)
        t0 = time.monotonic()
        with pytest.raises(Exception) as ei:
            rfs.read_file("/s3/z")
        el = time.monotonic() - t0
        assert el < 8.0, el
        assert "UNAVAILABLE" in str(ei.value).upper() or "timed out" in str(ei.value), ei.value
        deadline = time.time() + 10
        while st.cold_active > 0:
            assert time.time() < deadline
            time.sleep(0.02)
        assert st.cold_aborted > a0
        for b, _ in _blocks(rfs, "/s3/z"):
            assert not w.worker.has_block(b) and not w.worker.native.has_temp_block(b)
        srv.clear_faults()
        assert rfs.read_file("/s3/z") == objs["z"].tobytes()
    finally:
        rfs.close()
        fs.close()
        c.__exit__(None, None, None)


def test_stopping_worker_during_stalled_cold_read_is_clean(blob, tmp_path):
    """Stopping the worker while a cold read waits on a silent store: the reader is cancelled (it
    polls the cancel flag while its GET waits), the stop returns promptly, and the reader -- which
    holds its own reference to the store -- drops its temp block before the store goes away."""
    srv, base = blob
    data = np.random.default_rng(5).integers(0, 256, 6 * MB, dtype=np.uint8)
    _put(base, "ds/a", data[:MB])
    _put(base, "ds/b", data)
    c, fs = _s3_cluster(tmp_path, base, **{"alluxio.underfs.s3.socket.timeout": "60s",
                                          "alluxio.underfs.s3.request.timeout": "120s"})
    rfs = _remote_fs(c)
    import threading
    errs = []
    try:
        w = c.workers[0]
        st = w.data_server.stats
        assert rfs.read_file("/s3/a") == data[:MB].tobytes()
        srv.inject(3, "GET", 1, 1000, stall_ms=60000)

        def reader():
            try:
                rfs.read_file("/s3/b")
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        t = threading.Thread(target=reader, daemon=True)
        t.start()
        deadline = time.time() + 10
        while st.cold_active == 0:
            assert time.time() < deadline
            time.sleep(0.01)
        time.sleep(0.3)
        t0 = time.monotonic()
        w.data_server.stop()
        assert time.monotonic() - t0 < 5.0
        assert st.cold_active == 0
        t.join(30)
    finally:
        srv.clear_faults()
        rfs.close()
        fs.close()
        c.__exit__(None, None, None)
    assert errs                                    # the read failed instead of hanging


def test_native_s3_upload_retries_then_aborts(blob, tmp_path):
    """A part PUT that fails once is sent again (the object is complete and byte-exact); a part
    that keeps failing past max.error.retry fails the write and aborts the multipart upload."""
    srv, base = blob
    assert requests.put(base + "/bkt/ds/").status_code == 200
    c, fs = _s3_cluster(tmp_path, base, **{"alluxio.underfs.s3.streaming.upload.partition.size": "1MB",
                                          "alluxio.underfs.object.store.upload.buffer.size": "2MB"})
    rfs = _remote_fs(c)
    try:
        st = c.workers[0].data_server.stats
        rng = np.random.default_rng(8)
        first = rng.integers(0, 256, 3 * MB + 5, dtype=np.uint8)
        rfs.write_file("/s3/first", first, write_type="THROUGH")          # registers the mount
        n0 = st.ufs_write_streams
        ok = rng.integers(0, 256, 5 * MB + 9, dtype=np.uint8)
        srv.inject(1, "PUT", 2, 1)                                        # part 2: SlowDown once
        rfs.write_file("/s3/ok", ok, write_type="THROUGH")
        assert st.ufs_write_streams - n0 == 1
        assert requests.get(base + "/bkt/ds/ok").content == ok.tobytes()
        srv.inject(2, "PUT", 2, 100)                                      # part 2 keeps resetting
        with pytest.raises(Exception):
            rfs.write_file("/s3/bad", ok, write_type="THROUGH")
        srv.clear_faults()
        deadline = time.time() + 10
        while requests.get(base + "/bkt", params={"uploads": ""}).text.count("<Upload>"):
            assert time.time() < deadline
            time.sleep(0.05)
        assert requests.head(base + "/bkt/ds/bad").status_code == 404
    finally:
        rfs.close()
        fs.close()
        c.__exit__(None, None, None)


def test_first_cold_read_of_a_mount_resolves_natively(blob, tmp_path):
    """No Python detour for the first cold read of a mount (WorkerUfsManager.java:56-65 resolves an
    unknown mount from the master): an S3 mount the data server can reach is resolved on the
    reader's pool thread and read natively; a mount it cannot reach (native reader off) is read
    once through the worker's Python UFS by the same native stream, then its reads go to Python."""
    srv, base = blob
    rng = np.random.default_rng(12)
    objs = {k: rng.integers(0, 256, 5 * MB + 7 * i, dtype=np.uint8) for i, k in enumerate("abcd")}
    for k, d in objs.items():
        _put(base, "ds/" + k, d)
        _put(base, "py/" + k, d)
    c, fs = _s3_cluster(tmp_path, base)
    fs.mount("/py", "s3://bkt/py", properties={"alluxio.underfs.s3.endpoint": base,
                                               "alluxio.underfs.s3.native.reader.enabled": "false"})
    rfs = _remote_fs(c)
    try:
        w = c.workers[0]
        st = w.data_server.stats
        d0, s0 = st.declined, st.cold_streams
        assert rfs.read_file("/s3/a") == objs["a"].tobytes()
        assert st.declined == d0 and st.cold_streams - s0 == len(_blocks(rfs, "/s3/a"))
        mid = rfs.get_status("/s3/a").mountId
        assert w.data_server.ufs_roots.resolve_s3(mid, "s3://bkt/ds/a") == ("bkt", "ds/a")
        # a Python-only mount: its first cold block is still a native stream, fed by ReadUfsRange
        # (the file's later blocks already go to Python)
        d0, s0 = st.declined, st.cold_streams
        assert rfs.read_file("/py/a") == objs["a"].tobytes()
        assert st.cold_streams - s0 >= 1 and st.declined - d0 < len(_blocks(rfs, "/py/a"))
        d1 = st.declined
        assert rfs.read_file("/py/b") == objs["b"].tobytes()        # now straight to Python
        assert st.declined > d1
    finally:
        rfs.close()
        fs.close()
        c.__exit__(None, None, None)
