"""Native S3 data path (csrc/http_blob.cpp): the S3 under file system receives ranged GETs straight
into the caller's buffer over pooled connections, split into parallel sub-ranges; BlobServer is an
S3-style endpoint over a directory tree (sendfile GETs) that the UFS contract passes against.
Reference behaviour: underfs/s3a/.../S3AUnderFileSystem.java, S3AInputStream.java (ranged reads)."""
import io
import os

import numpy as np
import pytest
import requests

from alluxio_amd.cli import ufs_contract
from alluxio_amd.ops.native import lib
from alluxio_amd.underfs.registry import create as create_ufs


@pytest.fixture
def blob(tmp_path):
    srv = lib().BlobServer(str(tmp_path / "blobs"), "127.0.0.1", 0)
    srv.start()
    base = f"http://127.0.0.1:{srv.port}"
    assert requests.put(base + "/bkt").status_code == 200
    try:
        yield srv, base, tmp_path / "blobs"
    finally:
        srv.stop()


def test_contract_against_native_endpoint(blob):
    _, base, _ = blob
    out = io.StringIO()
    res = ufs_contract.run("s3a://bkt/contract", properties={"alluxio.underfs.s3.endpoint": base}, out=out,
                           large_file_size=1 << 20)
    assert res["failed"] == [], out.getvalue()[-3000:]
    assert len(res["passed"]) >= 40


def test_native_ranged_reads_into_buffer(blob):
    srv, base, root = blob
    data = np.random.default_rng(3).integers(0, 256, (9 << 20) + 12345, dtype=np.uint8).tobytes()
    (root / "bkt" / "d").mkdir(parents=True)
    (root / "bkt" / "d" / "obj").write_bytes(data)
    ufs = create_ufs("s3://bkt/", properties={"alluxio.underfs.s3.endpoint": base,
                                              "alluxio.underfs.s3.threads.max": "4",
                                              "alluxio.underfs.s3.read.part.size": "1MB"})
    buf = np.zeros(len(data), dtype=np.uint8)
    assert ufs._get_into("d/obj", 0, len(data), buf.ctypes.data)
    assert buf.tobytes() == data
    rd = ufs._native_reader()
    assert rd.requests >= 4                       # split into parallel sub-ranges
    before = rd.connects
    # unaligned ranges, repeated: pooled connections are reused
    for off, n in [(1, 1), (777, 5 << 20), (len(data) - 10, 10), (123457, 300000)]:
        out = np.zeros(n, dtype=np.uint8)
        assert ufs._get_into("d/obj", off, n, out.ctypes.data)
        assert out.tobytes() == data[off:off + n]
    assert rd.connects - before <= 4
    # the UFS stream: large readinto goes direct, small reads through the buffered path
    with ufs.open("s3://bkt/d/obj") as f:
        assert f.read(10) == data[:10]
        big = bytearray(4 << 20)
        assert f.readinto(big) == len(big) and bytes(big) == data[10:10 + len(big)]
        assert f.read() == data[10 + len(big):]
    with pytest.raises(FileNotFoundError):
        ufs._get_into("d/missing", 0, 10, buf.ctypes.data)
    assert srv.bytes_sent >= len(data)


def test_endpoint_wire_shapes(blob):
    _, base, root = blob
    (root / "bkt" / "x").mkdir(parents=True, exist_ok=True)
    (root / "bkt" / "x" / "a.bin").write_bytes(b"0123456789")
    r = requests.get(base + "/bkt/x/a.bin", headers={"Range": "bytes=-3"})
    assert r.status_code == 206 and r.content == b"789" and r.headers["Content-Range"] == "bytes 7-9/10"
    assert requests.get(base + "/bkt/x/a.bin", headers={"Range": "bytes=20-"}).status_code == 416
    r = requests.head(base + "/bkt/x/a.bin")
    assert r.status_code == 200 and r.headers["Content-Length"] == "10" and "Last-Modified" in r.headers
    assert requests.get(base + "/bkt/nope").status_code == 404
    assert requests.get(base + "/bkt/../etc/passwd").status_code in (400, 404)
    # folder markers, delimiter listing, pagination
    assert requests.put(base + "/bkt/x/sub/").status_code == 200
    for i in range(5):
        requests.put(base + f"/bkt/x/f{i}", data=b"z" * i)
    r = requests.get(base + "/bkt", params={"list-type": "2", "prefix": "x/", "delimiter": "/", "max-keys": "3"})
    assert "<IsTruncated>true</IsTruncated>" in r.text and "<Key>x/</Key>" not in r.text
    keys, token = [], None
    while True:
        q = {"list-type": "2", "prefix": "x/", "delimiter": "/", "max-keys": "2"}
        if token:
            q["continuation-token"] = token
        t = requests.get(base + "/bkt", params=q).text
        keys += [s.split("</Key>")[0] for s in t.split("<Key>")[1:]]
        keys += [s.split("</Prefix>")[0] for s in t.split("<CommonPrefixes><Prefix>")[1:]]
        if "<IsTruncated>true" not in t:
            break
        token = t.split("<NextContinuationToken>")[1].split("<")[0]
    assert sorted(keys) == ["x/a.bin"] + [f"x/f{i}" for i in range(5)] + ["x/sub/"]
    # deleting the last object under an unmarked prefix removes the prefix
    requests.put(base + "/bkt/y/only", data=b"1")
    assert os.path.isdir(root / "bkt" / "y")
    assert requests.delete(base + "/bkt/y/only").status_code == 204
    assert not os.path.exists(root / "bkt" / "y")
    # marked folders stay until their marker goes
    requests.put(base + "/bkt/x/sub/k", data=b"1")
    requests.delete(base + "/bkt/x/sub/k")
    assert requests.head(base + "/bkt/x/sub/").status_code == 200
    requests.delete(base + "/bkt/x/sub/")
    assert requests.head(base + "/bkt/x/sub/").status_code == 404


def _open_uploads(base):
    r = requests.get(base + "/bkt", params={"uploads": ""})
    assert r.status_code == 200
    return r.text.count("<Upload>")


@pytest.mark.parametrize("streaming", ["true", "false"])
def test_bounded_multipart_writer(blob, streaming):
    """create() of an object larger than a part streams parallel UploadParts (native PUT from the
    part buffer) with at most (in-flight + 1) part buffers, whatever the object size (reference
    S3ALowLevelOutputStream / S3AOutputStream with its spool file)."""
    srv, base, root = blob
    ufs = create_ufs("s3://bkt/", properties={"alluxio.underfs.s3.endpoint": base,
                                              "alluxio.underfs.s3.streaming.upload.enabled": streaming,
                                              "alluxio.underfs.s3.streaming.upload.partition.size": "1MB",
                                              "alluxio.underfs.object.store.upload.buffer.size": "3MB",
                                              "alluxio.underfs.s3.upload.threads.max": "8"})
    ufs.multipart_threshold = 1 << 20
    data = np.random.default_rng(4).integers(0, 256, (23 << 20) + 999, dtype=np.uint8)
    w = ufs.create("s3://bkt/big/obj")
    for i in range(0, len(data), 700_000):                 # writes that straddle parts
        w.write(data[i:i + 700_000])
    w.close()
    assert w.parts_uploaded == 24 and w.buffers_allocated <= 4
    assert (root / "bkt" / "big" / "obj").read_bytes() == data.tobytes()
    assert _open_uploads(base) == 0
    small = ufs.create("s3://bkt/big/small")               # below one part: a single PUT
    small.write(b"tiny")
    small.close()
    assert small.parts_uploaded == 0 and (root / "bkt" / "big" / "small").read_bytes() == b"tiny"


def test_failed_part_aborts_upload_and_cleanup(blob, monkeypatch):
    srv, base, root = blob
    ufs = create_ufs("s3://bkt/", properties={"alluxio.underfs.s3.endpoint": base,
                                              "alluxio.underfs.s3.streaming.upload.enabled": "true",
                                              "alluxio.underfs.s3.streaming.upload.partition.size": "1MB"})
    ufs.multipart_threshold = 1 << 20
    real = type(ufs)._mp_put_part

    def flaky(self, key, upload_id, num, buf, n):
        if num == 3:
            raise OSError("injected part failure")
        return real(self, key, upload_id, num, buf, n)
    monkeypatch.setattr(type(ufs), "_mp_put_part", flaky)
    w = ufs.create("s3://bkt/f/obj")
    with pytest.raises(IOError):
        for _ in range(8):
            w.write(b"x" * (1 << 20))
        w.close()
    if not w.closed:
        w.cancel()
    assert _open_uploads(base) == 0                        # aborted, no parts left behind
    assert not (root / "bkt" / "f" / "obj").exists()
    monkeypatch.setattr(type(ufs), "_mp_put_part", real)
    # an abandoned stream (never closed) aborts instead of completing a partial object
    w2 = ufs.create("s3://bkt/f/abandoned")
    w2.write(b"y" * (3 << 20))
    assert _open_uploads(base) == 1
    del w2
    import gc
    gc.collect()
    assert _open_uploads(base) == 0 and not (root / "bkt" / "f" / "abandoned").exists()
    # cleanup(): stale uploads under the mount are aborted, fresh ones kept
    stale = ufs._mp_init("f/stale")
    assert _open_uploads(base) == 1
    assert ufs.cleanup() == 0                              # younger than the 3-day default
    ufs.properties["alluxio.underfs.s3.intermediate.upload.clean.age"] = "0ms"
    assert ufs.cleanup() == 1 and _open_uploads(base) == 0
    assert stale


def test_master_ufs_cleaner_aborts_stale_uploads(blob, tmp_path):
    from alluxio_amd.conf import Configuration
    from alluxio_amd.master.process import AlluxioMasterProcess
    _, base, _ = blob
    conf = Configuration({"alluxio.master.journal.folder": str(tmp_path / "journal"),
                          "alluxio.security.authorization.permission.enabled": "false"})
    m = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    try:
        assert requests.put(base + "/bkt/m/").status_code == 200       # the mount's folder marker
        m.fs_master.mount("/s3", "s3://bkt/m", properties={
            "alluxio.underfs.s3.endpoint": base, "alluxio.underfs.s3.intermediate.upload.clean.age": "0ms"})
        ufs = create_ufs("s3://bkt/m", properties={"alluxio.underfs.s3.endpoint": base})
        ufs._mp_init("m/half-written")
        assert _open_uploads(base) == 1
        assert m.fs_master.cleanup_ufs() == 1
        assert _open_uploads(base) == 0
    finally:
        m.stop()
