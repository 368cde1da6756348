"""LZ4-frame UFS files (underfs/lz4frame.py): the frame writer/indexer/reader against each other
and the public frame-format constants, and a mount with ``alluxio.underfs.lz4.frame.decode``
through a cluster: listings show decompressed lengths, reads return the plain bytes (host decoder
on a DRAM worker; the GPU decode at ingest is exercised by the gpu-marked test), writes of
``*.lz4`` paths persist valid frames."""
import io
import os
import struct

import numpy as np
import pytest

from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.underfs import lz4frame as lf

KB = 1 << 10


def _data(n=300 * KB, seed=0):
    rng = np.random.default_rng(seed)
    words = [b"alluxio", b"hbm", b"block", b"worker", b",", b"\n"]
    text = b"".join(words[i] for i in rng.integers(0, len(words), n))[:n // 2]
    return text + os.urandom(n - len(text))        # compressible half + stored (raw) blocks


def test_header_checksum_matches_reference_frames():
    # default lz4 CLI header: FLG 0x64 (v01, independent blocks, content checksum), BD 0x40 (64 KiB):
    # the descriptor checksum byte in every such frame is 0xA7
    assert (lf._xxh32(b"\x64\x40") >> 8) & 0xFF == 0xA7
    # frames without a content size are not indexable: served as stored bytes
    assert lf.parse_header(b"\x04\x22\x4d\x18\x64\x40\xa7" + b"\x00" * 16) is None
    assert lf.parse_header(b"not a frame at all......") is None


def test_frame_roundtrip_and_random_access():
    data = _data()
    frame = lf.encode_frame(data)
    assert struct.unpack_from("<I", frame)[0] == lf.MAGIC
    idx = lf.read_index(io.BytesIO(frame))
    assert idx.content_size == len(data) and idx.block_max == 64 * KB
    assert len(idx.blocks) == 5 and any(raw for _, _, raw in idx.blocks) and not all(raw for _, _, raw in idx.blocks)
    assert len(frame) < len(data)
    for off, n in [(0, len(data)), (1, 10), (64 * KB - 3, 9), (200 * KB, 100 * KB)]:
        r = lf.Lz4FrameReader(lambda o: io.BytesIO(frame), idx, off)
        assert r.read(n) == data[off:off + n]
    # corrupt header checksum -> not a frame; a truncated frame fails loudly
    bad = bytearray(frame)
    bad[14] ^= 0xFF
    assert lf.read_index(io.BytesIO(bytes(bad))) is None
    with pytest.raises(IOError):
        lf.read_index(io.BytesIO(frame[:len(frame) // 2]))


def test_lz4_mount_through_cluster(tmp_path):
    ufs = tmp_path / "lz"
    ufs.mkdir()
    data = _data(700 * KB, seed=3)
    (ufs / "a.lz4").write_bytes(lf.encode_frame(data))
    (ufs / "plain.lz4").write_bytes(b"not a frame")
    with LocalAlluxioCluster(num_workers=1, conf={
            "alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": "64MB",
            "alluxio.user.block.size.bytes.default": "256KB"}, work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        fs.mount("/lz", str(ufs), properties={lf.PROP_DECODE: "true"})
        st = fs.get_status("/lz/a.lz4")
        assert st.info.length == len(data) and len(st.info.blockIds) == 3
        assert fs.get_status("/lz/plain.lz4").info.length == len(b"not a frame")
        assert fs.read_file("/lz/a.lz4") == data
        assert fs.read_file("/lz/plain.lz4") == b"not a frame"
        # written through: the UFS holds a frame that decodes to the bytes
        fs.write_file("/lz/out.lz4", data[:100 * KB], write_type="CACHE_THROUGH")
        raw = (ufs / "out.lz4").read_bytes()
        assert struct.unpack_from("<I", raw)[0] == lf.MAGIC
        idx = lf.read_index(io.BytesIO(raw))
        assert lf.Lz4FrameReader(lambda o: io.BytesIO(raw), idx).read() == data[:100 * KB]
        fs.close()


@pytest.mark.gpu
def test_lz4_frame_decoded_on_gpu_at_ingest(tmp_path):
    ufs = tmp_path / "lz"
    ufs.mkdir()
    data = _data(3 << 20, seed=5)
    (ufs / "big.lz4").write_bytes(lf.encode_frame(data))
    with LocalAlluxioCluster(num_workers=1, conf={
            "alluxio.worker.tieredstore.level0.dirs.path": "hbm",
            "alluxio.worker.tieredstore.level0.dirs.quota": "256MB",
            "alluxio.user.block.size.bytes.default": "1MB"}, work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        fs.mount("/lz", str(ufs), properties={lf.PROP_DECODE: "true"})
        assert fs.get_status("/lz/big.lz4").info.length == len(data)
        w = c.workers[0].worker
        before = w.metrics.counter("Lz4DecodedBytes").count
        assert fs.read_file("/lz/big.lz4") == data
        assert w.metrics.counter("Lz4DecodedBytes").count - before == len(data)
        fs.close()
