"""Zero-copy data framing (rpc/marshal.py) — golden bytes against protobuf, decode fast path and
fallbacks, and both stream directions through a real gRPC worker.

Reference: core/common/src/main/java/alluxio/grpc/ReadResponseMarshaller.java:30-105 (hand-built
header + raw buffer), WriteRequestMarshaller.java; alluxio.user.streaming.zerocopy.enabled.
"""
import numpy as np
import pytest

from alluxio_amd.proto import pb
from alluxio_amd.rpc import marshal

SIZES = [0, 1, 127, 128, 300, 16383, 16384, (1 << 20) - 1, 1 << 20, 2 << 20]


@pytest.mark.parametrize("n", SIZES)
def test_read_response_frame_matches_protobuf(n):
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    golden = pb.block.ReadResponse(chunk=pb.block.Chunk(data=data)).SerializeToString()
    f = marshal.read_response_frame(data)
    if n:
        assert f.SerializeToString() == golden
    # decode: zero-copy view into the received buffer
    d = marshal.decode_read_response(golden)
    assert bytes(d.chunk.data) == data
    if n:
        assert isinstance(d, marshal.DataFrame)
        assert d.chunk.data.obj is golden          # a view, not a copy


@pytest.mark.parametrize("n", SIZES)
def test_write_chunk_frame_matches_protobuf(n):
    data = bytes(range(256)) * (n // 256) + bytes(n % 256)
    golden = pb.block.WriteRequest(chunk=pb.block.Chunk(data=data)).SerializeToString()
    f = marshal.write_request_frame(data)
    if n:
        assert f.SerializeToString() == golden
    d = marshal.decode_write_request(golden)
    assert d.HasField("chunk") and bytes(d.chunk.data) == data


def test_empty_frame_roundtrips():
    # protobuf encodes an empty bytes field explicitly in proto2 when set
    f = marshal.read_response_frame(b"")
    back = pb.block.ReadResponse.FromString(f.SerializeToString())
    assert back.chunk.data == b""
    assert bytes(marshal.decode_read_response(f.SerializeToString()).chunk.data) == b""


def test_non_fast_forms_fall_back_to_protobuf():
    cmd = pb.block.WriteRequest(command=pb.block.WriteRequestCommand(type=0, id=7, offset=0, flush=True))
    d = marshal.decode_write_request(cmd.SerializeToString())
    assert isinstance(d, pb.block.WriteRequest) and d.command.id == 7
    # chunk with an unknown trailing field -> not the fast form
    raw = pb.block.ReadResponse(chunk=pb.block.Chunk(data=b"abc")).SerializeToString() + b"\x10\x01"
    d = marshal.decode_read_response(raw)
    assert isinstance(d, pb.block.ReadResponse) and d.chunk.data == b"abc"
    # truncated frame -> protobuf raises rather than returning a short view
    with pytest.raises(Exception):
        marshal.decode_read_response(marshal.read_response_frame(b"x" * 100).frame[:-1])


@pytest.mark.parametrize("zero_copy", [True, False])
def test_grpc_block_streams(tmp_path, monkeypatch, zero_copy):
    """Write a multi-block file over gRPC WriteBlock and read it back over ReadBlock, with the
    client framing on or off (the worker always frames: same bytes on the wire)."""
    from alluxio_amd.minicluster import LocalAlluxioCluster
    seen = {"read_frames": 0, "write_frames": 0}

    def dec_r(b):
        r = marshal.decode_read_response(b)
        seen["read_frames"] += isinstance(r, marshal.DataFrame)
        return r

    def dec_w(b):
        r = marshal.decode_write_request(b)
        seen["write_frames"] += isinstance(r, marshal.DataFrame)
        return r
    monkeypatch.setitem(marshal._ZERO_COPY, (marshal.BLOCK_WORKER, "ReadBlock"), (None, dec_r))
    monkeypatch.setitem(marshal._ZERO_COPY, (marshal.BLOCK_WORKER, "WriteBlock"), (dec_w, None))
    conf = {"alluxio.user.block.size.bytes.default": "3MB",
            "alluxio.user.streaming.zerocopy.enabled": str(zero_copy).lower(),
            "alluxio.user.network.inprocess.transport.enabled": "false",
            "alluxio.user.short.circuit.enabled": "false"}
    with LocalAlluxioCluster(num_workers=1, conf=conf, grpc=True, work_dir=str(tmp_path)) as cluster:
        fs = cluster.client()
        data = np.random.default_rng(1).integers(0, 256, (7 << 20) + 5, dtype=np.uint8)
        fs.write_file("/zc", data, write_type="MUST_CACHE")
        with fs.open_file("/zc") as f:
            out = f.read()
        assert np.array_equal(np.frombuffer(out, dtype=np.uint8), data)
        fs.close()
    assert seen["write_frames"] >= 8                       # worker side parses chunk frames
    assert (seen["read_frames"] >= 3) == zero_copy          # client side only when enabled


@pytest.mark.gpu
def test_grpc_read_frames_from_hbm(tmp_path, gpu):
    """ReadBlock frames built straight from HBM pages (BlockStore.read_frame: D2H into the frame)."""
    from alluxio_amd.minicluster import LocalAlluxioCluster
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "hbm:0",
            "alluxio.worker.tieredstore.level0.dirs.quota": "64MB",
            "alluxio.worker.hbm.page.size": "1MB",
            "alluxio.user.block.size.bytes.default": "4MB",
            "alluxio.user.network.inprocess.transport.enabled": "false",
            "alluxio.user.short.circuit.enabled": "false"}
    with LocalAlluxioCluster(num_workers=1, conf=conf, grpc=True, work_dir=str(tmp_path)) as cluster:
        fs = cluster.client()
        data = np.random.default_rng(2).integers(0, 256, (9 << 20) + 77, dtype=np.uint8)
        fs.write_file("/hbm", data, write_type="MUST_CACHE")
        with fs.open_file("/hbm") as f:
            out = f.read()
        assert np.array_equal(np.frombuffer(out, dtype=np.uint8), data)
        fs.close()
