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
            "alluxio.user.short.circuit.enabled": "false",
            # the grpcio client path (the native reader / writer frame in C++: test_data_server.py)
            "alluxio.user.native.reader.enabled": "false",
            "alluxio.user.native.writer.enabled": "false",
            # the grpcio port and its Python servicer (the default domain socket is the native one)
            "alluxio.worker.data.server.domain.socket.default.enabled": "false"}
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


# Golden bytes derived by hand from the reference, not from this project's own proto code:
# ReadResponseMarshaller.serialize (core/common/.../grpc/ReadResponseMarshaller.java:45-62) writes
# tag(ReadResponse.chunk=1, LEN)=0x0A, uint32(Chunk serialized size), tag(Chunk.data=1, LEN)=0x0A,
# uint32(n), then the payload; WriteRequest.chunk is field 2 (tag 0x12) of block_worker.proto:97-101.
@pytest.mark.parametrize("n,hdr", [
    (5, "0a070a05"),
    (127, "0a81010a7f"),                 # Chunk = 1 + 1 + 127 = 129 -> varint 81 01
    (128, "0a83010a8001"),               # Chunk = 1 + 2 + 128 = 131; data length 128 -> 80 01
    (300, "0aaf020aac02"),               # 303 -> af 02; 300 -> ac 02
    (1 << 20, "0a8480400a808040"),       # 1048580 -> 84 80 40; 1048576 -> 80 80 40
])
def test_read_response_frame_golden_bytes(n, hdr):
    from alluxio_amd.rpc import marshal
    data = bytes((i * 7) & 0xFF for i in range(n))
    f = marshal.read_response_frame(data)
    raw = f.SerializeToString()
    assert raw[:len(hdr) // 2] == bytes.fromhex(hdr) and raw[len(hdr) // 2:] == data
    assert marshal.read_response_header(n) == bytes.fromhex(hdr)
    w = marshal.write_request_frame(data).SerializeToString()
    assert w[:1] == b"\x12" and w[1:len(hdr) // 2] == bytes.fromhex(hdr)[1:]


def test_sasl_plain_golden_bytes():
    """The PLAIN initial response (RFC 4616: authzid NUL authcid NUL passwd, as the reference's
    PlainSaslServer parses it) inside SaslMessage{messageType=CHALLENGE(0), message=2,
    clientId=3, authenticationScheme=SIMPLE(1) (=4), channelRef=5} (sasl_server.proto)."""
    from alluxio_amd.proto import pb
    from alluxio_amd.security.authentication import SCHEMES, parse_plain, plain_payload
    p = plain_payload("alice", "pw")
    assert p == b"\x00alice\x00pw"
    assert plain_payload("bob", "", impersonate="carol") == b"carol\x00bob\x00"
    assert parse_plain(p)[1] == "alice"
    m = pb.sasl.SaslMessage(messageType=0, message=p, clientId="c1", authenticationScheme=SCHEMES["SIMPLE"],
                            channelRef="c1")
    expect = (b"\x08\x00"                      # messageType = CHALLENGE
              + b"\x12\x09" + p                # message (9 bytes)
              + b"\x1a\x02c1"                  # clientId
              + b"\x20\x01"                    # authenticationScheme = SIMPLE
              + b"\x2a\x02c1")                 # channelRef
    assert m.SerializeToString() == expect
