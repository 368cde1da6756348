"""Zero-copy framing of the block data streams (ReadBlock responses, WriteBlock chunks).

Reference: core/common/src/main/java/alluxio/grpc/ReadResponseMarshaller.java:30-105 and
WriteRequestMarshaller.java (a hand-encoded protobuf header followed by the raw ByteBuf, so the
chunk bytes never pass through a protobuf message), enabled by
``alluxio.user.streaming.zerocopy.enabled`` / ``alluxio.worker.network.zerocopy.enabled``
(PropertyKey.java:3898-3900).

Here the same wire bytes are produced and consumed without protobuf objects:

* worker side, ``ReadResponse{chunk{data}}`` frames are built in ONE bytes object -- header, then
  the block bytes copied straight from the HBM/DRAM page (``BlockStore.read_frame``) -- and the
  serializer hands that object to gRPC unchanged;
* client side, a frame in the fast form decodes to a :class:`DataFrame` whose ``chunk.data`` is a
  ``memoryview`` into the received buffer (no copy); any other encoding falls back to protobuf.

WriteBlock chunks go the other way with ``WriteRequest{chunk(2){data(1)}}`` frames.  The bytes are
identical to what protobuf produces for the same message (golden tests in tests/test_marshal.py),
so Java peers and our protobuf path interoperate with either side framing.
"""
from __future__ import annotations

from ..proto import pb

READ_RESPONSE_TAG = 0x0A      # ReadResponse.chunk = 1, length-delimited
WRITE_CHUNK_TAG = 0x12        # WriteRequest.chunk = 2, length-delimited
DATA_TAG = 0x0A               # Chunk.data = 1, length-delimited


def _varint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def _read_varint(buf, pos: int) -> tuple[int, int]:
    shift = result = 0
    n = len(buf)
    while pos < n:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if b < 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            break
    return -1, pos


def frame_header(tag: int, n: int) -> bytes:
    """Protobuf prefix of ``<outer tag>{ data = <n bytes> }``."""
    inner = bytes((DATA_TAG,)) + _varint(n)
    return bytes((tag,)) + _varint(len(inner) + n) + inner


def read_response_header(n: int) -> bytes:
    return frame_header(READ_RESPONSE_TAG, n)


def write_chunk_header(n: int) -> bytes:
    return frame_header(WRITE_CHUNK_TAG, n)


class DataFrame:
    """A serialized data message standing in for ``ReadResponse`` / ``WriteRequest(chunk=...)``:
    ``.chunk.data`` is a zero-copy view of the payload, ``SerializeToString()`` the frame itself."""

    __slots__ = ("frame", "offset")

    def __init__(self, frame: bytes, offset: int):
        self.frame = frame
        self.offset = offset

    @property
    def chunk(self) -> "DataFrame":
        return self

    @property
    def data(self) -> memoryview:
        return memoryview(self.frame)[self.offset:]

    def HasField(self, name: str) -> bool:  # noqa: N802 - protobuf API
        return name == "chunk"

    def WhichOneof(self, _group: str) -> str:  # noqa: N802
        return "chunk"

    def SerializeToString(self) -> bytes:  # noqa: N802
        return self.frame

    def __len__(self) -> int:
        return len(self.frame) - self.offset


def read_response_frame(data) -> DataFrame:
    hdr = read_response_header(len(data))
    return DataFrame(b"".join((hdr, data)), len(hdr))


def write_request_frame(data) -> DataFrame:
    hdr = write_chunk_header(len(data))
    return DataFrame(b"".join((hdr, data)), len(hdr))


def _fast_offset(buf: bytes, tag: int) -> int | None:
    """Payload offset when ``buf`` is exactly ``tag{data=...}``, else None."""
    if len(buf) < 2 or buf[0] != tag:
        return None
    outer, p = _read_varint(buf, 1)
    if outer < 0 or p + outer != len(buf):
        return None
    if outer == 0:
        return p                                   # empty chunk: chunk{} (data unset)
    if buf[p] != DATA_TAG:
        return None
    n, q = _read_varint(buf, p + 1)
    if n < 0 or q + n != len(buf):
        return None
    return q


def decode_read_response(buf: bytes):
    off = _fast_offset(buf, READ_RESPONSE_TAG)
    if off is None:
        return pb.block.ReadResponse.FromString(buf)
    return DataFrame(buf, off)


def decode_write_request(buf: bytes):
    off = _fast_offset(buf, WRITE_CHUNK_TAG)
    if off is None:
        return pb.block.WriteRequest.FromString(buf)
    return DataFrame(buf, off)


def serialize(msg) -> bytes:
    return msg.SerializeToString()


def length_delimited(tag: int, payload: bytes) -> bytes:
    """``tag`` (one byte: field number << 3 | 2) + varint length + payload."""
    return b"".join((bytes((tag,)), _varint(len(payload)), payload))


class RawReply:
    """A reply that is already serialized (cached metadata replies).  gRPC and the native
    transport send ``data`` as is (``SerializeToString``); the in-process transport parses it
    (``materialize``) so callers always receive a message."""

    __slots__ = ("data", "type")

    def __init__(self, data: bytes, msg_type):
        self.data = data
        self.type = msg_type

    def SerializeToString(self) -> bytes:  # noqa: N802 - protobuf message protocol
        return self.data

    def materialize(self):
        return self.type.FromString(self.data)


def materialize(reply):
    return reply.materialize() if isinstance(reply, RawReply) else reply


BLOCK_WORKER = "alluxio.grpc.block.BlockWorker"
# (service, method) -> (request deserializer, response deserializer) replacing protobuf parsing
_ZERO_COPY = {
    (BLOCK_WORKER, "ReadBlock"): (None, decode_read_response),
    (BLOCK_WORKER, "WriteBlock"): (decode_write_request, None),
}


def marshallers(spec, zero_copy: bool = True):
    """``(request_serializer, request_deserializer, response_serializer, response_deserializer)``
    for a method spec; data streams get the frame-aware codecs when ``zero_copy``."""
    req_ser, req_des = serialize, spec.request.FromString
    resp_ser, resp_des = serialize, spec.response.FromString
    if zero_copy:
        override = _ZERO_COPY.get((spec.service, spec.name))
        if override is not None:
            req_des = override[0] or req_des
            resp_des = override[1] or resp_des
    return req_ser, req_des, resp_ser, resp_des
