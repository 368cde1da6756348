"""Byte-level journal formats.

* Log/checkpoint entries: protobuf ``writeDelimitedTo`` framing — varint length + message
  (reference UfsJournalLogWriter.java:115-142, JournalEntryStreamReader).
* Typed checkpoint streams: an 8-byte big-endian type id (``DataOutputStream.writeLong``)
  followed by the payload (checkpoint/CheckpointType.java:19-41, CheckpointOutputStream.java).
* File names: ``0x<start>-0x<end>`` hex sequence ranges, end exclusive; the open log's end is
  Long.MAX_VALUE (UfsJournalFile.java:117-145, UfsJournal.UNKNOWN_SEQUENCE_NUMBER).
"""
from __future__ import annotations

import enum
import io
import struct

from ..proto import pb

UNKNOWN_SEQUENCE_NUMBER = (1 << 63) - 1


class CheckpointType(enum.IntEnum):
    JOURNAL_ENTRY = 0
    COMPOUND = 1
    LONGS = 2
    ROCKS = 3
    INODE_PROTOS = 4
    LONG = 5


def encode_varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def read_varint(f) -> int | None:
    shift = 0
    result = 0
    while True:
        b = f.read(1)
        if not b:
            if shift == 0:
                return None
            raise EOFError("truncated varint")
        v = b[0]
        result |= (v & 0x7F) << shift
        if not v & 0x80:
            return result
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def write_delimited(f, msg) -> int:
    data = msg.SerializeToString()
    hdr = encode_varint(len(data))
    f.write(hdr)
    f.write(data)
    return len(hdr) + len(data)


def read_delimited(f, cls=None):
    """Read one delimited message; returns None at clean EOF, raises on a torn tail."""
    n = read_varint(f)
    if n is None:
        return None
    data = f.read(n)
    if len(data) != n:
        raise EOFError("truncated journal entry")
    m = (cls or pb.journal.JournalEntry)()
    m.ParseFromString(data)
    return m


def iter_delimited(f, cls=None, tolerate_torn_tail: bool = True):
    from google.protobuf.message import DecodeError
    while True:
        try:
            m = read_delimited(f, cls)
        except (EOFError, DecodeError):
            # a torn final record (crash mid-write) ends the log; recovery rewrites from there
            if tolerate_torn_tail:
                return
            raise
        if m is None:
            return
        yield m


class RawEntryBatch:
    """A batched JournalEntry (``repeated journal_entries = 39``, journal.proto:20-61) whose body
    was serialized natively (csrc/meta_codec.cpp); the writer adds the sequence number (field 1:
    protobuf fields may come in any order).  Duck-types the bits of a JournalEntry the journal
    writers use (``sequence_number``, ``SerializeToString``)."""

    __slots__ = ("body", "count", "sequence_number")

    def __init__(self, body: bytes, count: int):
        self.body = body
        self.count = count
        self.sequence_number = 0

    def SerializeToString(self) -> bytes:  # noqa: N802 - protobuf API name
        return self.body + b"\x08" + encode_varint(self.sequence_number & ((1 << 64) - 1))

    def to_proto(self):
        e = pb.journal.JournalEntry.FromString(self.body)
        e.sequence_number = self.sequence_number
        return e


def encode_file_name(start: int, end: int) -> str:
    return f"0x{start:x}-0x{end:x}"


def decode_file_name(name: str) -> tuple[int, int] | None:
    try:
        a, b = name.split("-")
        if not (a.startswith("0x") and b.startswith("0x")):
            return None
        return int(a, 16), int(b, 16)
    except ValueError:
        return None


def write_checkpoint_header(f, ctype: CheckpointType) -> None:
    f.write(struct.pack(">q", int(ctype)))


def read_checkpoint_header(f) -> CheckpointType:
    b = f.read(8)
    if len(b) != 8:
        raise EOFError("empty checkpoint")
    return CheckpointType(struct.unpack(">q", b)[0])


# ---- Kryo chunked COMPOUND checkpoints ------------------------------------------------------
# Reference: JournalUtils.writeToCheckpoint (core/server/common/.../journal/JournalUtils.java:
# 128-137) wraps a CheckpointOutputStream(COMPOUND) in Kryo's OutputChunked(64 KB): per component
# it writes the CheckpointName with Kryo's writeString, then the component's own checkpoint stream
# (an 8-byte big-endian CheckpointType followed by its data), then endChunks().  On the wire a
# chunk is a Kryo varint length (7 bits per byte, 0x80 = more) followed by that many bytes; a
# zero-length chunk ends a component.  CompoundCheckpointFormat.CompoundCheckpointReader reads it
# back with InputChunked (nextChunks skips to the byte after the zero marker).
KRYO_CHUNK = 64 * 1024
# component (master) name <-> CheckpointName (checkpoint/CheckpointName.java)
CHECKPOINT_NAMES = {"FileSystemMaster": "FILE_SYSTEM_MASTER", "BlockMaster": "BLOCK_MASTER",
                    "MetaMaster": "META_MASTER", "TableMaster": "TABLE_MASTER", "Noop": "NOOP"}
_NAMES_BACK = {v: k for k, v in CHECKPOINT_NAMES.items()}


def kryo_varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def kryo_string(s: str | None) -> bytes:
    """Kryo Output.writeString: 1 < len < 64 ASCII -> the bytes with bit 7 set on the last one;
    otherwise a UTF-8 length header (charCount + 1; 0 = null) and the characters."""
    if s is None:
        return b"\x80"
    n = len(s)
    if n == 0:
        return bytes([1 | 0x80])
    if 1 < n < 64 and all(ord(c) < 128 for c in s):
        b = bytearray(s.encode("ascii"))
        b[-1] |= 0x80
        return bytes(b)
    v = n + 1
    hdr = bytearray()
    # writeUtf8Length: 6 bits + (0x80 = UTF-8 flag, 0x40 = more), then 7-bit groups
    first = (v & 0x3F) | 0x80
    v >>= 6
    if v:
        first |= 0x40
    hdr.append(first)
    while v:
        b = v & 0x7F
        v >>= 7
        hdr.append(b | (0x80 if v else 0))
    return bytes(hdr) + s.encode("utf-8", "surrogatepass")


class _ChunkedReader:
    """Kryo InputChunked over a whole (small enough) checkpoint body."""

    def __init__(self, data: bytes, pos: int = 0):
        self.data, self.pos = data, pos

    def _varint(self) -> int:
        shift = out = 0
        while True:
            if self.pos >= len(self.data):
                raise EOFError("truncated chunk length")
            b = self.data[self.pos]
            self.pos += 1
            out |= (b & 0x7F) << shift
            if not b & 0x80:
                return out
            shift += 7

    def component(self) -> bytes | None:
        """Bytes of the next component (its chunks up to the zero marker), None at EOF."""
        if self.pos >= len(self.data):
            return None
        parts = []
        while True:
            n = self._varint()
            if n == 0:
                return b"".join(parts)
            parts.append(self.data[self.pos:self.pos + n])
            if len(parts[-1]) != n:
                raise EOFError("truncated chunk")
            self.pos += n


def kryo_read_string(buf: bytes, pos: int = 0) -> tuple[str | None, int]:
    b = buf[pos]
    if not b & 0x80:                         # ASCII: until the byte with bit 7 set
        end = pos
        while not buf[end] & 0x80:
            end += 1
        s = bytes(buf[pos:end]) + bytes([buf[end] & 0x7F])
        return s.decode("ascii"), end + 1
    v = b & 0x3F
    pos += 1
    if b & 0x40:
        shift = 6
        while True:
            c = buf[pos]
            pos += 1
            v |= (c & 0x7F) << shift
            shift += 7
            if not c & 0x80:
                break
    if v == 0:
        return None, pos
    chars = v - 1
    out = []
    while len(out) < chars:                   # Kryo's UTF-8 of UTF-16 units
        c = buf[pos]
        if c < 0x80:
            out.append(chr(c))
            pos += 1
        elif c >> 5 == 0x6:
            out.append(chr(((c & 0x1F) << 6) | (buf[pos + 1] & 0x3F)))
            pos += 2
        else:
            out.append(chr(((c & 0x0F) << 12) | ((buf[pos + 1] & 0x3F) << 6) | (buf[pos + 2] & 0x3F)))
            pos += 3
    return "".join(out), pos


def write_compound(f, parts: list[tuple[str, bytes]], sub_type: "CheckpointType | None" = None) -> None:
    """COMPOUND checkpoint (header included) in the reference's Kryo chunked layout.  ``parts``
    = (component name, component checkpoint body); the body gets its own 8-byte CheckpointType
    header (``sub_type``, default JOURNAL_ENTRY = delimited journal entries)."""
    sub_type = CheckpointType.JOURNAL_ENTRY if sub_type is None else sub_type
    write_checkpoint_header(f, CheckpointType.COMPOUND)
    for name, data in parts:
        payload = kryo_string(CHECKPOINT_NAMES.get(name, name)) + struct.pack(">q", int(sub_type)) + data
        # OutputChunked(64 KB): full buffers go out as 65536-byte chunks, endChunks() flushes the
        # rest and writes the zero-length marker
        for i in range(0, len(payload), KRYO_CHUNK):
            piece = payload[i:i + KRYO_CHUNK]
            f.write(kryo_varint(len(piece)))
            f.write(piece)
        f.write(b"\x00")


def read_compound(f) -> list:
    """Components of a COMPOUND checkpoint (header included) as ``(master name, Checkpoint)``:
    every CheckpointType the reference emits is parsed (nested COMPOUND recursively, LONGS, LONG,
    INODE_PROTOS, JOURNAL_ENTRY); ROCKS stays an opaque body (see journal/checkpoint.py)."""
    from .checkpoint import parse
    cp = parse(f.read())
    if cp.type != CheckpointType.COMPOUND:
        raise ValueError(f"not a COMPOUND checkpoint: {cp.type.name}")
    return [(_NAMES_BACK.get(p.name, p.name), p) for p in cp.parts]


def read_legacy_compound(f) -> list[tuple[str, bytes]]:
    """Round-1 snapshots of this repo: a 4-byte count, then (4-byte name length, name, 8-byte data
    length, delimited journal entries) per master -- read so old snapshots still install."""
    (n,) = struct.unpack(">i", f.read(4))
    out = []
    for _ in range(n):
        (ln,) = struct.unpack(">i", f.read(4))
        name = f.read(ln).decode()
        (dl,) = struct.unpack(">q", f.read(8))
        out.append((name, f.read(dl)))
    return out


def entries_to_bytes(entries) -> bytes:
    b = io.BytesIO()
    for e in entries:
        write_delimited(b, e)
    return b.getvalue()


def bytes_to_entries(data: bytes) -> list:
    return list(iter_delimited(io.BytesIO(data)))
