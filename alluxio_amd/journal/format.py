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


def write_compound(f, parts: list[tuple[str, bytes]]) -> None:
    """COMPOUND checkpoint body: repeated (utf8 name, payload) with 4-byte BE lengths.

    The reference uses kryo chunked encoding here; the framing is ours, the semantics (named
    sub-checkpoints, one per master component) are the same.
    """
    f.write(struct.pack(">i", len(parts)))
    for name, data in parts:
        nb = name.encode()
        f.write(struct.pack(">i", len(nb)))
        f.write(nb)
        f.write(struct.pack(">q", len(data)))
        f.write(data)


def read_compound(f) -> list[tuple[str, bytes]]:
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
