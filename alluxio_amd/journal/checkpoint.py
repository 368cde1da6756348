"""Typed, nested master checkpoints in the reference's byte format.

Parity (core/server/common/src/main/java/alluxio/master/journal/):
* ``checkpoint/CheckpointOutputStream.java`` / ``CheckpointInputStream.java``: every checkpoint
  stream starts with its ``CheckpointType`` id as an 8-byte big-endian long
  (``checkpoint/CheckpointType.java:19-41``: JOURNAL_ENTRY 0, COMPOUND 1, LONGS 2, ROCKS 3,
  INODE_PROTOS 4, LONG 5);
* ``JournalUtils.writeToCheckpoint`` (JournalUtils.java:128-137) / ``CompoundCheckpointFormat``:
  COMPOUND = header written straight to the output, then per component, inside Kryo's
  ``OutputChunked(64 KB)``: ``writeString(CheckpointName)``, the component's own checkpoint stream
  (header + data, possibly itself COMPOUND: the chunking nests), ``endChunks()``;
* ``LongsCheckpointFormat`` (DataOutputStream longs until EOF), ``LongCheckpointFormat`` (one long),
  ``InodeProtosCheckpointFormat`` (delimited ``alluxio.proto.meta.Inode``),
  ``JournalCheckpointFormat`` (delimited ``JournalEntry``);
* ``JournaledGroup`` / ``CheckpointName.java``: component names.

The reference's FileSystemMaster checkpoint (DefaultFileSystemMaster.java:487,
InodeTreePersistentState.java:719-741) is the nested tree::

    FILE_SYSTEM_MASTER: COMPOUND
      INODE_TREE: COMPOUND
        HEAP_INODE_STORE: INODE_PROTOS   (HeapInodeStore.java:131-142)
        PINNED_INODE_FILE_IDS / REPLICATION_LIMITED_FILE_IDS / TO_BE_PERSISTED_FILE_IDS: LONGS
                                         (CheckpointedIdHashSet.java:42)
        TTL_BUCKET_LIST: LONGS           (TtlBucketList.java:176-187)
        INODE_COUNTER: LONG              (InodeCounter.java:39-46)
      INODE_DIRECTORY_ID_GENERATOR / MOUNT_TABLE / MASTER_UFS_MANAGER / ACTIVE_SYNC_MANAGER:
        JOURNAL_ENTRY

:func:`parse` reads any of these (recursively) so a checkpoint of every type the reference emits
is accepted; ROCKS bodies are kept opaque (a RocksDB tarball needs RocksDB to restore).
"""
from __future__ import annotations

import io
import struct
from dataclasses import dataclass, field

from . import format as fmt
from .format import CheckpointType

_Q = struct.Struct(">q")


# ---- writing ---------------------------------------------------------------------------------
def typed(ctype: CheckpointType, body: bytes) -> bytes:
    return _Q.pack(int(ctype)) + body


def journal_entries(entries) -> bytes:
    return typed(CheckpointType.JOURNAL_ENTRY, fmt.entries_to_bytes(entries))


def longs(values) -> bytes:
    vals = list(values)
    return typed(CheckpointType.LONGS, struct.pack(f">{len(vals)}q", *vals))


def long_(value: int) -> bytes:
    return typed(CheckpointType.LONG, _Q.pack(int(value)))


def inode_protos(protos) -> bytes:
    b = io.BytesIO()
    b.write(_Q.pack(int(CheckpointType.INODE_PROTOS)))
    for p in protos:
        fmt.write_delimited(b, p)
    return b.getvalue()


def compound(parts) -> bytes:
    """``parts`` = [(CheckpointName, component checkpoint bytes incl. its type header)]."""
    b = io.BytesIO()
    b.write(_Q.pack(int(CheckpointType.COMPOUND)))
    for name, data in parts:
        payload = fmt.kryo_string(name) + data
        for i in range(0, len(payload), fmt.KRYO_CHUNK):
            piece = payload[i:i + fmt.KRYO_CHUNK]
            b.write(fmt.kryo_varint(len(piece)))
            b.write(piece)
        b.write(b"\x00")
    return b.getvalue()


# ---- reading ---------------------------------------------------------------------------------
@dataclass
class Checkpoint:
    """One parsed checkpoint stream: its type, raw body (after the 8-byte type) and, for
    COMPOUND, its named components in order."""
    type: CheckpointType
    body: bytes
    name: str | None = None
    parts: list = field(default_factory=list)

    def component(self, name: str) -> "Checkpoint | None":
        for p in self.parts:
            if p.name == name:
                return p
        return None

    # typed views
    def longs(self) -> list[int]:
        self._expect(CheckpointType.LONGS)
        n = len(self.body) // 8
        return list(struct.unpack(f">{n}q", self.body[:n * 8]))

    def long(self) -> int:
        self._expect(CheckpointType.LONG)
        return _Q.unpack(self.body[:8])[0]

    def entries(self) -> list:
        self._expect(CheckpointType.JOURNAL_ENTRY)
        return fmt.bytes_to_entries(self.body)

    def inodes(self) -> list:
        from ..proto import pb
        self._expect(CheckpointType.INODE_PROTOS)
        return list(fmt.iter_delimited(io.BytesIO(self.body), pb.metastore.Inode, tolerate_torn_tail=False))

    def _expect(self, t: CheckpointType) -> None:
        if self.type != t:
            raise ValueError(f"checkpoint {self.name or ''}: expected {t.name}, found {self.type.name}")


def parse(data: bytes, name: str | None = None) -> Checkpoint:
    """Parse a typed checkpoint stream (header included); COMPOUND components recursively."""
    if len(data) < 8:
        raise EOFError("empty checkpoint stream")
    (tid,) = _Q.unpack(data[:8])
    try:
        ctype = CheckpointType(tid)
    except ValueError:
        raise ValueError(f"unknown checkpoint type id {tid}") from None
    cp = Checkpoint(ctype, data[8:], name)
    if ctype == CheckpointType.COMPOUND:
        r = fmt._ChunkedReader(cp.body)
        while True:
            comp = r.component()
            if comp is None:
                break
            cname, pos = fmt.kryo_read_string(comp, 0)
            cp.parts.append(parse(comp[pos:], cname))
    return cp


def describe(cp: Checkpoint, indent: str = "") -> list[str]:
    """Human-readable outline (reference CheckpointFormat.parseToHumanReadable)."""
    head = f"{indent}{cp.name or '<root>'}: {cp.type.name}"
    if cp.type == CheckpointType.COMPOUND:
        out = [head]
        for p in cp.parts:
            out.extend(describe(p, indent + "  "))
        return out
    if cp.type == CheckpointType.LONGS:
        return [f"{head} ({len(cp.body) // 8} longs)"]
    if cp.type == CheckpointType.LONG:
        return [f"{head} = {cp.long()}"]
    if cp.type == CheckpointType.INODE_PROTOS:
        return [f"{head} ({len(cp.inodes())} inodes)"]
    if cp.type == CheckpointType.JOURNAL_ENTRY:
        return [f"{head} ({len(cp.entries())} entries)"]
    return [f"{head} ({len(cp.body)} bytes, opaque)"]


# ---- the Journaled checkpoint contract --------------------------------------------------------
def write_journaled(j) -> bytes:
    """A component's checkpoint: its own ``write_checkpoint`` when it has one (nested formats),
    else the reference's ``Journaled`` default: JOURNAL_ENTRY of its entry iterator."""
    w = getattr(j, "write_checkpoint", None)
    if w is not None:
        return w()
    return journal_entries(j.journal_entries())


def restore_journaled(j, cp: Checkpoint, apply) -> None:
    """Restore ``j`` from ``cp``: its ``restore_checkpoint`` for typed formats, else reset +
    ``apply(j, entry)`` for every entry of a JOURNAL_ENTRY checkpoint."""
    r = getattr(j, "restore_checkpoint", None)
    if r is not None and cp.type != CheckpointType.JOURNAL_ENTRY:
        r(cp)
        return
    if cp.type != CheckpointType.JOURNAL_ENTRY:
        raise ValueError(f"{getattr(j, 'journal_name', j)} cannot restore a {cp.type.name} checkpoint")
    j.reset_state()
    for e in cp.entries():
        apply(j, e)
