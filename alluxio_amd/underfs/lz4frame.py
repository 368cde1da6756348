"""Transparent LZ4-frame files in a UFS mount, decoded on the GPU when cached.

A mount with ``alluxio.underfs.lz4.frame.decode=true`` presents every ``*.lz4`` file that is a
standard LZ4 frame (the ``lz4`` CLI / liblz4 frame format) with independent blocks and a
content-size field as its *decompressed* bytes: listings report the content size, reads return
plain bytes.  Caching such a file into an HBM worker reads the compressed span of the block from
the UFS (1/ratio of the bytes over the UFS link), ships it to the GPU and decodes every frame block
in one launch of the K11 LZ4 kernel straight into HBM (worker/block_worker.py); CPU-side readers
(read-through streams, workers without a GPU) decode with the host codec.  Writes of ``*.lz4``
paths produce such frames (host encoder), so persisted files round-trip.

The reference has no counterpart (its UFS layer is byte-transparent); the frame layout follows
the public LZ4 frame format spec (magic 0x184D2204, FLG/BD descriptor, header checksum byte =
second byte of XXH32 of the descriptor, blocks with a 4-byte size whose top bit marks a stored
block, end mark 0, optional XXH32 block / content checksums).
"""
from __future__ import annotations

import io
import logging
import os
import struct
import tempfile
import threading
from dataclasses import dataclass, field

from .base import UfsFileStatus, UnderFileSystem

LOG = logging.getLogger(__name__)

MAGIC = 0x184D2204
SUFFIX = ".lz4"
BLOCK_MAX = {4: 64 << 10, 5: 256 << 10, 6: 1 << 20, 7: 4 << 20}
PROP_DECODE = "alluxio.underfs.lz4.frame.decode"


def _xxh32(data: bytes) -> int:
    import xxhash
    return xxhash.xxh32_intdigest(data, seed=0)


@dataclass
class FrameIndex:
    content_size: int
    block_max: int
    header_bytes: int
    block_checksum: bool
    content_checksum: bool
    # per frame block: (offset of its data in the file, stored bytes, stored raw)
    blocks: list = field(default_factory=list)

    def block_len(self, j: int) -> int:
        """Decompressed bytes of frame block j (all blocks but the last are full)."""
        return min(self.block_max, self.content_size - j * self.block_max)


def parse_header(head: bytes):
    """(content size, block max, header bytes, block checksum, content checksum) of a frame
    header, or None when the bytes are not a frame this layer can index (needs independent
    blocks and a content size)."""
    if len(head) < 7 or struct.unpack_from("<I", head)[0] != MAGIC:
        return None
    flg, bd = head[4], head[5]
    if flg >> 6 != 1 or not (flg & 0x20) or not (flg & 0x08):
        return None
    bmax = BLOCK_MAX.get((bd >> 4) & 7)
    if bmax is None:
        return None
    n = 6 + 8 + (4 if flg & 1 else 0)
    if len(head) < n + 1:
        return None
    if (_xxh32(head[4:n]) >> 8) & 0xFF != head[n]:
        return None
    size = struct.unpack_from("<Q", head, 6)[0]
    return size, bmax, n + 1, bool(flg & 0x10), bool(flg & 0x04)


def read_index(f) -> FrameIndex | None:
    """Index a frame from a seekable binary file: the header plus one 4-byte size read per block."""
    h = parse_header(f.read(23))
    if h is None:
        return None
    size, bmax, hbytes, bsum, csum = h
    idx = FrameIndex(size, bmax, hbytes, bsum, csum)
    pos = hbytes
    while True:
        f.seek(pos)
        b = f.read(4)
        if len(b) < 4:
            raise IOError("truncated LZ4 frame")
        word = struct.unpack("<I", b)[0]
        if word == 0:
            break
        n = word & 0x7FFFFFFF
        idx.blocks.append((pos + 4, n, bool(word >> 31)))
        pos += 4 + n + (4 if bsum else 0)
    if len(idx.blocks) != -(-size // bmax):
        raise IOError(f"LZ4 frame has {len(idx.blocks)} blocks for content size {size} (block max {bmax}); "
                      "only frames whose blocks are all full but the last are supported")
    return idx


def encode_frame(data, block_max: int = 64 << 10) -> bytes:
    """A whole frame of ``data`` (host encoder; stored blocks for incompressible input)."""
    out = io.BytesIO()
    w = Lz4FrameWriter(out, block_max, close_inner=False)
    w.write(data)
    w.close()
    return out.getvalue()


class Lz4FrameWriter(io.RawIOBase):
    """Writes an LZ4 frame (independent blocks, content size, content checksum) to ``inner``:
    blocks are encoded into a spool file as data arrives; close() writes the header (now that the
    content size is known) and the spooled blocks."""

    def __init__(self, inner, block_max: int = 64 << 10, close_inner: bool = True):
        import xxhash
        self._inner = inner
        self._close_inner = close_inner
        self._bmax = block_max
        self._buf = bytearray()
        self._spool = tempfile.TemporaryFile()
        self._size = 0
        self._hash = xxhash.xxh32(seed=0)

    def writable(self):
        return True

    def write(self, b) -> int:
        mv = memoryview(b).cast("B")
        self._buf += mv
        self._hash.update(mv)
        self._size += len(mv)
        while len(self._buf) >= self._bmax:
            self._emit(bytes(self._buf[:self._bmax]))
            del self._buf[:self._bmax]
        return len(mv)

    def _emit(self, raw: bytes) -> None:
        from ..ops.native import lib
        comp = lib().lz4_compress(raw)
        if len(comp) < len(raw):
            self._spool.write(struct.pack("<I", len(comp)) + comp)
        else:
            self._spool.write(struct.pack("<I", len(raw) | 0x80000000) + raw)

    def close(self) -> None:
        if self.closed:
            return
        if self._buf:
            self._emit(bytes(self._buf))
            self._buf.clear()
        bd = {v: k for k, v in BLOCK_MAX.items()}[self._bmax] << 4
        desc = bytes([0x40 | 0x20 | 0x08 | 0x04, bd]) + struct.pack("<Q", self._size)
        self._inner.write(struct.pack("<I", MAGIC) + desc + bytes([(_xxh32(desc) >> 8) & 0xFF]))
        self._spool.seek(0)
        while True:
            chunk = self._spool.read(8 << 20)
            if not chunk:
                break
            self._inner.write(chunk)
        self._inner.write(struct.pack("<I", 0) + struct.pack("<I", self._hash.intdigest()))
        self._spool.close()
        if self._close_inner:
            self._inner.close()
        super().close()


class Lz4FrameReader(io.RawIOBase):
    """Decompressed view of a frame from decompressed offset ``offset`` (host decoder)."""

    def __init__(self, inner_open, idx: FrameIndex, offset: int = 0):
        self._open = inner_open
        self._idx = idx
        self._pos = offset
        self._f = None
        self._cur = (-1, b"")

    def readable(self):
        return True

    def _block(self, j: int) -> bytes:
        if self._cur[0] == j:
            return self._cur[1]
        from ..ops.native import lib
        off, n, raw = self._idx.blocks[j]
        if self._f is None or not self._f.seekable():
            if self._f is not None:
                self._f.close()
            self._f = self._open(off)
            if self._f.seekable() and self._f.tell() != off:
                self._f.seek(off)
        else:
            self._f.seek(off)
        data = self._f.read(n)
        if len(data) != n:
            raise IOError("truncated LZ4 frame block")
        if not raw:
            data = lib().lz4_decompress(data, self._idx.block_max)
        if len(data) != self._idx.block_len(j):
            raise IOError(f"LZ4 frame block {j} decoded to {len(data)} bytes, expected {self._idx.block_len(j)}")
        self._cur = (j, data)
        return data

    def readinto(self, b) -> int:
        mv = memoryview(b).cast("B")
        done = 0
        while done < len(mv) and self._pos < self._idx.content_size:
            j, within = divmod(self._pos, self._idx.block_max)
            blk = self._block(j)
            n = min(len(mv) - done, len(blk) - within)
            mv[done:done + n] = blk[within:within + n]
            done += n
            self._pos += n
        return done

    def seekable(self):
        return True

    def seek(self, pos, whence=io.SEEK_SET):
        self._pos = pos if whence == io.SEEK_SET else (self._pos + pos if whence == io.SEEK_CUR
                                                        else self._idx.content_size + pos)
        return self._pos

    def tell(self):
        return self._pos

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None
        super().close()


class Lz4FrameUnderFileSystem(UnderFileSystem):
    """Decorator over a UFS: ``*.lz4`` frames appear decompressed (see module docstring)."""

    def __init__(self, inner: UnderFileSystem):
        super().__init__(inner.root_uri, inner.conf, inner.properties)
        self.inner = inner
        self.scheme = inner.scheme
        self.ufs_type = inner.ufs_type
        self._lock = threading.Lock()
        self._index: dict[str, tuple[tuple, FrameIndex | None]] = {}

    def __getattr__(self, item):
        return getattr(self.inner, item)

    # ---- frames ----------------------------------------------------------------------------
    def frame_index(self, path: str, status=None) -> FrameIndex | None:
        """The frame index of ``path`` (cached per length + mtime), None if it is no indexable
        frame."""
        if not path.endswith(SUFFIX):
            return None
        st = status if status is not None else self.inner.get_status(path)
        if not isinstance(st, UfsFileStatus):
            return None
        key = (st.content_length, st.last_modified_ms)
        with self._lock:
            hit = self._index.get(path)
        if hit is not None and hit[0] == key:
            return hit[1]
        from .base import OpenOptions
        try:
            with self.inner.open(path, OpenOptions(offset=0)) as f:
                f = f if f.seekable() else io.BytesIO(f.read())
                idx = read_index(f)
        except (IOError, OSError, ValueError) as e:
            LOG.warning("%s is not a decodable LZ4 frame (%s): served as stored bytes", path, e)
            idx = None
        with self._lock:
            self._index[path] = (key, idx)
        return idx

    def _adjust(self, path: str, st):
        if st is None or not isinstance(st, UfsFileStatus) or not path.endswith(SUFFIX):
            return st
        idx = self.frame_index(path, st)
        if idx is None:
            return st
        return _with_length(st, idx.content_size)

    # ---- UnderFileSystem ----------------------------------------------------------------------
    def create(self, path, options=None):
        out = self.inner.create(path, options)
        return Lz4FrameWriter(out) if path.endswith(SUFFIX) else out

    def open(self, path, options=None):
        idx = self.frame_index(path)
        if idx is None:
            return self.inner.open(path, options)
        from .base import OpenOptions
        off = options.offset if options is not None else 0
        return Lz4FrameReader(lambda o: self.inner.open(path, OpenOptions(offset=o)), idx, off)

    def delete_file(self, path):
        return self.inner.delete_file(path)

    def delete_directory(self, path, options=None):
        return self.inner.delete_directory(path, options)

    def get_status(self, path):
        return self._adjust(path, self.inner.get_status(path))

    def list_status(self, path, options=None):
        out = self.inner.list_status(path, options)
        if out is None:
            return None
        base = path.rstrip("/")
        return [self._adjust(base + "/" + s.name, s) if s.name.endswith(SUFFIX) else s for s in out]

    def mkdirs(self, path, options=None):
        return self.inner.mkdirs(path, options)

    def rename_file(self, src, dst):
        return self.inner.rename_file(src, dst)

    def rename_directory(self, src, dst):
        return self.inner.rename_directory(src, dst)


def _with_length(st, length: int):
    import copy
    s2 = copy.copy(st)
    s2.content_length = length
    return s2


def wrap(ufs: UnderFileSystem, properties: dict | None, conf=None) -> UnderFileSystem:
    """Apply the decorator when the mount (or the site configuration) asks for it."""
    v = (properties or {}).get(PROP_DECODE)
    if v is None and conf is not None:
        v = conf.get_bool(PROP_DECODE, "false")
    if str(v).lower() == "true":
        return Lz4FrameUnderFileSystem(ufs)
    return ufs
