"""Object-store UFS base: directories emulated over a flat key space.

Parity: core/common/src/main/java/alluxio/underfs/ObjectUnderFileSystem.java (1,207 lines):
directory = zero-byte marker object ``<key><suffix>`` (suffix ``/`` by default), implicit
directories inferred from key prefixes, rename = copy + delete, recursive delete by prefix
listing, multi-range reads (``alluxio.underfs.object.store.multi.range.chunk.size``).  Concrete
stores implement six primitives (put/get-range/head/delete/list/copy).
"""
from __future__ import annotations

import abc
import io
import posixpath

from .base import (CreateOptions, DeleteOptions, ListOptions, MkdirsOptions, OpenOptions,
                   UfsDirectoryStatus, UfsFileStatus, UnderFileSystem)


class ObjectMeta:
    __slots__ = ("key", "size", "etag", "mtime_ms")

    def __init__(self, key, size, etag="", mtime_ms=None):
        self.key, self.size, self.etag, self.mtime_ms = key, size, etag, mtime_ms


class _ObjectWriter(io.RawIOBase):
    """Buffers the object in memory (or a spill file) and uploads on close."""

    def __init__(self, ufs: "ObjectUnderFileSystem", key: str):
        super().__init__()
        self._ufs, self._key = ufs, key
        self._buf = io.BytesIO()

    def writable(self):
        return True

    def write(self, b):
        return self._buf.write(b)

    def close(self):
        if not self.closed:
            self._ufs._put(self._key, self._buf.getvalue())
        super().close()


class _RangeReader(io.RawIOBase):
    """Sequential reader that fetches ``chunk`` bytes per ranged GET (multi-range stream).  Stores
    with a native ``_get_into`` receive reads of at least ``_direct_min`` bytes directly into the
    caller's buffer."""

    _direct_min = 256 << 10

    def __init__(self, ufs, key, size, offset, chunk):
        super().__init__()
        self._ufs, self._key, self._size = ufs, key, size
        self._pos = offset
        self._chunk = chunk
        self._cur = b""
        self._cur_off = offset

    def readable(self):
        return True

    def seekable(self):
        return True

    def seek(self, off, whence=0):
        self._pos = {0: off, 1: self._pos + off, 2: self._size + off}[whence]
        return self._pos

    def tell(self):
        return self._pos

    def readinto(self, b):
        if self._pos >= self._size:
            return 0
        get_into = getattr(self._ufs, "_get_into", None)
        if get_into is not None and len(b) >= self._direct_min:
            # straight into the caller's buffer (the ingest pipeline's pinned staging)
            n = min(len(b), self._size - self._pos)
            import numpy as np
            arr = np.frombuffer(b, dtype=np.uint8, count=n)
            if get_into(self._key, self._pos, n, arr.ctypes.data):
                self._pos += n
                return n
        rel = self._pos - self._cur_off
        if rel < 0 or rel >= len(self._cur):
            n = min(self._chunk, self._size - self._pos)
            self._cur = self._ufs._get_range(self._key, self._pos, n)
            self._cur_off = self._pos
            rel = 0
        n = min(len(b), len(self._cur) - rel)
        b[:n] = self._cur[rel:rel + n]
        self._pos += n
        return n


class ObjectUnderFileSystem(UnderFileSystem):
    folder_suffix = "/"
    read_chunk = 8 << 20

    # ---- primitives -------------------------------------------------------------------------
    @abc.abstractmethod
    def _put(self, key: str, data: bytes) -> None: ...

    @abc.abstractmethod
    def _get_range(self, key: str, offset: int, length: int) -> bytes: ...

    @abc.abstractmethod
    def _head(self, key: str) -> ObjectMeta | None: ...

    @abc.abstractmethod
    def _delete(self, keys: list[str]) -> None: ...

    @abc.abstractmethod
    def _list(self, prefix: str, delimiter: str | None) -> tuple[list[ObjectMeta], list[str]]: ...

    def _copy(self, src: str, dst: str) -> None:
        meta = self._head(src)
        self._put(dst, self._get_range(src, 0, meta.size) if meta and meta.size else b"")

    # ---- key mapping ------------------------------------------------------------------------
    def _key(self, path: str) -> str:
        if "://" in path:
            path = path.split("://", 1)[1]
            path = path.split("/", 1)[1] if "/" in path else ""
        return path.lstrip("/")

    def is_object_storage(self) -> bool:
        return True

    def is_seekable(self) -> bool:
        return True

    def supports_flush(self) -> bool:
        return False

    # ---- UnderFileSystem --------------------------------------------------------------------
    def create(self, path, options: CreateOptions | None = None):
        return _ObjectWriter(self, self._key(path))

    def open(self, path, options: OpenOptions | None = None):
        key = self._key(path)
        meta = self._head(key)
        if meta is None:
            raise FileNotFoundError(path)
        off = options.offset if options else 0
        return io.BufferedReader(_RangeReader(self, key, meta.size, off, self.read_chunk), 1 << 20)

    def delete_file(self, path):
        key = self._key(path)
        if self._head(key) is None:
            return False
        self._delete([key])
        return True

    def delete_directory(self, path, options: DeleteOptions | None = None):
        key = self._key(path).rstrip("/")
        prefix = key + "/" if key else ""
        objs, _ = self._list(prefix, None)
        if not self.is_directory(path):
            return False
        children = [o.key for o in objs if o.key != prefix and o.key != key + self.folder_suffix]
        if children and not (options and options.recursive):
            return False
        self._delete([o.key for o in objs] + [key + self.folder_suffix])
        return True

    def get_status(self, path):
        key = self._key(path).rstrip("/")
        name = posixpath.basename(key) or "/"
        if not key:
            return UfsDirectoryStatus("/")
        meta = self._head(key)
        if meta is not None and not key.endswith(self.folder_suffix.rstrip("/") or "\0"):
            return UfsFileStatus(name, meta.size, meta.etag, meta.mtime_ms)
        if self._head(key + self.folder_suffix) is not None:
            return UfsDirectoryStatus(name)
        objs, prefixes = self._list(key + "/", "/")
        if objs or prefixes:
            return UfsDirectoryStatus(name)  # implicit directory
        return None

    def list_status(self, path, options: ListOptions | None = None):
        key = self._key(path).rstrip("/")
        prefix = key + "/" if key else ""
        if key and not self.is_directory(path):
            return None
        recursive = bool(options and options.recursive)
        objs, prefixes = self._list(prefix, None if recursive else "/")
        out: dict[str, object] = {}
        for o in objs:
            rel = o.key[len(prefix):]
            if not rel:
                continue
            if rel.endswith(self.folder_suffix) and self.folder_suffix == "/":
                d = rel.rstrip("/")
                if d:
                    out[d] = UfsDirectoryStatus(d)
                continue
            out[rel] = UfsFileStatus(rel, o.size, o.etag, o.mtime_ms)
            if recursive:  # implicit parents
                parts = rel.split("/")[:-1]
                for i in range(1, len(parts) + 1):
                    d = "/".join(parts[:i])
                    out.setdefault(d, UfsDirectoryStatus(d))
        for p in prefixes:
            d = p[len(prefix):].rstrip("/")
            if d:
                out.setdefault(d, UfsDirectoryStatus(d))
        return [out[k] for k in sorted(out)]

    def mkdirs(self, path, options: MkdirsOptions | None = None):
        key = self._key(path).rstrip("/")
        if not key or self.is_directory(path):
            return False
        if options and not options.create_parent:
            parent = posixpath.dirname(key)
            if parent and not self.is_directory(parent):
                return False
        parts = key.split("/")
        for i in range(1, len(parts) + 1):
            k = "/".join(parts[:i]) + self.folder_suffix
            if self._head(k) is None:
                self._put(k, b"")
        return True

    def rename_file(self, src, dst):
        s, d = self._key(src), self._key(dst)
        if self._head(s) is None:
            return False
        self._copy(s, d)
        self._delete([s])
        return True

    def rename_directory(self, src, dst):
        s, d = self._key(src).rstrip("/"), self._key(dst).rstrip("/")
        if not self.is_directory(src) or self.exists(dst):
            return False
        objs, _ = self._list(s + "/", None)
        for o in objs:
            self._copy(o.key, d + o.key[len(s):])
        if self._head(s + self.folder_suffix) is not None:
            self._put(d + self.folder_suffix, b"")
        self._delete([o.key for o in objs] + [s + self.folder_suffix])
        return True
