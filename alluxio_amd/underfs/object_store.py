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


_POOL_LOCK = __import__("threading").Lock()


class ObjectMeta:
    __slots__ = ("key", "size", "etag", "mtime_ms")

    def __init__(self, key, size, etag="", mtime_ms=None):
        self.key, self.size, self.etag, self.mtime_ms = key, size, etag, mtime_ms


class _ObjectWriter(io.RawIOBase):
    """Single-PUT writer of a store without multipart uploads: the object is spooled to a temp
    file under ``alluxio.tmp.dirs`` (memory holds at most one spool buffer) and PUT at close."""

    def __init__(self, ufs: "ObjectUnderFileSystem", key: str):
        super().__init__()
        import tempfile
        self._ufs, self._key = ufs, key
        self._buf = tempfile.SpooledTemporaryFile(max_size=8 << 20, dir=ufs._tmp_dir())

    def writable(self):
        return True

    def write(self, b):
        return self._buf.write(b)

    def cancel(self):
        if not self.closed:
            self._buf.close()
            super().close()

    def close(self):
        if not self.closed:
            try:
                self._buf.seek(0)
                self._ufs._put(self._key, self._buf.read())
            finally:
                self._buf.close()
        super().close()


class _MultipartWriter(io.RawIOBase):
    """Bounded-memory multipart upload of one object (reference
    underfs/s3a/src/main/java/alluxio/underfs/s3a/S3ALowLevelOutputStream.java:309-360 / :435 and
    S3AOutputStream.java:97).

    * streaming (``alluxio.underfs.s3.streaming.upload.enabled``): each full part buffer of
      ``alluxio.underfs.s3.streaming.upload.partition.size`` bytes is uploaded on the store's upload
      executor while the caller keeps writing into the next buffer;
    * spooled (the reference default): the bytes go to a temp file under ``alluxio.tmp.dirs``; at
      close the file is uploaded in parallel parts read back with pread.

    At most ``max_inflight`` part buffers exist, so memory stays bounded by (max_inflight + 1) x the
    part size whatever the object size.  An object smaller than one part is a single PUT.  Any
    failure -- a part upload, the completion, or a caller abandoning the stream (``cancel`` or
    garbage collection without ``close``) -- aborts the multipart upload, so no parts linger.
    """

    def __init__(self, ufs: "ObjectUnderFileSystem", key: str, part_size: int, max_inflight: int, spool: bool):
        import threading
        super().__init__()
        self._ufs, self._key = ufs, key
        self._part = max(64 << 10, part_size)     # real S3 wants >= 5 MiB parts (but the last)
        self._inflight = max(1, max_inflight)
        self._sem = threading.BoundedSemaphore(self._inflight)
        self._pool: list = []
        self._pool_lock = threading.Lock()
        self._buf = None
        self._fill = 0
        self._upload_id = None
        self._next = 1
        self._etags: dict[int, str] = {}
        self._futs = []
        self._error: BaseException | None = None
        self._spool = None
        self._size = 0
        if spool:
            import tempfile
            self._spool = tempfile.TemporaryFile(dir=ufs._tmp_dir())
        self.parts_uploaded = 0
        self.buffers_allocated = 0
        self.timings: dict = {}

    def writable(self):
        return True

    # ---- buffers ----------------------------------------------------------------------------
    def _take(self):
        import numpy as np
        with self._pool_lock:
            if self._pool:
                return self._pool.pop()
            self.buffers_allocated += 1
        return np.empty(self._part, dtype=np.uint8)   # numpy slices copy at memcpy speed (bytearray ~1 GB/s)

    def _give(self, buf) -> None:
        with self._pool_lock:
            self._pool.append(buf)

    # ---- writing ----------------------------------------------------------------------------
    def write(self, b):
        if self._error is not None:
            raise IOError(f"upload of {self._key} failed: {self._error}") from self._error
        import numpy as np
        mv = memoryview(b).cast("B")
        n = len(mv)
        if self._spool is not None:
            self._spool.write(mv)
            self._size += n
            return n
        src = np.frombuffer(mv, dtype=np.uint8)
        off = 0
        while off < n:
            if self._buf is None:
                self._buf = self._take()
            k = min(n - off, self._part - self._fill)
            self._buf[self._fill:self._fill + k] = src[off:off + k]
            self._fill += k
            off += k
            if self._fill == self._part:
                self._submit(self._buf, self._fill)
                self._buf, self._fill = None, 0
        self._size += n
        return n

    def _submit(self, buf, n: int) -> None:
        if self._upload_id is None:
            self._upload_id = self._ufs._mp_init(self._key)
        self._sem.acquire()                 # at most max_inflight buffers out: bounded memory
        if self._error is not None:
            self._sem.release()
            self._give(buf)
            raise IOError(f"upload of {self._key} failed: {self._error}") from self._error
        num = self._next
        self._next += 1
        self._futs.append(self._ufs._mp_executor().submit(self._upload, num, buf, n))

    def _upload(self, num: int, buf, n: int) -> None:
        try:
            self._etags[num] = self._ufs._mp_put_part(self._key, self._upload_id, num, buf, n)
            self.parts_uploaded += 1
        except BaseException as e:  # noqa: BLE001
            if self._error is None:
                self._error = e
            raise
        finally:
            self._give(buf)
            self._sem.release()

    def _drain(self) -> None:
        futs, self._futs = self._futs, []
        for f in futs:
            try:
                f.result()
            except BaseException:  # noqa: BLE001 -- recorded in self._error
                pass

    # ---- end --------------------------------------------------------------------------------
    def close(self):
        if self.closed:
            return
        try:
            if self._spool is not None:
                self._close_spooled()
            elif self._upload_id is None:
                data = self._buf[:self._fill].tobytes() if self._buf is not None else b""
                self._ufs._put_single(self._key, data)
            else:
                if self._fill:
                    self._submit(self._buf, self._fill)
                    self._buf, self._fill = None, 0
                self._complete()
        except BaseException:
            self._abort()
            raise
        finally:
            self._release()
            super().close()

    def _close_spooled(self) -> None:
        import os
        f = self._spool
        f.flush()
        if self._size <= self._part:
            f.seek(0)
            self._ufs._put_single(self._key, f.read())
            return
        fd = f.fileno()
        for off in range(0, self._size, self._part):
            n = min(self._part, self._size - off)
            buf = self._take()
            got = os.preadv(fd, [memoryview(buf)[:n]], off)
            if got != n:
                self._give(buf)
                raise IOError(f"short read of the spool file of {self._key}")
            self._submit(buf, n)
        self._complete()

    def _complete(self) -> None:
        import time
        t0 = time.perf_counter()
        self._drain()
        t1 = time.perf_counter()
        if self._error is not None:
            raise IOError(f"upload of {self._key} failed: {self._error}") from self._error
        self._ufs._mp_complete(self._key, self._upload_id, sorted(self._etags.items()))
        self.timings = {"drain_s": round(t1 - t0, 3), "complete_s": round(time.perf_counter() - t1, 3)}
        self._upload_id = None

    def _abort(self) -> None:
        self._drain()
        uid, self._upload_id = self._upload_id, None
        if uid is not None:
            try:
                self._ufs._mp_abort(self._key, uid)
            except Exception:  # noqa: BLE001 -- the UFS cleaner aborts stale uploads later
                import logging
                logging.getLogger(__name__).warning("abort of multipart upload %s of %s failed", uid, self._key)

    def _release(self) -> None:
        if self._spool is not None:
            self._spool.close()
            self._spool = None
        self._buf = None
        with self._pool_lock:
            self._pool.clear()

    def cancel(self):
        """Abandon the object: abort the multipart upload, write nothing."""
        if self.closed:
            return
        try:
            self._abort()
        finally:
            self._release()
            super().close()

    def __del__(self):
        # an abandoned stream must not complete a partial object (IOBase.__del__ would close)
        if not self.closed:
            try:
                self.cancel()
            except Exception:  # noqa: BLE001
                pass


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

    # ---- multipart primitives (stores with multipart uploads override these) ----------------
    multipart = False

    def _put_single(self, key: str, data) -> None:
        """One request for a whole (small) object."""
        self._put(key, data)

    def _mp_init(self, key: str) -> str:
        raise NotImplementedError

    def _mp_put_part(self, key: str, upload_id: str, num: int, buf, n: int) -> str:
        raise NotImplementedError

    def _mp_complete(self, key: str, upload_id: str, parts: list[tuple[int, str]]) -> None:
        raise NotImplementedError

    def _mp_abort(self, key: str, upload_id: str) -> None:
        raise NotImplementedError

    def _mp_list(self, prefix: str) -> list[tuple[str, str, int]]:
        """(key, upload id, initiated ms) of the multipart uploads still open under ``prefix``."""
        return []

    def _opt(self, name: str, default: str) -> str:
        p = self.properties or {}
        if name in p:
            return str(p[name])
        if self.conf is not None and self.conf.get_raw(name) is not None:
            return str(self.conf.get(name))
        return default

    # errors that no retry can fix: the answer itself
    _FINAL_ERRORS = (FileNotFoundError, FileExistsError, PermissionError, IsADirectoryError, NotADirectoryError)

    def _retry(self, op, what: str):
        """ObjectUnderFileSystem.retryOnException (ObjectUnderFileSystem.java:1153-1168): run ``op``
        again after an I/O error -- a store that timed out, dropped the connection or kept answering
        5xx past its client's own retries, or eventual consistency -- with the exponential back-off
        of ``alluxio.underfs.eventual.consistency.retry.{base.sleep, max.sleep, max.num}``
        (ExponentialBackoffRetry, :1194-1199).  The last error is raised when attempts run out."""
        import logging
        import time
        from ..utils.format import parse_time_size
        base = parse_time_size(self._opt("alluxio.underfs.eventual.consistency.retry.base.sleep", "50ms")) / 1000.0
        cap = parse_time_size(self._opt("alluxio.underfs.eventual.consistency.retry.max.sleep", "30sec")) / 1000.0
        tries = max(1, int(self._opt("alluxio.underfs.eventual.consistency.retry.max.num", "20")))
        for attempt in range(1, tries + 1):
            try:
                return op()
            except self._FINAL_ERRORS:
                raise
            except OSError as e:
                if attempt >= tries:
                    raise
                logging.getLogger(__name__).debug("attempt %d to %s failed: %s", attempt, what, e)
                time.sleep(min(cap, base * (2 ** (attempt - 1))))

    def _tmp_dir(self) -> str:
        import os
        d = self._opt("alluxio.tmp.dirs", "/tmp").split(",")[0].strip() or "/tmp"
        os.makedirs(d, exist_ok=True)
        return d

    def _mp_executor(self):
        import threading
        from concurrent.futures import ThreadPoolExecutor
        ex = getattr(self, "_upload_pool", None)
        if ex is None:
            with _POOL_LOCK:
                ex = getattr(self, "_upload_pool", None)
                if ex is None:
                    n = max(1, int(self._opt("alluxio.underfs.s3.upload.threads.max", "20")))
                    ex = self._upload_pool = ThreadPoolExecutor(max_workers=n, thread_name_prefix="ufs-upload")
        return ex

    # ---- UnderFileSystem --------------------------------------------------------------------
    def upload_shape(self) -> tuple[int, int]:
        """(part bytes, part buffers in flight) of a multipart upload: parts of
        ``alluxio.underfs.s3.streaming.upload.partition.size`` (at most the multipart threshold),
        as many in flight as ``alluxio.underfs.object.store.upload.buffer.size`` holds, at most
        ``alluxio.underfs.s3.upload.threads.max``."""
        from ..utils.format import parse_space_size
        part = parse_space_size(self._opt("alluxio.underfs.s3.streaming.upload.partition.size", "64MB"))
        part = min(part, getattr(self, "multipart_threshold", part))   # objects above it go multipart
        budget = parse_space_size(self._opt("alluxio.underfs.object.store.upload.buffer.size", "256MB"))
        threads = max(1, int(self._opt("alluxio.underfs.s3.upload.threads.max", "20")))
        return part, max(1, min(threads, budget // max(1, part)))

    def create(self, path, options: CreateOptions | None = None):
        if not self.multipart:
            return _ObjectWriter(self, self._key(path))
        part, inflight = self.upload_shape()
        spool = self._opt("alluxio.underfs.s3.streaming.upload.enabled", "false").lower() != "true"
        return _MultipartWriter(self, self._key(path), part, inflight, spool)

    def cleanup(self) -> int:
        """Abort multipart uploads under this mount older than
        ``alluxio.underfs.s3.intermediate.upload.clean.age`` (S3AUnderFileSystem.cleanup,
        run by the master's UfsCleaner); returns how many were aborted."""
        import time
        from ..utils.format import parse_time_size
        age_ms = parse_time_size(self._opt("alluxio.underfs.s3.intermediate.upload.clean.age", "3day"))
        cutoff = int(time.time() * 1000) - age_ms
        n = 0
        for key, uid, initiated in self._mp_list(self._key(self.root_uri).rstrip("/")):
            if initiated <= cutoff:
                try:
                    self._mp_abort(key, uid)
                    n += 1
                except Exception:  # noqa: BLE001
                    pass
        return n

    def open(self, path, options: OpenOptions | None = None):
        key = self._key(path)
        meta = self._retry(lambda: self._head(key), f"open {path}")
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
        return self._retry(lambda: self._get_status(path), f"get status of {path}")

    def _get_status(self, path):
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
