"""In-memory UFS (``mem://``) — a process-local namespace used by tests and the minicluster,
the Python analogue of the reference's test-only in-memory UFS factories."""
from __future__ import annotations

import hashlib
import io
import posixpath
import threading
import time

from .base import (CreateOptions, DeleteOptions, ListOptions, MkdirsOptions, OpenOptions,
                   UfsDirectoryStatus, UfsFileStatus, UnderFileSystem)

_STORES: dict[str, dict] = {}
_STORES_LOCK = threading.Lock()


def _norm(path: str) -> str:
    if "://" in path:
        path = path.split("://", 1)[1]
        path = "/" + path.split("/", 1)[1] if "/" in path else "/"
    return posixpath.normpath("/" + path.lstrip("/"))


class _MemWriter(io.BytesIO):
    def __init__(self, ufs: "MemoryUnderFileSystem", path: str, mode: int):
        super().__init__()
        self._ufs, self._path, self._mode = ufs, path, mode

    def close(self):
        if not self.closed:
            self._ufs._put(self._path, self.getvalue(), self._mode)
        super().close()


class MemoryUnderFileSystem(UnderFileSystem):
    scheme = "mem"
    ufs_type = "mem"

    def __init__(self, root_uri: str, conf=None, properties=None):
        super().__init__(root_uri, conf, properties)
        key = root_uri.split("://", 1)[1].split("/", 1)[0] if "://" in root_uri else "default"
        with _STORES_LOCK:
            self._store = _STORES.setdefault(key, {"files": {}, "dirs": {"/": time.time()}, "lock": threading.RLock()})
        self._lock = self._store["lock"]

    @staticmethod
    def reset(name: str = "default") -> None:
        with _STORES_LOCK:
            _STORES.pop(name, None)

    def _put(self, path, data, mode):
        with self._lock:
            self._ensure_parents(path)
            self._store["files"][path] = (data, time.time(), mode)

    def _ensure_parents(self, path):
        d = posixpath.dirname(path)
        while d and d not in self._store["dirs"]:
            self._store["dirs"][d] = time.time()
            d = posixpath.dirname(d) if d != "/" else ""

    def create(self, path, options: CreateOptions | None = None):
        return _MemWriter(self, _norm(path), (options or CreateOptions()).mode)

    def open(self, path, options: OpenOptions | None = None):
        p = _norm(path)
        with self._lock:
            if p not in self._store["files"]:
                raise FileNotFoundError(p)
            data = self._store["files"][p][0]
        b = io.BytesIO(data)
        if options and options.offset:
            b.seek(options.offset)
        return b

    def delete_file(self, path):
        with self._lock:
            return self._store["files"].pop(_norm(path), None) is not None

    def delete_directory(self, path, options: DeleteOptions | None = None):
        p = _norm(path)
        with self._lock:
            if p not in self._store["dirs"]:
                return False
            prefix = p.rstrip("/") + "/"
            kids = [f for f in self._store["files"] if f.startswith(prefix)] + \
                   [d for d in self._store["dirs"] if d.startswith(prefix)]
            if kids and not (options and options.recursive):
                return False
            for k in kids:
                self._store["files"].pop(k, None)
                self._store["dirs"].pop(k, None)
            self._store["dirs"].pop(p, None)
            return True

    def get_status(self, path):
        p = _norm(path)
        with self._lock:
            if p in self._store["files"]:
                data, mt, mode = self._store["files"][p]
                return UfsFileStatus(posixpath.basename(p), len(data), hashlib.md5(data).hexdigest(),
                                     int(mt * 1000), "", "", mode)
            if p in self._store["dirs"]:
                return UfsDirectoryStatus(posixpath.basename(p) or "/", last_modified_ms=int(self._store["dirs"][p] * 1000))
        return None

    def list_status(self, path, options: ListOptions | None = None):
        p = _norm(path)
        with self._lock:
            if p not in self._store["dirs"]:
                return None
            prefix = "/" if p == "/" else p + "/"
            names = set()
            out = []
            for coll in (self._store["dirs"], self._store["files"]):
                for k in coll:
                    if k == p or not k.startswith(prefix):
                        continue
                    rel = k[len(prefix):]
                    if not (options and options.recursive) and "/" in rel:
                        continue
                    if rel in names:
                        continue
                    names.add(rel)
                    st = self.get_status(k)
                    st.name = rel
                    out.append(st)
        return sorted(out, key=lambda s: s.name)

    def mkdirs(self, path, options: MkdirsOptions | None = None):
        p = _norm(path)
        with self._lock:
            if p in self._store["dirs"]:
                return False
            parent = posixpath.dirname(p)
            if options and not options.create_parent and parent not in self._store["dirs"]:
                return False
            self._ensure_parents(p)
            self._store["dirs"][p] = time.time()
            return True

    def rename_file(self, src, dst):
        s, d = _norm(src), _norm(dst)
        with self._lock:
            if s not in self._store["files"]:
                return False
            self._ensure_parents(d)
            self._store["files"][d] = self._store["files"].pop(s)
            return True

    def rename_directory(self, src, dst):
        s, d = _norm(src), _norm(dst)
        with self._lock:
            if s not in self._store["dirs"] or d in self._store["dirs"]:
                return False
            sp = s + "/"
            for coll in ("files", "dirs"):
                for k in [k for k in self._store[coll] if k == s or k.startswith(sp)]:
                    self._store[coll][d + k[len(s):]] = self._store[coll].pop(k)
            self._ensure_parents(d)
            return True
