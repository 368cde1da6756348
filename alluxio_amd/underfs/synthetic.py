"""Synthetic, read-only UFS for dataset-scale benchmarks (``synth://``).

BASELINE config 4 is 1 M x 128 KB image files (docs/en/compute/Deep-Learning.md:94-96): 131 GB
that no test disk here holds.  This UFS serves such a namespace deterministically without storing
it: every directory ``/<name>`` at the mount root lists ``files`` entries ``%07d.JPEG`` of ``size``
bytes, and the bytes of file ``i`` are those of backing file ``i % backing`` -- ``backing`` real
files of ``size`` bytes each, generated once (splitmix64 of the file index and offset) in
``backing.dir``.  Content is therefore a pure function of the path, every listing/status is
computed, and the worker's native bulk ingest reads the backing file with ``pread`` exactly as it
reads a local UFS (``native_path``).

Mount properties (or configuration keys):
  alluxio.underfs.synthetic.files        files per directory          (default 1000)
  alluxio.underfs.synthetic.size         bytes per file               (default 131072)
  alluxio.underfs.synthetic.backing      distinct backing files       (default 4096)
  alluxio.underfs.synthetic.backing.dir  where they live              (default <tmp>/alluxio_synth)
  alluxio.underfs.synthetic.dirs         comma list of directory names (default "data")
"""
from __future__ import annotations

import io
import os
import tempfile
import threading

import numpy as np

from .base import UfsDirectoryStatus, UfsFileStatus, UnderFileSystem
from .registry import UnderFileSystemFactory, register_factory

_GEN_LOCK = threading.Lock()
_MTIME = 1_600_000_000_000


def backing_bytes(index: int, size: int) -> bytes:
    """Deterministic content of backing file ``index`` (splitmix64 words of (index, word))."""
    n = (size + 7) // 8
    with np.errstate(over="ignore"):
        x = np.arange(n, dtype=np.uint64) + np.uint64(index) * np.uint64(0x9E3779B97F4A7C15)
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return x.tobytes()[:size]


class SyntheticUnderFileSystem(UnderFileSystem):
    scheme = "synth"
    ufs_type = "synthetic"

    def __init__(self, root_uri: str, conf=None, properties=None):
        super().__init__(root_uri, conf, properties)
        p = dict(properties or {})

        def get(k, d):
            if k in p:
                return p[k]
            if conf is not None and conf.get_raw(k) is not None:
                return conf.get_raw(k)
            return d
        self.files = int(get("alluxio.underfs.synthetic.files", "1000"))
        self.size = int(get("alluxio.underfs.synthetic.size", str(128 << 10)))
        self.backing = max(1, int(get("alluxio.underfs.synthetic.backing", "4096")))
        self.dirs = [d for d in str(get("alluxio.underfs.synthetic.dirs", "data")).split(",") if d]
        self.backing_dir = str(get("alluxio.underfs.synthetic.backing.dir",
                                   os.path.join(tempfile.gettempdir(), "alluxio_synth")))
        self._ready = False

    # ---- layout ----------------------------------------------------------------------------
    def _rel(self, path: str) -> list[str]:
        if "://" in path:
            path = path.split("://", 1)[1]
            path = path[path.find("/"):] if "/" in path else "/"
        root = self.root_uri.split("://", 1)[1] if "://" in self.root_uri else self.root_uri
        root = root[root.find("/"):] if "/" in root else ""
        rel = path[len(root):] if root and path.startswith(root) else path
        comps = [c for c in rel.split("/") if c]
        if not comps or comps[0] not in self.dirs:
            # an instance created for a file URI (a worker opening one file) has that file as its
            # root: recognise the layout from the tail instead (<dir>/<name> or <dir>)
            every = [c for c in path.split("/") if c]
            if len(every) >= 2 and every[-2] in self.dirs:
                return every[-2:]
            if every and every[-1] in self.dirs:
                return every[-1:]
        return comps

    def _index(self, name: str) -> int | None:
        if not name.endswith(".JPEG") or len(name) != 12 or not name[:7].isdigit():
            return None
        i = int(name[:7])
        return i if i < self.files else None

    def _file_status(self, name: str, i: int) -> UfsFileStatus:
        return UfsFileStatus(name, content_length=self.size, content_hash=f"synth-{i % self.backing}-{self.size}",
                             last_modified_ms=_MTIME, owner="synthetic", group="synthetic", mode=0o444)

    def _ensure_backing(self) -> None:
        if self._ready:
            return
        with _GEN_LOCK:
            os.makedirs(self.backing_dir, exist_ok=True)
            for j in range(self.backing):
                f = os.path.join(self.backing_dir, f"{self.size}-{j:06d}")
                if not os.path.exists(f) or os.path.getsize(f) != self.size:
                    tmp = f + ".tmp"
                    with open(tmp, "wb") as out:
                        out.write(backing_bytes(j, self.size))
                    os.replace(tmp, f)
            self._ready = True

    def backing_path(self, i: int) -> str:
        return os.path.join(self.backing_dir, f"{self.size}-{i % self.backing:06d}")

    def native_path(self, path: str) -> str | None:
        """Local file the worker's native ingest preads for ``path``."""
        comps = self._rel(path)
        if len(comps) != 2 or comps[0] not in self.dirs:
            return None
        i = self._index(comps[1])
        if i is None:
            return None
        self._ensure_backing()
        return self.backing_path(i)

    # ---- read API ----------------------------------------------------------------------------
    def get_status(self, path: str):
        comps = self._rel(path)
        if not comps:
            return UfsDirectoryStatus("", owner="synthetic", group="synthetic", mode=0o555, last_modified_ms=_MTIME)
        if comps[0] not in self.dirs or len(comps) > 2:
            return None
        if len(comps) == 1:
            return UfsDirectoryStatus(comps[0], owner="synthetic", group="synthetic", mode=0o555,
                                      last_modified_ms=_MTIME)
        i = self._index(comps[1])
        return None if i is None else self._file_status(comps[1], i)

    def list_status(self, path: str, options=None):
        comps = self._rel(path)
        if not comps:
            return [UfsDirectoryStatus(d, owner="synthetic", group="synthetic", mode=0o555, last_modified_ms=_MTIME)
                    for d in self.dirs]
        if len(comps) != 1 or comps[0] not in self.dirs:
            return None
        return [self._file_status(f"{i:07d}.JPEG", i) for i in range(self.files)]

    def open(self, path: str, options=None):
        p = self.native_path(path)
        if p is None:
            raise FileNotFoundError(path)
        f = open(p, "rb")
        off = getattr(options, "offset", 0) if options is not None else 0
        if off:
            f.seek(off)
        return f

    # ---- read-only -----------------------------------------------------------------------------
    def create(self, path, options=None):
        raise PermissionError("synthetic UFS is read-only")

    def delete_file(self, path):
        raise PermissionError("synthetic UFS is read-only")

    def delete_directory(self, path, options=None):
        raise PermissionError("synthetic UFS is read-only")

    def mkdirs(self, path, options=None):
        raise PermissionError("synthetic UFS is read-only")

    def rename_file(self, src, dst):
        raise PermissionError("synthetic UFS is read-only")

    def rename_directory(self, src, dst):
        raise PermissionError("synthetic UFS is read-only")


class _Factory(UnderFileSystemFactory):
    scheme = "synth"

    def create(self, uri, conf=None, properties=None):
        return SyntheticUnderFileSystem(uri, conf, properties)


register_factory(_Factory())
del io
