"""Local-filesystem UFS (reference underfs/local/.../LocalUnderFileSystem.java:71-107).

Paths may be given as ``/abs/path`` or ``file:///abs/path``.  ``create`` writes to a temp file
and renames on close when ``ensure_atomic`` is set (reference ``AtomicFileOutputStream``).
"""
from __future__ import annotations

import grp
import hashlib
import io
import os
import pwd
import shutil
import stat as statmod
import uuid

from .base import (CreateOptions, DeleteOptions, ListOptions, MkdirsOptions, OpenOptions, SpaceType,
                   UfsDirectoryStatus, UfsFileStatus, UnderFileSystem)


def strip_scheme(path: str) -> str:
    """``file:///x`` (or the ``sleepfs:///x`` test wrapper's URIs) -> ``/x``."""
    if path.startswith("file://"):
        path = path[len("file://"):]
    elif path.startswith("sleepfs://"):
        path = path[len("sleepfs://"):]
    return path or "/"


_IDS: dict = {}   # (uid, gid) -> (owner, group): NSS lookups once per id pair, not per file


def _unlink(p: str) -> None:
    """Remove file ``p``.  With the native module loaded, a large file's name goes now and its
    pages are freed on a background thread (``unlink_deferred``): the caller -- a master Remove --
    does not wait ~20 ms per 256 MiB for the kernel's teardown."""
    from ..ops import native
    mod = native._mod
    if mod is not None and hasattr(mod, "unlink_deferred"):
        e = mod.unlink_deferred(p)
        if e:
            raise OSError(e, os.strerror(e), p)
        return
    os.remove(p)


def _owner(st) -> tuple[str, str]:
    key = (st.st_uid, st.st_gid)
    hit = _IDS.get(key)
    if hit is not None:
        return hit
    try:
        owner = pwd.getpwuid(st.st_uid).pw_name
    except KeyError:
        owner = str(st.st_uid)
    try:
        group = grp.getgrgid(st.st_gid).gr_name
    except KeyError:
        group = str(st.st_gid)
    if len(_IDS) < 4096:
        _IDS[key] = (owner, group)
    return owner, group


class _FullWriter(io.FileIO):
    """FileIO whose write() writes everything: a single write(2) stops at 2 GiB - 4 KiB (and may
    stop early on signals), and raw FileIO reports that partial count instead of looping."""

    def write(self, b) -> int:
        mv = memoryview(b).cast("B")
        n = len(mv)
        done = 0
        while done < n:
            k = super().write(mv[done:])
            if k is None:                    # non-blocking fd with no room: not used here
                continue
            if k == 0:
                raise OSError(f"write to {self.name} made no progress at {done} of {n} bytes")
            done += k
        return n


class _AtomicWriter(_FullWriter):
    def __init__(self, final: str, mode: int):
        self._final = final
        self._tmp = f"{final}.alluxio.{uuid.uuid4().hex[:8]}.tmp"
        super().__init__(self._tmp, "w")
        self._mode = mode

    def close(self):
        if self.closed:
            return
        super().close()
        os.chmod(self._tmp, self._mode)
        os.replace(self._tmp, self._final)


class LocalUnderFileSystem(UnderFileSystem):
    scheme = "file"
    ufs_type = "local"

    def _p(self, path: str) -> str:
        return strip_scheme(path)

    def create(self, path, options: CreateOptions | None = None):
        options = options or CreateOptions()
        p = self._p(path)
        parent = os.path.dirname(p)
        if options.create_parent and parent:
            os.makedirs(parent, exist_ok=True)
        if options.ensure_atomic:
            return _AtomicWriter(p, options.mode or 0o644)
        f = _FullWriter(p, "w")
        try:
            os.chmod(p, options.mode or 0o644)
        except OSError:
            pass
        return f

    def open(self, path, options: OpenOptions | None = None):
        options = options or OpenOptions()
        f = io.FileIO(self._p(path), "r")
        if options.offset:
            f.seek(options.offset)
        return f

    def delete_file(self, path) -> bool:
        p = self._p(path)
        if not os.path.isfile(p):
            return False
        _unlink(p)
        return True

    def delete_directory(self, path, options: DeleteOptions | None = None) -> bool:
        p = self._p(path)
        if not os.path.isdir(p):
            return False
        if options and options.recursive:
            shutil.rmtree(p)
            return True
        try:
            os.rmdir(p)
            return True
        except OSError:
            return False

    def get_status(self, path):
        p = self._p(path)
        try:
            st = os.stat(p)
        except FileNotFoundError:
            return None
        name = os.path.basename(p.rstrip("/")) or "/"
        owner, group = _owner(st)
        mode = statmod.S_IMODE(st.st_mode)
        mtime = int(st.st_mtime * 1000)
        if statmod.S_ISDIR(st.st_mode):
            return UfsDirectoryStatus(name, owner, group, mode, mtime)
        h = hashlib.md5(f"{st.st_size}:{st.st_mtime_ns}".encode()).hexdigest()
        return UfsFileStatus(name, st.st_size, h, mtime, owner, group, mode)

    def list_status(self, path, options: ListOptions | None = None):
        p = self._p(path)
        if not os.path.isdir(p):
            return None
        out = []
        if options and options.recursive:
            for root, dirs, files in os.walk(p):
                rel = os.path.relpath(root, p)
                for n in sorted(dirs) + sorted(files):
                    child = os.path.join(root, n)
                    st = self.get_status(child)
                    if st is None:
                        continue
                    st.name = n if rel == "." else os.path.join(rel, n)
                    out.append(st)
            return out
        for n in sorted(os.listdir(p)):
            st = self.get_status(os.path.join(p, n))
            if st is not None:
                st.name = n
                out.append(st)
        return out

    def mkdirs(self, path, options: MkdirsOptions | None = None) -> bool:
        options = options or MkdirsOptions()
        p = self._p(path)
        if os.path.isdir(p):
            return False
        parent = os.path.dirname(p.rstrip("/"))
        if not options.create_parent and parent and not os.path.isdir(parent):
            return False
        os.makedirs(p, exist_ok=True)
        try:
            os.chmod(p, options.mode or 0o755)
        except OSError:
            pass
        return True

    def rename_file(self, src, dst) -> bool:
        s, d = self._p(src), self._p(dst)
        if not os.path.isfile(s):
            return False
        os.makedirs(os.path.dirname(d) or "/", exist_ok=True)
        os.replace(s, d)
        return True

    def rename_directory(self, src, dst) -> bool:
        s, d = self._p(src), self._p(dst)
        if not os.path.isdir(s) or os.path.exists(d):
            return False
        os.rename(s, d)
        return True

    def get_space(self, path, space_type: SpaceType) -> int:
        p = self._p(path)
        while p and not os.path.exists(p):
            p = os.path.dirname(p)
        st = os.statvfs(p or "/")
        total = st.f_blocks * st.f_frsize
        free = st.f_bavail * st.f_frsize
        return {SpaceType.SPACE_TOTAL: total, SpaceType.SPACE_FREE: free,
                SpaceType.SPACE_USED: total - free}[space_type]

    def set_mode(self, path, mode) -> None:
        os.chmod(self._p(path), mode)

    def set_owner(self, path, owner, group) -> None:
        try:
            uid = pwd.getpwnam(owner).pw_uid if owner else -1
            gid = grp.getgrnam(group).gr_gid if group else -1
            os.chown(self._p(path), uid, gid)
        except (KeyError, PermissionError):
            pass

    def get_file_locations(self, path, options=None):
        return ["localhost"]
