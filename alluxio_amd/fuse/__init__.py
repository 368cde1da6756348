"""POSIX (FUSE) view of the namespace.

Parity: integration/fuse/src/main/java/alluxio/fuse/AlluxioFuseFileSystem.java:178-900
(chmod/chown/create/flush/getattr/mkdir/open/read/readdir/release/rename/rmdir/statfs/truncate/
unlink/utimens/write; open-file table keyed by fd; write-once files with sequential writes and
duplicate-offset suppression; truncate unsupported except to 0 on a just-created file; reads
seek + loop), AlluxioFuseUtils.java (user/group ids, error mapping) and OpenFileEntry.java.

``AlluxioFuseOps`` is the operation layer in fusepy's ``Operations`` calling convention
(``path``-based methods returning ints/dicts, raising ``FuseOSError(errno)``).  ``mount()``
attaches it to a mountpoint through this package's own ``/dev/fuse`` protocol server
(:mod:`alluxio_amd.fuse.kernel`: no libfuse or fusepy needed), or through fusepy when asked.  Reads of cached blocks are served by the page-gather kernel; a
``read_device`` extension fills a GPU tensor without a host bounce.
"""
from __future__ import annotations

import errno
import itertools
import logging
import os
import stat
import threading
import time

from ..utils.exceptions import (AlluxioStatusException, AlreadyExistsException, InvalidArgumentException,
                                NotFoundException, PermissionDeniedException)

LOG = logging.getLogger(__name__)


class FuseOSError(OSError):
    def __init__(self, code: int):
        super().__init__(code, os.strerror(code))


def _errno(e: Exception) -> int:
    if isinstance(e, NotFoundException):
        return errno.ENOENT
    if isinstance(e, AlreadyExistsException):
        return errno.EEXIST
    if isinstance(e, PermissionDeniedException):
        return errno.EACCES
    if isinstance(e, InvalidArgumentException):
        return errno.EINVAL
    if isinstance(e, AlluxioStatusException):
        name = type(e).__name__
        if "DirectoryNotEmpty" in name:
            return errno.ENOTEMPTY
        return errno.EIO
    if isinstance(e, OSError) and e.errno:
        return e.errno
    return errno.EIO


class _OpenFile:
    def __init__(self, fd, path, fin=None, fout=None):
        self.fd, self.path, self.fin, self.fout = fd, path, fin, fout
        self.write_offset = 0
        self.lock = threading.Lock()


class AlluxioFuseOps:
    def __init__(self, fs, root: str = "/", uid: int | None = None, gid: int | None = None,
                 max_cached_paths: int = 500, user_group_translation: bool = False):
        self.fs = fs
        self.root = "/" + root.strip("/") if root.strip("/") else ""
        self.uid = os.getuid() if uid is None else uid
        self.gid = os.getgid() if gid is None else gid
        self.translate = user_group_translation
        self._open: dict[int, _OpenFile] = {}
        self._fds = itertools.count(1)
        self._lock = threading.Lock()
        self.max_cached_paths = max_cached_paths

    def _p(self, path: str) -> str:
        return (self.root + ("/" + path.lstrip("/") if path.strip("/") else "")) or "/"

    def _call(self, fn, *a, **kw):
        try:
            return fn(*a, **kw)
        except FuseOSError:
            raise
        except Exception as e:  # noqa: BLE001
            LOG.debug("fuse op failed", exc_info=True)
            raise FuseOSError(_errno(e)) from None

    # ---- metadata -----------------------------------------------------------------------------
    def getattr(self, path, fh=None):
        return self.stat_info(path)[0]

    def stat_info(self, path):
        """(fusepy attribute dict, FileInfo) of ``path``: the kernel server caches the info's file
        id and blocks natively for opens served without Python."""
        st = self._call(self.fs.get_status, self._p(path))
        return self._attrs(st.info), st.info

    def list_infos(self, path):
        """[(name, attribute dict, FileInfo)] of a directory's children from ONE listing (the
        kernel server's OPENDIR fills its attribute cache from it)."""
        kids = self._call(self.fs.list_status, self._p(path))
        return [(k.name, self._attrs(k.info), k.info) for k in kids]

    def list_chunks(self, path):
        """Serialized ListStatus replies of a directory (the native FUSE server decodes and caches
        them without per-entry Python), or None when attributes need per-entry Python (user/group
        translation) or the client has no raw listing."""
        if self.translate or not hasattr(self.fs, "list_status_chunks"):
            return None
        return self._call(self.fs.list_status_chunks, self._p(path))

    def _attrs(self, i) -> dict:
        # files still being written report their open size
        size = i.length
        if not i.completed and not i.folder:
            with self._lock:
                for of in self._open.values():
                    if of.path == i.path and of.fout is not None:
                        size = of.fout.tell()
        mode = (stat.S_IFDIR if i.folder else stat.S_IFREG) | (i.mode & 0o7777)
        mtime = i.lastModificationTimeMs / 1000.0
        uid, gid = self.uid, self.gid
        if self.translate:
            import grp
            import pwd
            try:
                uid = pwd.getpwnam(i.owner).pw_uid
            except KeyError:
                pass
            try:
                gid = grp.getgrnam(i.group).gr_gid
            except KeyError:
                pass
        return {"st_mode": mode, "st_nlink": 2 if i.folder else 1, "st_size": size, "st_uid": uid, "st_gid": gid,
                "st_complete": bool(i.completed) and size == i.length,   # immutable from here on
                "st_mtime": mtime, "st_ctime": mtime, "st_atime": (i.lastAccessTimeMs or i.lastModificationTimeMs) / 1000.0,
                "st_blksize": i.blockSizeBytes or 4096, "st_blocks": (size + 511) // 512}

    def readdir(self, path, fh=None):
        kids = self._call(self.fs.list_status, self._p(path))
        return [".", ".."] + [k.name for k in kids]

    def statfs(self, path):
        cap, used = self._call(self.fs.capacity)
        bs = 4096
        return {"f_bsize": bs, "f_frsize": bs, "f_blocks": cap // bs, "f_bfree": (cap - used) // bs,
                "f_bavail": (cap - used) // bs, "f_files": 1 << 20, "f_ffree": 1 << 20, "f_namemax": 255}

    def chmod(self, path, mode):
        self._call(self.fs.set_attribute, self._p(path), mode=mode & 0o7777)
        return 0

    def chown(self, path, uid, gid):
        import grp
        import pwd
        owner = group = None
        if uid not in (-1, 0xFFFFFFFF):
            try:
                owner = pwd.getpwuid(uid).pw_name
            except KeyError:
                owner = str(uid)
        if gid not in (-1, 0xFFFFFFFF):
            try:
                group = grp.getgrgid(gid).gr_name
            except KeyError:
                group = str(gid)
        self._call(self.fs.set_attribute, self._p(path), owner=owner, group=group)
        return 0

    def utimens(self, path, times=None):
        return 0  # no settable access/modification time (reference: no-op)

    # ---- namespace ----------------------------------------------------------------------------
    def mkdir(self, path, mode):
        if len(os.path.basename(path)) > 255:
            raise FuseOSError(errno.ENAMETOOLONG)
        self._call(self.fs.create_directory, self._p(path), mode=mode & 0o7777)
        return 0

    def rmdir(self, path):
        if self._call(self.fs.list_status, self._p(path)):
            raise FuseOSError(errno.ENOTEMPTY)
        self._call(self.fs.delete, self._p(path))
        return 0

    def unlink(self, path):
        self._call(self.fs.delete, self._p(path))
        return 0

    def rename(self, old, new):
        p_new = self._p(new)
        try:
            if self.fs.exists(p_new):
                st = self.fs.get_status(p_new)
                if st.is_folder and self.fs.list_status(p_new):
                    raise FuseOSError(errno.ENOTEMPTY)
                self.fs.delete(p_new, recursive=st.is_folder)
        except AlluxioStatusException as e:
            raise FuseOSError(_errno(e)) from None
        self._call(self.fs.rename, self._p(old), p_new)
        return 0

    def truncate(self, path, length, fh=None):
        """Write-once files: only truncate(0) of a file opened for writing with nothing written
        yet (what ``O_TRUNC`` on create does) is supported."""
        with self._lock:
            for of in self._open.values():
                if of.path == self._p(path) and of.fout is not None and of.fout.tell() == 0 and length == 0:
                    return 0
        st = self._call(self.fs.get_status, self._p(path))
        if length == st.length:
            return 0
        if length == 0:
            # re-create empty (delete + create) as the reference fuse shell does for O_TRUNC
            self._call(self.fs.delete, self._p(path))
            self._call(self.fs.create_file, self._p(path)).close()
            return 0
        raise FuseOSError(errno.EOPNOTSUPP)

    # ---- file handles -------------------------------------------------------------------------
    def create(self, path, mode, fi=None):
        if len(os.path.basename(path)) > 255:
            raise FuseOSError(errno.ENAMETOOLONG)
        out = self._call(self.fs.create_file, self._p(path), mode=mode & 0o7777)
        fd = next(self._fds)
        with self._lock:
            self._open[fd] = _OpenFile(fd, self._p(path), fout=out)
        return fd

    def open(self, path, flags):
        acc = flags & (os.O_RDONLY | os.O_WRONLY | os.O_RDWR)
        p = self._p(path)
        fd = next(self._fds)
        if acc == os.O_RDONLY:
            fin = self._call(self.fs.open_file, p)
            of = _OpenFile(fd, p, fin=fin)
        else:
            # write-once: opening for write is only valid for a new/empty file (O_TRUNC/O_CREAT)
            try:
                st = self.fs.get_status(p)
                if st.length > 0 and not (flags & os.O_TRUNC):
                    raise FuseOSError(errno.EACCES)
                self.fs.delete(p)
            except NotFoundException:
                pass
            except AlluxioStatusException as e:
                raise FuseOSError(_errno(e)) from None
            of = _OpenFile(fd, p, fout=self._call(self.fs.create_file, p))
        with self._lock:
            self._open[fd] = of
        return fd

    def _entry(self, fh) -> _OpenFile:
        with self._lock:
            of = self._open.get(fh)
        if of is None:
            raise FuseOSError(errno.EBADF)
        return of

    def file_id(self, fh) -> int:
        """Alluxio file id behind a read handle (0 if unknown)."""
        with self._lock:
            of = self._open.get(fh)
        st = getattr(getattr(of, "fin", None), "status", None)
        return int(getattr(st, "fileId", 0) or 0)

    def is_write_handle(self, fh) -> bool:
        with self._lock:
            of = self._open.get(fh)
        return of is not None and of.fout is not None

    def read(self, path, size, offset, fh):
        of = self._entry(fh)
        if of.fin is None:
            raise FuseOSError(errno.EBADF)
        with of.lock:
            of.fin.seek(offset)
            return self._call(of.fin.read, size)

    def read_device(self, fh, tensor, offset: int) -> int:
        """Extension: fill a (GPU) tensor from an open file at ``offset`` (no host bounce)."""
        of = self._entry(fh)
        if of.fin is None:
            raise FuseOSError(errno.EBADF)
        with of.lock:
            of.fin.seek(offset)
            return self._call(of.fin.read_into, tensor)

    def write(self, path, data, offset, fh):
        of = self._entry(fh)
        if of.fout is None:
            raise FuseOSError(errno.EEXIST)  # existing files cannot be overwritten
        with of.lock:
            if offset < of.write_offset:
                return len(data)  # duplicate write of an already-written range (OSXFUSE quirk)
            if offset > of.write_offset:
                raise FuseOSError(errno.EOPNOTSUPP)  # random writes are not supported
            # the request body outlives this synchronous write: no copy of it (8 MiB batches)
            self._call(of.fout.write, data if isinstance(data, (bytes, bytearray, memoryview)) else bytes(data))
            of.write_offset = offset + len(data)
        return len(data)

    def flush(self, path, fh):
        """close(2) of a write handle completes the file, so a reader that opens it next sees
        every byte (close-to-open consistency; the kernel's RELEASE arrives asynchronously)."""
        with self._lock:
            of = self._open.get(fh)
        if of is not None and of.fout is not None:
            with of.lock:
                out, of.fout = of.fout, None
                if out is not None:
                    self._call(out.close)
        return 0

    def release(self, path, fh):
        with self._lock:
            of = self._open.pop(fh, None)
        if of is None:
            raise FuseOSError(errno.EBADF)
        if of.fin is not None:
            of.fin.close()
        if of.fout is not None:
            self._call(of.fout.close)
        return 0

    def fsync(self, path, datasync, fh):
        return 0

    def open_files(self) -> int:
        with self._lock:
            return len(self._open)

    def destroy(self, path=None):
        with self._lock:
            fds = list(self._open)
        for fd in fds:
            try:
                self.release(None, fd)
            except Exception:  # noqa: BLE001
                pass


def mount(ops: AlluxioFuseOps, mountpoint: str, foreground: bool = True, debug: bool = False,
          backend: str = "kernel", threads: int = 4):
    """Attach ``ops`` at ``mountpoint``.  ``backend="kernel"`` (default) serves the ``/dev/fuse``
    protocol directly (needs mount(2) permission: root or CAP_SYS_ADMIN); ``"fusepy"`` goes through
    fusepy + libfuse when installed.  In the foreground the call serves until interrupted."""
    if backend == "kernel":
        from .kernel import mount_kernel
        srv = mount_kernel(ops, mountpoint, threads=threads)
        if not foreground:
            return srv
        try:
            threading.Event().wait()
        except KeyboardInterrupt:
            pass
        finally:
            srv.unmount()
        return srv
    try:
        import fuse as fusepy  # noqa: F401
    except ImportError as e:
        raise RuntimeError("the fusepy backend needs the fusepy module and libfuse; use backend='kernel'") from e

    class _Bridge(fusepy.Operations):
        pass

    for name in ("getattr", "readdir", "statfs", "chmod", "chown", "utimens", "mkdir", "rmdir", "unlink", "rename",
                 "truncate", "create", "open", "read", "write", "flush", "release", "fsync", "destroy"):
        setattr(_Bridge, name, staticmethod(getattr(ops, name)))
    return fusepy.FUSE(_Bridge(), mountpoint, foreground=foreground, debug=debug, nothreads=False)


def main(argv=None) -> int:  # pragma: no cover - CLI entry
    import argparse
    ap = argparse.ArgumentParser(description="alluxio_amd FUSE mount")
    ap.add_argument("mountpoint")
    ap.add_argument("--root", default="/")
    ap.add_argument("--master", default=None)
    a = ap.parse_args(argv)
    from ..client.file_system import FileSystem
    fs = FileSystem(master_address=a.master)
    mount(AlluxioFuseOps(fs, a.root), a.mountpoint)
    return 0


__all__ = ["AlluxioFuseOps", "FuseOSError", "mount", "time"]
