"""FUSE kernel-protocol server: mount :class:`AlluxioFuseOps` without libfuse or fusepy.

Parity: integration/fuse/src/main/java/alluxio/fuse/AlluxioFuse.java (mount the namespace at a
local mountpoint, foreground serving, unmount on exit) + AlluxioFuseFileSystem.java (the
operations, here :class:`alluxio_amd.fuse.AlluxioFuseOps`).  The reference goes through jnr-fuse
and libfuse; this server speaks the kernel's ``/dev/fuse`` protocol (``linux/fuse.h``, protocol
7.x) directly: it opens ``/dev/fuse``, calls ``mount(2)`` with ``fd=<n>``, and answers requests
from a pool of threads, each reading one request at a time (the multi-threaded libfuse loop).

The kernel speaks in node ids; the op layer is path based (as the reference's), so the server keeps
a node-id <-> path table (LOOKUP/CREATE/MKDIR allocate, FORGET drops, RENAME rewrites the moved
subtree).  Directory listings are snapshotted at OPENDIR and paged out by offset.
"""
from __future__ import annotations

import ctypes
import errno
import logging
import os
import stat
import struct
import threading

from . import AlluxioFuseOps, FuseOSError

LOG = logging.getLogger(__name__)

# opcodes (linux/fuse.h enum fuse_opcode)
LOOKUP, FORGET, GETATTR, SETATTR = 1, 2, 3, 4
MKDIR, UNLINK, RMDIR, RENAME = 9, 10, 11, 12
OPEN, READ, WRITE, STATFS, RELEASE, FSYNC = 14, 15, 16, 17, 18, 20
GETXATTR, LISTXATTR, FLUSH, INIT, OPENDIR, READDIR, RELEASEDIR, FSYNCDIR = 22, 23, 25, 26, 27, 28, 29, 30
ACCESS, CREATE, INTERRUPT, DESTROY, BATCH_FORGET, RENAME2 = 34, 35, 36, 38, 42, 45

IOCTL = 39
OP_NAMES = {LOOKUP: "LOOKUP", FORGET: "FORGET", GETATTR: "GETATTR", SETATTR: "SETATTR", MKDIR: "MKDIR",
            UNLINK: "UNLINK", RMDIR: "RMDIR", RENAME: "RENAME", OPEN: "OPEN", READ: "READ", WRITE: "WRITE",
            STATFS: "STATFS", RELEASE: "RELEASE", FSYNC: "FSYNC", GETXATTR: "GETXATTR", LISTXATTR: "LISTXATTR",
            FLUSH: "FLUSH", INIT: "INIT", OPENDIR: "OPENDIR", READDIR: "READDIR", RELEASEDIR: "RELEASEDIR",
            FSYNCDIR: "FSYNCDIR", ACCESS: "ACCESS", CREATE: "CREATE", INTERRUPT: "INTERRUPT", IOCTL: "IOCTL",
            DESTROY: "DESTROY", BATCH_FORGET: "BATCH_FORGET", RENAME2: "RENAME2"}

IN_HDR = struct.Struct("<IIQQIIII")            # len opcode unique nodeid uid gid pid padding
OUT_HDR = struct.Struct("<IiQ")                # len error unique
ATTR = struct.Struct("<QQQQQQIIIIIIIIII")      # fuse_attr (88 bytes)
ENTRY_HEAD = struct.Struct("<QQQQII")          # nodeid generation entry_valid attr_valid + nsecs
ATTR_OUT_HEAD = struct.Struct("<QII")
INIT_OUT = struct.Struct("<IIIIHHIIHH32x")     # major minor max_readahead flags max_bg cong max_write gran pages align
OPEN_OUT = struct.Struct("<QII")
READ_IN = struct.Struct("<QQIIQII")
WRITE_IN = struct.Struct("<QQIIQII")
SETATTR_IN = struct.Struct("<IIQQQQQQIIIIIIII")
KSTATFS = struct.Struct("<QQQQQIIII24x")
DIRENT = struct.Struct("<QQII")

FATTR_MODE, FATTR_UID, FATTR_GID, FATTR_SIZE = 1 << 0, 1 << 1, 1 << 2, 1 << 3
FATTR_ATIME, FATTR_MTIME = 1 << 4, 1 << 5
FUSE_ASYNC_READ, FUSE_ATOMIC_O_TRUNC, FUSE_BIG_WRITES = 1 << 0, 1 << 3, 1 << 5
FOPEN_KEEP_CACHE = 1 << 1
MS_NOSUID, MS_NODEV = 2, 4
MNT_DETACH = 2
MAX_WRITE = 128 << 10
ROOT_ID = 1
TTL_S = 1              # directories / entries (the namespace can change under them)
TTL_COMPLETE_S = 60    # attributes of completed (write-once, immutable) files


def _ts(t: float) -> tuple[int, int]:
    s = int(t)
    return s, int((t - s) * 1e9)


class FuseKernelServer:
    """Serve ``ops`` at ``mountpoint`` until :meth:`unmount`."""

    def __init__(self, ops: AlluxioFuseOps, mountpoint: str, threads: int = 4, allow_other: bool = False,
                 keep_cache: bool = False):
        self.ops = ops
        self.keep_cache = keep_cache
        self.mountpoint = os.path.abspath(mountpoint)
        self.nthreads = max(1, threads)
        self.allow_other = allow_other
        self.fd = -1
        self._threads: list[threading.Thread] = []
        self._lock = threading.Lock()
        self._paths = {ROOT_ID: "/"}                 # node id -> path
        self._ids = {"/": ROOT_ID}                   # path -> node id
        self._next_id = ROOT_ID + 1
        self._dirs: dict[int, list] = {}             # opendir handle -> [(name, mode)]
        self._next_dir = 1
        self._stop = threading.Event()
        self.requests = 0
        self.op_counts: dict[int, int] = {}           # opcode -> requests served (diagnostics)

    # ---- mount / unmount ---------------------------------------------------------------------
    def mount(self) -> "FuseKernelServer":
        libc = ctypes.CDLL(None, use_errno=True)
        self.fd = os.open("/dev/fuse", os.O_RDWR | os.O_CLOEXEC)
        opts = f"fd={self.fd},rootmode=40000,user_id={os.getuid()},group_id={os.getgid()}"
        if self.allow_other:
            opts += ",allow_other"
        rc = libc.mount(b"alluxio", self.mountpoint.encode(), b"fuse.alluxio",
                        ctypes.c_ulong(MS_NOSUID | MS_NODEV), opts.encode())
        if rc != 0:
            err = ctypes.get_errno()
            os.close(self.fd)
            self.fd = -1
            raise OSError(err, f"mount {self.mountpoint}: {os.strerror(err)}")
        for i in range(self.nthreads):
            t = threading.Thread(target=self._loop, name=f"fuse-{i}", daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def unmount(self) -> None:
        if self.fd < 0:
            return
        self._stop.set()
        libc = ctypes.CDLL(None, use_errno=True)
        libc.umount2(self.mountpoint.encode(), MNT_DETACH)
        try:
            os.close(self.fd)        # aborts the connection: readers return ENODEV / EBADF
        except OSError:
            pass
        self.fd = -1
        for t in self._threads:
            t.join(timeout=5)
        self._threads = []
        self.ops.destroy()

    def __enter__(self):
        return self.mount()

    def __exit__(self, *exc):
        self.unmount()

    # ---- node table --------------------------------------------------------------------------
    def _path(self, nodeid: int) -> str:
        with self._lock:
            p = self._paths.get(nodeid)
        if p is None:
            raise FuseOSError(errno.ESTALE)
        return p

    def _node(self, path: str) -> int:
        with self._lock:
            nid = self._ids.get(path)
            if nid is None:
                nid = self._next_id
                self._next_id += 1
                self._ids[path] = nid
                self._paths[nid] = path
            return nid

    def _forget_path(self, path: str) -> None:
        with self._lock:
            nid = self._ids.pop(path, None)
            if nid is not None and nid != ROOT_ID:
                self._paths.pop(nid, None)

    def _moved(self, old: str, new: str) -> None:
        with self._lock:
            pre = old.rstrip("/") + "/"
            for p in [p for p in self._ids if p == old or p.startswith(pre)]:
                nid = self._ids.pop(p)
                np_ = new + p[len(old):]
                self._ids[np_] = nid
                self._paths[nid] = np_

    @staticmethod
    def _child(parent: str, name: str) -> str:
        return parent.rstrip("/") + "/" + name

    # ---- encoding ----------------------------------------------------------------------------
    def _attr(self, nodeid: int, a: dict) -> bytes:
        at, an = _ts(a.get("st_atime", 0.0))
        mt, mn = _ts(a.get("st_mtime", 0.0))
        ct, cn = _ts(a.get("st_ctime", 0.0))
        return ATTR.pack(nodeid, a.get("st_size", 0), a.get("st_blocks", 0), at, mt, ct, an, mn, cn,
                         a["st_mode"], a.get("st_nlink", 1), a.get("st_uid", 0), a.get("st_gid", 0), 0,
                         a.get("st_blksize", 4096), 0)

    @staticmethod
    def _attr_ttl(a: dict) -> int:
        # a file's size changes while it is written (and at completion): cache attrs only once the
        # file is complete -- Alluxio files are write-once, so a completed file's size is final
        if a.get("st_complete"):
            return TTL_COMPLETE_S
        return TTL_S if stat.S_ISDIR(a["st_mode"]) else 0

    def _entry(self, path: str) -> bytes:
        a = self.ops.getattr(path)
        nid = self._node(path)
        ttl = self._attr_ttl(a)
        return ENTRY_HEAD.pack(nid, 0, max(TTL_S, ttl), ttl, 0, 0) + self._attr(nid, a)

    # ---- request loop ------------------------------------------------------------------------
    def _loop(self) -> None:
        bufsize = MAX_WRITE + 4096
        while not self._stop.is_set():
            try:
                req = os.read(self.fd, bufsize)
            except OSError as e:
                if e.errno in (errno.EINTR, errno.ENOENT, errno.EAGAIN):
                    continue                  # interrupted / already-answered request
                return                        # ENODEV / EBADF: unmounted
            if not req:
                return
            try:
                self._dispatch(req)
            except Exception:  # noqa: BLE001 - never kill a serving thread
                LOG.exception("fuse request failed")

    def _reply(self, unique: int, err: int = 0, payload: bytes = b"") -> None:
        try:
            os.write(self.fd, OUT_HDR.pack(OUT_HDR.size + len(payload), -err, unique) + payload)
        except OSError as e:
            if e.errno not in (errno.ENOENT, errno.EBADF, errno.ENODEV):   # ENOENT: request interrupted
                raise

    def _dispatch(self, req: bytes) -> None:
        _, op, unique, nodeid, uid, gid, pid, _ = IN_HDR.unpack_from(req)
        body = memoryview(req)[IN_HDR.size:]
        self.requests += 1
        self.op_counts[op] = self.op_counts.get(op, 0) + 1
        if op in (FORGET, BATCH_FORGET, INTERRUPT):
            return                             # no reply; node ids stay valid for renamed paths
        try:
            payload = self._handle(op, nodeid, body)
        except FuseOSError as e:
            self._reply(unique, e.errno or errno.EIO)
            return
        except OSError as e:
            self._reply(unique, e.errno or errno.EIO)
            return
        except Exception:  # noqa: BLE001
            LOG.debug("fuse op %d failed", op, exc_info=True)
            self._reply(unique, errno.EIO)
            return
        if op == DESTROY:
            self._reply(unique)
            return
        self._reply(unique, 0, payload)

    @staticmethod
    def _name(body, off: int = 0) -> tuple[str, int]:
        raw = bytes(body[off:])
        end = raw.index(b"\0")
        return raw[:end].decode(), off + end + 1

    def _handle(self, op: int, nodeid: int, body) -> bytes:
        ops = self.ops
        if op == INIT:
            major, minor, max_ra, flags = struct.unpack_from("<IIII", body)
            if major != 7:
                raise FuseOSError(errno.EPROTO)
            want = FUSE_ASYNC_READ | FUSE_ATOMIC_O_TRUNC | FUSE_BIG_WRITES
            return INIT_OUT.pack(7, min(minor, 34), max_ra, flags & want, 16, 12, MAX_WRITE, 1, 0, 0)
        if op == DESTROY:
            return b""
        if op == LOOKUP:
            name, _ = self._name(body)
            return self._entry(self._child(self._path(nodeid), name))
        if op == GETATTR:
            a = ops.getattr(self._path(nodeid))
            return ATTR_OUT_HEAD.pack(self._attr_ttl(a), 0, 0) + self._attr(nodeid, a)
        if op == SETATTR:
            f = SETATTR_IN.unpack_from(body)
            valid, fh, size, mode, uid, gid = f[0], f[2], f[3], f[11], f[13], f[14]
            path = self._path(nodeid)
            if valid & FATTR_MODE:
                ops.chmod(path, mode)
            if valid & (FATTR_UID | FATTR_GID):
                ops.chown(path, uid if valid & FATTR_UID else -1, gid if valid & FATTR_GID else -1)
            if valid & FATTR_SIZE:
                ops.truncate(path, size, fh or None)
            a = ops.getattr(path)
            return ATTR_OUT_HEAD.pack(self._attr_ttl(a), 0, 0) + self._attr(nodeid, a)
        if op == ACCESS:
            ops.getattr(self._path(nodeid))
            return b""
        if op == STATFS:
            s = ops.statfs(self._path(nodeid))
            return KSTATFS.pack(s["f_blocks"], s["f_bfree"], s["f_bavail"], s["f_files"], s["f_ffree"],
                                s["f_bsize"], s["f_namemax"], s["f_frsize"], 0)
        if op == MKDIR:
            mode, _umask = struct.unpack_from("<II", body)
            name, _ = self._name(body, 8)
            path = self._child(self._path(nodeid), name)
            ops.mkdir(path, mode)
            return self._entry(path)
        if op in (UNLINK, RMDIR):
            name, _ = self._name(body)
            path = self._child(self._path(nodeid), name)
            (ops.unlink if op == UNLINK else ops.rmdir)(path)
            self._forget_path(path)
            return b""
        if op in (RENAME, RENAME2):
            newdir = struct.unpack_from("<Q", body)[0]
            off = 8 if op == RENAME else 16
            if op == RENAME2 and struct.unpack_from("<I", body, 8)[0]:
                raise FuseOSError(errno.EINVAL)          # RENAME_NOREPLACE / EXCHANGE unsupported
            old, off = self._name(body, off)
            new, _ = self._name(body, off)
            src = self._child(self._path(nodeid), old)
            dst = self._child(self._path(newdir), new)
            ops.rename(src, dst)
            self._moved(src, dst)
            return b""
        if op == CREATE:
            flags, mode, _umask, _oflags = struct.unpack_from("<IIII", body)
            name, _ = self._name(body, 16)
            path = self._child(self._path(nodeid), name)
            fh = ops.create(path, mode)
            return self._entry(path) + OPEN_OUT.pack(fh, 0, 0)
        if op == OPEN:
            flags = struct.unpack_from("<I", body)[0]
            path = self._path(nodeid)
            fh = ops.open(path, flags)
            keep = 0
            if flags & (os.O_WRONLY | os.O_RDWR) == 0 and self.keep_cache:
                # completed files never change: keep the kernel page cache across opens
                # (a second epoch over a dataset is served from it)
                keep = FOPEN_KEEP_CACHE
            return OPEN_OUT.pack(fh, keep, 0)
        if op == READ:
            fh, offset, size = READ_IN.unpack_from(body)[:3]
            return bytes(ops.read(self._path(nodeid), size, offset, fh))
        if op == WRITE:
            fh, offset, size = WRITE_IN.unpack_from(body)[:3]
            data = body[WRITE_IN.size:WRITE_IN.size + size]
            n = ops.write(self._path(nodeid), data, offset, fh)
            return struct.pack("<II", n, 0)
        if op == FLUSH:
            fh = struct.unpack_from("<Q", body)[0]
            ops.flush(None, fh)
            return b""
        if op in (FSYNC, FSYNCDIR):
            return b""
        if op == RELEASE:
            fh = struct.unpack_from("<Q", body)[0]
            try:
                ops.release(None, fh)
            except FuseOSError:
                pass                          # already finished at FLUSH
            return b""
        if op == OPENDIR:
            path = self._path(nodeid)
            names = ops.readdir(path)
            entries = []
            for n in names:
                if n in (".", ".."):
                    entries.append((n, stat.S_IFDIR))
                    continue
                try:
                    m = ops.getattr(self._child(path, n))["st_mode"]
                except FuseOSError:
                    continue
                entries.append((n, m))
            with self._lock:
                h = self._next_dir
                self._next_dir += 1
                self._dirs[h] = entries
            return OPEN_OUT.pack(h, 0, 0)
        if op == READDIR:
            fh, offset, size = READ_IN.unpack_from(body)[:3]
            with self._lock:
                entries = self._dirs.get(fh)
            if entries is None:
                raise FuseOSError(errno.EBADF)
            out = bytearray()
            for i in range(offset, len(entries)):
                name, mode = entries[i]
                nb = name.encode()
                rec = DIRENT.size + len(nb)
                rec_pad = (rec + 7) & ~7
                if len(out) + rec_pad > size:
                    break
                out += DIRENT.pack(0xFFFFFFFF, i + 1, len(nb), (mode & 0o170000) >> 12) + nb + b"\0" * (rec_pad - rec)
            return bytes(out)
        if op == RELEASEDIR:
            fh = struct.unpack_from("<Q", body)[0]
            with self._lock:
                self._dirs.pop(fh, None)
            return b""
        if op in (GETXATTR, LISTXATTR):
            raise FuseOSError(errno.ENODATA if op == GETXATTR else errno.ENOSYS)
        if op == IOCTL:
            raise FuseOSError(errno.ENOTTY)   # isatty() probes of open(): "not a terminal"
        raise FuseOSError(errno.ENOSYS)


def mount_kernel(ops: AlluxioFuseOps, mountpoint: str, threads: int = 4, allow_other: bool = False,
                 keep_cache: bool = False) -> FuseKernelServer:
    """Mount ``ops`` at ``mountpoint`` through ``/dev/fuse``; returns the running server."""
    return FuseKernelServer(ops, mountpoint, threads, allow_other, keep_cache).mount()
