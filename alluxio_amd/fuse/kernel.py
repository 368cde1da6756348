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

Native mode (default when the extension is built): the ``/dev/fuse`` request loop runs in C++
(csrc/fuse_server.cpp).  LOOKUP/GETATTR are answered from a native attribute cache that this
module fills (every Python getattr, and a whole directory at OPENDIR from one listing); OPEN of a
completed file whose blocks are all in the co-located worker's store (``store=``: the worker's
native BlockStore -- the worker-embedded FUSE deployment) read-locks the blocks natively, and READ,
FLUSH and RELEASE of such handles never reach Python (READ replies gather straight from the DRAM
arena with writev, or D2H-copy from HBM).  Everything else -- mutations, misses, files not cached
locally -- is queued to Python handler threads.  Mutations invalidate the cached attributes.
A LOOKUP miss lists the parent directory once (decoded natively into the cache), OPENDIR does the
same, and READDIRPLUS gives the kernel every entry of a listed directory at once.  ``read_only``
(``-o ro``) negotiates zero-message opens (no OPEN/RELEASE per file); ``passthrough`` hands the
kernel the block file of a single-block file held in a file tier (tmpfs) so its reads bypass us.

Kernel page cache (``keep_cache``): ``"auto"`` (default) keeps it across opens only while the
file's Alluxio file id is unchanged (files are write-once; a re-created path gets a new id),
``True`` always, ``False`` never.
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
WRITE_BATCH = 4096      # write-behind batch of the native server (FuseServer::kOpWriteBatch)
GETXATTR, LISTXATTR, FLUSH, INIT, OPENDIR, READDIR, RELEASEDIR, FSYNCDIR = 22, 23, 25, 26, 27, 28, 29, 30
ACCESS, CREATE, INTERRUPT, DESTROY, BATCH_FORGET, READDIRPLUS, RENAME2 = 34, 35, 36, 38, 42, 44, 45

IOCTL = 39
OP_NAMES = {LOOKUP: "LOOKUP", FORGET: "FORGET", GETATTR: "GETATTR", SETATTR: "SETATTR", MKDIR: "MKDIR",
            UNLINK: "UNLINK", RMDIR: "RMDIR", RENAME: "RENAME", OPEN: "OPEN", READ: "READ", WRITE: "WRITE",
            STATFS: "STATFS", RELEASE: "RELEASE", FSYNC: "FSYNC", GETXATTR: "GETXATTR", LISTXATTR: "LISTXATTR",
            FLUSH: "FLUSH", INIT: "INIT", OPENDIR: "OPENDIR", READDIR: "READDIR", RELEASEDIR: "RELEASEDIR",
            FSYNCDIR: "FSYNCDIR", ACCESS: "ACCESS", CREATE: "CREATE", INTERRUPT: "INTERRUPT", IOCTL: "IOCTL",
            DESTROY: "DESTROY", BATCH_FORGET: "BATCH_FORGET", READDIRPLUS: "READDIRPLUS", RENAME2: "RENAME2"}

IN_HDR = struct.Struct("<IIQQIIII")            # len opcode unique nodeid uid gid pid padding
OUT_HDR = struct.Struct("<IiQ")                # len error unique
ATTR = struct.Struct("<QQQQQQIIIIIIIIII")      # fuse_attr (88 bytes)
ENTRY_HEAD = struct.Struct("<QQQQII")          # nodeid generation entry_valid attr_valid + nsecs
ATTR_OUT_HEAD = struct.Struct("<QII")
INIT_OUT = struct.Struct("<IIIIHHIIHH32x")     # major minor max_readahead flags max_bg cong max_write gran pages align
INIT_OUT_EXT = struct.Struct("<IIIIHHIIHHII24x")  # ... + flags2 max_stack_depth (protocol 7.36 / 7.40)
OPEN_OUT = struct.Struct("<QII")
READ_IN = struct.Struct("<QQIIQII")
WRITE_IN = struct.Struct("<QQIIQII")
SETATTR_IN = struct.Struct("<IIQQQQQQIIIIIIII")
KSTATFS = struct.Struct("<QQQQQIIII24x")
DIRENT = struct.Struct("<QQII")
ENTRY_OUT_SIZE = 40 + 88                       # fuse_entry_out: ENTRY_HEAD + fuse_attr

FATTR_MODE, FATTR_UID, FATTR_GID, FATTR_SIZE = 1 << 0, 1 << 1, 1 << 2, 1 << 3
FATTR_ATIME, FATTR_MTIME = 1 << 4, 1 << 5
FUSE_ASYNC_READ, FUSE_ATOMIC_O_TRUNC, FUSE_BIG_WRITES = 1 << 0, 1 << 3, 1 << 5
FUSE_AUTO_INVAL_DATA, FUSE_NO_OPEN_SUPPORT, FUSE_INIT_EXT = 1 << 12, 1 << 17, 1 << 30
FUSE_MAX_PAGES = 1 << 22
NATIVE_MAX_WRITE = 1 << 20       # native server: 1 MiB WRITE requests (max_pages 256, kernel 4.20+)
FUSE_PASSTHROUGH_HI = 1 << (37 - 32)           # FUSE_PASSTHROUGH, in flags2
FUSE_DO_READDIRPLUS, FUSE_READDIRPLUS_AUTO = 1 << 13, 1 << 14
FOPEN_KEEP_CACHE = 1 << 1
MS_RDONLY, MS_NOSUID, MS_NODEV = 1, 2, 4
MNT_DETACH = 2
MAX_WRITE = 128 << 10
ROOT_ID = 1
TTL_S = 1              # directories / entries (the namespace can change under them)
TTL_COMPLETE_S = 60    # attributes of completed (write-once, immutable) files
RO_HANDLES = 256       # python read handles kept for fh-0 READs (read-only, zero-message opens)


def _ts(t: float) -> tuple[int, int]:
    s = int(t)
    return s, int((t - s) * 1e9)


class FuseKernelServer:
    """Serve ``ops`` at ``mountpoint`` until :meth:`unmount`."""

    def __init__(self, ops: AlluxioFuseOps, mountpoint: str, threads: int = 4, allow_other: bool = False,
                 keep_cache="auto", native: bool | None = None, store=None, session: int = 0,
                 py_threads: int | None = None, read_only: bool = False, passthrough: bool = False,
                 file_ttl_s: int = TTL_COMPLETE_S, write_behind: bool = True):
        self.ops = ops
        # sequential writes gathered by the native server into 8 MiB batches (one Python call each)
        self.write_behind = write_behind
        self._wb_handles: set[int] = set()
        self.file_ttl_s = file_ttl_s
        self.read_only = read_only
        self.passthrough = passthrough
        self.passthrough_active = False
        self._ro_open: dict[str, int] = {}               # fh-0 READs: path -> python read handle (LRU)
        self.keep_cache = keep_cache
        self._keep_mode = 2 if keep_cache == "auto" else (1 if keep_cache else 0)
        self._last_fid: dict[int, int] = {}           # python-path opens: node -> file id (keep_cache auto)
        self.native = native
        self.store = store
        self.session = session
        self.py_threads = py_threads
        self._srv = None
        self._listing: dict[str, threading.Event] = {}   # directory listings in flight (LOOKUP prefetch)
        self._listed: dict[str, float] = {}              # directory -> prefetched until (monotonic s)
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
        self._dir_paths: dict[int, str] = {}         # opendir handle -> directory path
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
                        ctypes.c_ulong(MS_NOSUID | MS_NODEV | (MS_RDONLY if self.read_only else 0)),
                        opts.encode())
        if rc != 0:
            err = ctypes.get_errno()
            os.close(self.fd)
            self.fd = -1
            raise OSError(err, f"mount {self.mountpoint}: {os.strerror(err)}")
        srv_cls = None
        if self.native is not False:
            try:
                from ..ops.native import lib
                srv_cls = getattr(lib(), "FuseServer", None)
            except Exception:  # noqa: BLE001 - extension not built
                srv_cls = None
            if srv_cls is None and self.native:
                self.unmount()
                raise RuntimeError("native FUSE server requested but the extension has no FuseServer")
        if srv_cls is not None:
            native_store = getattr(self.store, "native", self.store)     # TieredStore or BlockStore
            self._srv = srv_cls(self.fd, self.nthreads, native_store, self.session, self._keep_mode)
            for arena in getattr(self.store, "arenas", None) or []:
                if arena is not None and getattr(arena, "fd", -1) >= 0:
                    self._srv.add_arena(arena.base, arena.nbytes, arena.fd)
            self._srv.start()
            target, n = self._py_loop, self.py_threads or self.nthreads
        else:
            target, n = self._loop, self.nthreads
        for i in range(n):
            t = threading.Thread(target=target, name=f"fuse-{i}", daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def unmount(self) -> None:
        if self.fd < 0:
            return
        self._stop.set()
        libc = ctypes.CDLL(None, use_errno=True)
        libc.umount2(self.mountpoint.encode(), MNT_DETACH)
        if self._srv is not None:
            self._srv.stop()                 # native readers poll with a timeout: they exit here
        # Once the detached mount's superblock goes (no file left open on it) the kernel aborts
        # the connection and blocked /dev/fuse readers return ENODEV: join them BEFORE closing the
        # fd, so no reader can call read() on a descriptor number that was closed and reused.
        # Only readers still blocked after that (a file held open elsewhere) are woken by close.
        for t in self._threads:
            t.join(timeout=2)
        fd, self.fd = self.fd, -1
        try:
            os.close(fd)             # aborts the connection: remaining readers return ENODEV / EBADF
        except OSError:
            pass
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
        if self._srv is not None:
            p = self._srv.path_of(nodeid)
            if p is None:
                raise FuseOSError(errno.ESTALE)
            return p
        with self._lock:
            p = self._paths.get(nodeid)
        if p is None:
            raise FuseOSError(errno.ESTALE)
        return p

    def _node(self, path: str) -> int:
        if self._srv is not None:
            return self._srv.node_of(path)
        with self._lock:
            nid = self._ids.get(path)
            if nid is None:
                nid = self._next_id
                self._next_id += 1
                self._ids[path] = nid
                self._paths[nid] = path
            return nid

    def _forget_path(self, path: str) -> None:
        if self._srv is not None:
            self._srv.forget_path(path)
            return
        with self._lock:
            nid = self._ids.pop(path, None)
            if nid is not None and nid != ROOT_ID:
                self._paths.pop(nid, None)
                self._last_fid.pop(nid, None)

    def _moved(self, old: str, new: str) -> None:
        if self._srv is not None:
            self._srv.moved(old, new)
            return
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

    def _attr_ttl(self, a: dict) -> int:
        # a file's size changes while it is written (and at completion): cache attrs only once the
        # file is complete -- Alluxio files are write-once, so a completed file's size is final
        if a.get("st_complete"):
            return self.file_ttl_s
        return TTL_S if stat.S_ISDIR(a["st_mode"]) else 0

    def _entry(self, path: str) -> bytes:
        a, info = self.ops.stat_info(path)
        nid = self._node(path)
        ttl = self._attr_ttl(a)
        self._cache(path, a, info, ttl)
        return ENTRY_HEAD.pack(nid, 0, max(TTL_S, ttl), ttl, 0, 0) + self._attr(nid, a)

    def _cache(self, path: str, a: dict, info, ttl: int) -> None:
        """Hand the attributes (and, for a completed file, its blocks) to the native server."""
        if self._srv is None or ttl <= 0:
            return
        blocks, lens = [], []
        complete = bool(a.get("st_complete")) and not stat.S_ISDIR(a["st_mode"])
        if complete:
            bs = info.blockSizeBytes or 1
            blocks = list(info.blockIds)
            lens = [min(bs, info.length - i * bs) for i in range(len(blocks))]
        self._srv.put_attr(path, self._attr(0, a), ttl * 1000, ttl, int(info.fileId or 0), complete, blocks, lens)

    def _prefetch(self, parent: str, name: str):
        """A LOOKUP missed the native cache: list the parent directory once (one RPC instead of
        one per sibling) and cache every child, so the siblings' LOOKUPs never reach Python.
        Returns (attrs, info) of ``name`` when the listing holds it, else None."""
        import time as _time
        now = _time.monotonic()
        with self._lock:
            ev = self._listing.get(parent)
            mine = ev is None
            if mine:
                if self._listed.get(parent, 0.0) > now:
                    return None                     # listed recently: this miss is a genuine one
                ev = self._listing[parent] = threading.Event()
        if not mine:
            ev.wait(10.0)
            return None
        found = None
        try:
            found = self._list_into_cache(parent, name)
            with self._lock:
                self._listed[parent] = now + self.file_ttl_s
        except (FuseOSError, OSError):
            pass                                    # not a directory / gone: the plain path decides
        finally:
            with self._lock:
                self._listing.pop(parent, None)
            ev.set()
        return found

    def _list_into_cache(self, parent: str, name: str | None = None, entries: list | None = None):
        """One listing of ``parent`` into the native attribute cache (natively decoded when the
        op layer hands out raw replies).  Returns the LOOKUP payload of ``name`` if listed;
        ``entries`` collects (name, mode) for READDIR."""
        chunks = self.ops.list_chunks(parent)
        if chunks is None:
            found = None
            for n, a, info in self.ops.list_infos(parent):
                path = self._child(parent, n)
                self._cache(path, a, info, self._attr_ttl(a))
                if entries is not None:
                    entries.append((n, a["st_mode"]))
                if n == name:
                    found = self._entry_payload(path, a)
            return found
        self._srv.cache_listing(chunks, self.ops.root, self.ops.uid, self.ops.gid, self.file_ttl_s, TTL_S)
        if entries is not None:
            from ..ops.native import lib
            cols = lib().decode_file_infos(chunks)
            for p, folder in zip(cols["paths"], cols["folder"].tolist()):
                entries.append((p.rsplit("/", 1)[-1], stat.S_IFDIR if folder else stat.S_IFREG))
        return None if name is None else self._srv.entry(self._child(parent, name))

    def _entry_payload(self, path: str, a: dict) -> bytes:
        nid = self._node(path)
        ttl = self._attr_ttl(a)
        return ENTRY_HEAD.pack(nid, 0, max(TTL_S, ttl), ttl, 0, 0) + self._attr(nid, a)

    def _mode_of(self, parent: str, name: str) -> int:
        try:
            return self.ops.getattr(self._child(parent, name))["st_mode"]
        except FuseOSError:
            return 0

    def _ro_handle(self, path: str) -> int:
        """Read handle of ``path`` for fh-0 READs of a zero-message-open mount: opened on the first
        READ the native server could not serve, reused, closed least-recently-used first."""
        with self._lock:
            fh = self._ro_open.pop(path, None)
            if fh is not None:
                self._ro_open[path] = fh
                return fh
        fh = self.ops.open(path, os.O_RDONLY)
        drop = []
        with self._lock:
            old = self._ro_open.pop(path, None)
            if old is not None:
                drop.append(old)
            self._ro_open[path] = fh
            while len(self._ro_open) > RO_HANDLES:
                drop.append(self._ro_open.pop(next(iter(self._ro_open))))
        for d in drop:
            try:
                self.ops.release(None, d)
            except FuseOSError:
                pass
        return fh

    def _inval(self, *paths: str) -> None:
        if self._srv is None:
            return
        with self._lock:
            for p in paths:
                self._listed.pop(p.rsplit("/", 1)[0] or "/", None)
        for p in paths:
            self._srv.invalidate(p, True)                              # the path and its subtree
            self._srv.invalidate(p.rsplit("/", 1)[0] or "/", False)    # the parent's own attrs

    def op_stats(self) -> dict:
        """Requests per opcode: {"native": {...}, "python": {...}} (python only without the extension)."""
        if self._srv is None:
            return {"native": {}, "python": {OP_NAMES.get(k, str(k)): v for k, v in sorted(self.op_counts.items())}}
        v = self._srv.stats()
        name = lambda k: OP_NAMES.get(k, str(k))  # noqa: E731
        return {"native": {name(k): v[k] for k in range(64) if v[k]},
                "python": {name(k): v[64 + k] for k in range(64) if v[64 + k]},
                "native_us_per_op": {name(k): round(v[128 + k] / v[k] / 1e3, 2) for k in range(64) if v[k]},
                "read_write_us": round(v[128 + 63] / max(1, v[READ]) / 1e3, 2),
                "native_opens": self._srv.native_opens, "passthrough_opens": self._srv.passthrough_opens, "fallback_opens": self._srv.fallback_opens,
                "native_reads": self._srv.native_reads}

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

    def _py_loop(self) -> None:
        srv = self._srv
        while True:
            reqs = srv.poll(16, 200)
            if not reqs:
                if self._stop.is_set() or not srv.alive:
                    return
                continue
            for unique, op, nodeid, _uid, _gid, _pid, body in reqs:
                try:
                    if op == WRITE_BATCH:
                        self._apply_batch(nodeid, body)
                    else:
                        self._serve(op, unique, nodeid, body)
                except Exception:  # noqa: BLE001 - never kill a serving thread
                    LOG.exception("fuse request failed")

    def _apply_batch(self, nodeid: int, body) -> None:
        """Sequential WRITEs the native server already answered, gathered into one batch
        (csrc/fuse_server.cpp write-behind): written through the handle's output stream; the
        outcome goes back to the server, and a FLUSH / RELEASE of the handle reports a failure."""
        fh, off = struct.unpack_from("<QQ", body)
        err = 0
        try:
            self.ops.write(self._path(nodeid), memoryview(body)[16:], off, fh)
        except FuseOSError as e:
            err = e.errno or errno.EIO
        except OSError as e:
            err = e.errno or errno.EIO
        except Exception:  # noqa: BLE001
            LOG.debug("fuse write batch failed", exc_info=True)
            err = errno.EIO
        self._srv.batch_done(fh, err)

    def _write_behind(self, fh: int) -> None:
        if self._srv is not None and self.write_behind:
            self._srv.register_write_handle(fh, 0)
            with self._lock:
                self._wb_handles.add(fh)

    def _wait_writes(self, fh: int, release: bool = False) -> None:
        """Every batched write of ``fh`` applied (raises the first failure as FuseOSError)."""
        with self._lock:
            registered = fh in self._wb_handles
            if release:
                self._wb_handles.discard(fh)
        if not registered:
            return
        err = self._srv.wait_batches(fh)
        if release:
            self._srv.unregister_write_handle(fh)
        if err:
            raise FuseOSError(err)

    def _reply(self, unique: int, err: int = 0, payload: bytes = b"") -> None:
        if self._srv is not None:
            self._srv.reply(unique, err, payload)
            return
        try:
            os.write(self.fd, OUT_HDR.pack(OUT_HDR.size + len(payload), -err, unique) + payload)
        except OSError as e:
            if e.errno not in (errno.ENOENT, errno.EBADF, errno.ENODEV):   # ENOENT: request interrupted
                raise

    def _dispatch(self, req: bytes) -> None:
        _, op, unique, nodeid, uid, gid, pid, _ = IN_HDR.unpack_from(req)
        self._serve(op, unique, nodeid, memoryview(req)[IN_HDR.size:])

    def _serve(self, op: int, unique: int, nodeid: int, body) -> None:
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
            if self._srv is not None:
                # a listed directory hands the kernel every child's entry + attributes at once
                # (dataset scans such as ImageFolder's): those files need no LOOKUP afterwards
                want |= FUSE_DO_READDIRPLUS | FUSE_READDIRPLUS_AUTO
            if self.read_only and self._srv is not None:
                # zero-message opens (no OPEN/RELEASE per file) + page cache dropped whenever a
                # refreshed attribute shows another mtime/size (a replaced file)
                want |= FUSE_NO_OPEN_SUPPORT | FUSE_AUTO_INVAL_DATA
                if flags & FUSE_NO_OPEN_SUPPORT:
                    self._srv.set_no_open(True)
            elif (self.passthrough and self._srv is not None and self.store is not None and minor >= 40
                  and flags & FUSE_INIT_EXT and len(body) >= 20):
                flags2 = struct.unpack_from("<I", body, 16)[0]
                if flags2 & FUSE_PASSTHROUGH_HI:
                    # opens of blocks held as files (tmpfs tier) hand the kernel the block file:
                    # reads are served by it directly (protocol 7.40 passthrough)
                    self._srv.set_passthrough(True)
                    self.passthrough_active = True
                    return INIT_OUT_EXT.pack(7, 40, max_ra, (flags & want) | FUSE_INIT_EXT, 16, 12, MAX_WRITE, 1,
                                             0, 0, FUSE_PASSTHROUGH_HI, 1)
            max_write, max_pages = MAX_WRITE, 0
            if self._srv is not None and flags & FUSE_MAX_PAGES and not self.read_only:
                # fewer, larger WRITE requests (the native server reads up to 1 MiB + headers)
                want |= FUSE_MAX_PAGES
                max_write, max_pages = NATIVE_MAX_WRITE, NATIVE_MAX_WRITE >> 12
            return INIT_OUT.pack(7, min(minor, 34), max_ra, flags & want, 16, 12, max_write, 1, max_pages, 0)
        if op == DESTROY:
            return b""
        if op == LOOKUP:
            name, _ = self._name(body)
            parent = self._path(nodeid)
            if self._srv is not None:
                hit = self._prefetch(parent, name)
                if hit is not None:
                    return hit
            return self._entry(self._child(parent, name))
        if op == GETATTR:
            path = self._path(nodeid)
            a, info = ops.stat_info(path)
            ttl = self._attr_ttl(a)
            self._cache(path, a, info, ttl)
            return ATTR_OUT_HEAD.pack(ttl, 0, 0) + self._attr(nodeid, a)
        if op == SETATTR:
            f = SETATTR_IN.unpack_from(body)
            valid, fh, size, mode, uid, gid = f[0], f[2], f[3], f[11], f[13], f[14]
            path = self._path(nodeid)
            if fh and valid & FATTR_SIZE:
                self._wait_writes(fh)          # an ftruncate lands after the writes acked before it
            if valid & FATTR_MODE:
                ops.chmod(path, mode)
            if valid & (FATTR_UID | FATTR_GID):
                ops.chown(path, uid if valid & FATTR_UID else -1, gid if valid & FATTR_GID else -1)
            if valid & FATTR_SIZE:
                ops.truncate(path, size, fh or None)
            self._inval(path)
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
            self._inval(path)
            return self._entry(path)
        if op in (UNLINK, RMDIR):
            name, _ = self._name(body)
            path = self._child(self._path(nodeid), name)
            (ops.unlink if op == UNLINK else ops.rmdir)(path)
            self._inval(path)
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
            self._inval(src, dst)
            self._moved(src, dst)
            return b""
        if op == CREATE:
            flags, mode, _umask, _oflags = struct.unpack_from("<IIII", body)
            name, _ = self._name(body, 16)
            path = self._child(self._path(nodeid), name)
            fh = ops.create(path, mode)
            self._inval(path)
            self._write_behind(fh)
            return self._entry(path) + OPEN_OUT.pack(fh, 0, 0)
        if op == OPEN:
            flags = struct.unpack_from("<I", body)[0]
            path = self._path(nodeid)
            if flags & (os.O_WRONLY | os.O_RDWR):
                self._inval(path)
            fh = ops.open(path, flags)
            if flags & (os.O_WRONLY | os.O_RDWR):
                self._write_behind(fh)
            keep = 0
            if flags & (os.O_WRONLY | os.O_RDWR) == 0 and self._keep_mode:
                # completed (write-once) files never change under one file id: keep the kernel
                # page cache across opens (a second epoch over a dataset is served from it)
                if self._keep_mode == 1:
                    keep = FOPEN_KEEP_CACHE
                elif self._srv is not None:
                    keep = FOPEN_KEEP_CACHE if self._srv.keep_open(nodeid, ops.file_id(fh)) else 0
                else:
                    fid = ops.file_id(fh)
                    with self._lock:
                        if fid and self._last_fid.get(nodeid, fid) == fid:
                            keep = FOPEN_KEEP_CACHE
                        self._last_fid[nodeid] = fid
            return OPEN_OUT.pack(fh, keep, 0)
        if op == READ:
            fh, offset, size = READ_IN.unpack_from(body)[:3]
            path = self._path(nodeid)
            if fh == 0:
                fh = self._ro_handle(path)          # zero-message open (read-only mount)
            return bytes(ops.read(path, size, offset, fh))
        if op == WRITE:
            fh, offset, size = WRITE_IN.unpack_from(body)[:3]
            # a write the native server passed up (out of order, or after a batch error) goes after
            # the batches it already acknowledged for this handle
            self._wait_writes(fh)
            data = body[WRITE_IN.size:WRITE_IN.size + size]
            n = ops.write(self._path(nodeid), data, offset, fh)
            return struct.pack("<II", n, 0)
        if op == FLUSH:
            fh = struct.unpack_from("<Q", body)[0]
            self._wait_writes(fh)
            if ops.is_write_handle(fh):
                self._inval(self._path(nodeid))
            ops.flush(None, fh)
            return b""
        if op == FSYNC:
            fh = struct.unpack_from("<Q", body)[0]
            self._wait_writes(fh)              # acknowledged bytes are in the output stream on return
            return b""
        if op == FSYNCDIR:
            return b""
        if op == RELEASE:
            fh = struct.unpack_from("<Q", body)[0]
            try:
                self._wait_writes(fh, release=True)
            except FuseOSError:
                pass                          # reported at FLUSH; release still frees the handle
            try:
                ops.release(None, fh)
            except FuseOSError:
                pass                          # already finished at FLUSH
            return b""
        if op == OPENDIR:
            path = self._path(nodeid)
            entries = [(".", stat.S_IFDIR), ("..", stat.S_IFDIR)]
            if self._srv is not None:
                self._list_into_cache(path, None, entries)
            else:
                entries += [(n, m) for n in ops.readdir(path)[2:] for m in [self._mode_of(path, n)] if m]
            with self._lock:
                h = self._next_dir
                self._next_dir += 1
                self._dirs[h] = entries
                self._dir_paths[h] = path
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
        if op == READDIRPLUS:
            fh, offset, size = READ_IN.unpack_from(body)[:3]
            with self._lock:
                entries = self._dirs.get(fh)
                parent = self._dir_paths.get(fh)
            if entries is None:
                raise FuseOSError(errno.EBADF)
            out = bytearray()
            for i in range(offset, len(entries)):
                name, mode = entries[i]
                nb = name.encode()
                rec = ENTRY_OUT_SIZE + DIRENT.size + len(nb)
                rec_pad = (rec + 7) & ~7
                if len(out) + rec_pad > size:
                    break
                ent = None
                if name not in (".", "..") and self._srv is not None:
                    ent = self._srv.entry(self._child(parent, name))     # cached at OPENDIR
                if ent is None:
                    ent = bytes(ENTRY_OUT_SIZE)            # nodeid 0: "no entry for this one"
                    ino = 0xFFFFFFFF
                else:
                    ino = struct.unpack_from("<Q", ent)[0]
                out += ent + DIRENT.pack(ino, i + 1, len(nb), (mode & 0o170000) >> 12) + nb + b"\0" * (rec_pad - rec)
            return bytes(out)
        if op == RELEASEDIR:
            fh = struct.unpack_from("<Q", body)[0]
            with self._lock:
                self._dirs.pop(fh, None)
                self._dir_paths.pop(fh, None)
            return b""
        if op in (GETXATTR, LISTXATTR):
            raise FuseOSError(errno.ENODATA if op == GETXATTR else errno.ENOSYS)
        if op == IOCTL:
            raise FuseOSError(errno.ENOTTY)   # isatty() probes of open(): "not a terminal"
        raise FuseOSError(errno.ENOSYS)


def mount_kernel(ops: AlluxioFuseOps, mountpoint: str, threads: int = 4, allow_other: bool = False,
                 keep_cache="auto", native: bool | None = None, store=None, session: int = 0,
                 py_threads: int | None = None, read_only: bool = False, passthrough: bool = False,
                 file_ttl_s: int = TTL_COMPLETE_S, write_behind: bool = True) -> FuseKernelServer:
    """Mount ``ops`` at ``mountpoint`` through ``/dev/fuse``; returns the running server.
    ``store``: the co-located worker's native BlockStore (native opens/reads of cached files).
    ``read_only``: ``-o ro`` -- with the native server this also negotiates zero-message opens.
    ``write_behind``: the native server gathers sequential writes into 8 MiB batches."""
    return FuseKernelServer(ops, mountpoint, threads, allow_other, keep_cache, native, store, session,
                            py_threads, read_only, passthrough, file_ttl_s, write_behind).mount()
