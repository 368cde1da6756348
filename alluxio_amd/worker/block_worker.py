"""Block worker facade: session-scoped block operations over the native HBM store.

Parity: core/server/worker/src/main/java/alluxio/worker/block/BlockWorker.java:38-429 and
DefaultBlockWorker.java (commitBlock :274-306 -> master CommitBlock; createBlock :321-346;
openUfsBlock :513; metrics :573-616), UnderFileSystemBlockReader (read-through caching of a
cold block: UFS -> staging -> temp block -> commit), AsyncCacheRequestManager.java:60-259
(deduplicated background caching from UFS or a remote worker), Sessions / SessionCleaner
(locks and temp blocks of dead sessions are released).

Data movement on the device tier never goes through Python bytes: reads land in caller buffers
(device pointers via the batched page-gather kernel, host pointers via DMA), writes come from
caller buffers.  ``read_bytes`` exists only for the gRPC byte-stream path used by host clients.
"""
from __future__ import annotations

import logging
import threading
import time
from concurrent.futures import ThreadPoolExecutor

from .. import metrics as msys
from ..ops.native import has_gpu, native_errors
from ..utils.tracing import traced
from ..proto import pb
from ..utils import ids
from ..rpc import marshal
from ..utils.exceptions import (BlockDoesNotExistException, DeadlineExceededException,
                                NotFoundException)
from .store import TieredStore

LOG = logging.getLogger(__name__)

HOST, DEVICE = 0, 1


class _Staging:
    """Pool of pinned host buffers for D2H/H2D staging of byte-stream I/O."""

    def __init__(self, size: int, count: int = 8):
        import torch
        from ..ops.native import has_gpu
        self.size = size
        self._free = [torch.empty(size, dtype=torch.uint8, pin_memory=has_gpu()) for _ in range(count)]
        self._cond = threading.Condition()

    def acquire(self):
        with self._cond:
            while not self._free:
                self._cond.wait()
            return self._free.pop()

    def release(self, t) -> None:
        with self._cond:
            self._free.append(t)
            self._cond.notify()


class BlockWorker:
    def __init__(self, conf, store: TieredStore, master_channel=None, address=None, ufs_resolver=None):
        self.conf = conf
        self.store = store
        self.native = store.native
        self.master_channel = master_channel
        self.address = address or pb.grpc.WorkerNetAddress(host="127.0.0.1")
        self.worker_id = ids.INVALID_WORKER_ID
        self.metrics = msys.metrics("Worker")
        self._ufs_resolver = ufs_resolver
        self._ufs_cache: dict[int, object] = {}
        self._ufs_uris: dict[int, str] = {}     # mount id -> mount point URI in the UFS
        self.native_ufs_roots = None             # csrc LocalUfsRoots of the native data server
        self._sessions: dict[int, float] = {}
        self._session_lock = threading.Lock()
        self._async_inflight: set[int] = set()
        self._async_lock = threading.Lock()
        self._async_pool = ThreadPoolExecutor(
            max_workers=conf.get_int("alluxio.worker.network.async.cache.manager.threads.max"),
            thread_name_prefix="async-cache")
        self._staging = None
        self._staging_lock = threading.Lock()
        self._ingest = None   # K3 pipelines (worker/ingest.py), created on first UFS caching
        self._bulk_buf = None  # pinned staging of the bulk small-file ingest
        self._bulk_lock = threading.Lock()
        self._bulk_threads = conf.get_int("alluxio.worker.ufs.ingest.bulk.threads", "16")
        self.bulk_stats = {"native_s": 0.0, "crc_s": 0.0, "report_s": 0.0}   # where bulk ingest time goes
        self.pinned_files: set[int] = set()
        self.persisted_files: list[int] = []
        self._block_master = None
        self._fs_master = None
        self.transfer_plane = None   # parallel.transfer.TransferPlane when ranks form a node group
        self._peer_channels: dict = {}
        self._peer_lock = threading.Lock()
        self.crc_enabled = conf.get_bool("alluxio.worker.data.crc.enabled")
        # HBM blocks get their per-page CRC32C at commit by default (one kernel pass at ~3.6 TB/s):
        # peers verify pulled blocks against it, short-circuit readers may too
        self.crc_device = conf.get_bool("alluxio.worker.data.crc.device.enabled", "true")
        self.page_check = conf.get_bool("alluxio.worker.debug.page.accounting.check", "false")
        self.crc: dict[int, tuple[int, list[int]]] = {}   # block id -> (piece bytes, CRC32Cs)
        self._install_gauges()

    # ---- wiring -------------------------------------------------------------------------------
    def _bm(self):
        if self._block_master is None and self.master_channel is not None:
            self._block_master = self.master_channel.stub("alluxio.grpc.block.BlockMasterWorkerService")
        return self._block_master

    def _fsm(self):
        if self._fs_master is None and self.master_channel is not None:
            self._fs_master = self.master_channel.stub("alluxio.grpc.file.FileSystemMasterWorkerService")
        return self._fs_master

    def peer_channel(self, address: str):
        """Pooled channel to another worker (GrpcConnectionPool keyed by address)."""
        from ..rpc import Channel
        with self._peer_lock:
            ch = self._peer_channels.get(address)
            if ch is None:
                ch = self._peer_channels[address] = Channel(address)
        return ch

    def peer_stub(self, address: str):
        """BlockWorker stub of another worker (pooled channels)."""
        return self.peer_channel(address).stub("alluxio.grpc.block.BlockWorker")

    def peer_fetcher(self, host: str, port: int, length: int | None):
        """Block source for async caching from a peer: xGMI pull through the transfer plane when
        the peer is in this node's worker group, else the gRPC block stream."""
        plane = self.transfer_plane
        if plane is not None and plane.can_reach((host, port)):
            return lambda block_id: plane.pull_block(block_id, (host, port), length or 0)
        from .remote import remote_block_fetcher
        return remote_block_fetcher(self, host, port, length)

    def _install_gauges(self) -> None:
        m = self.metrics
        m.gauge("CapacityTotal", lambda: sum(self.store.capacity_by_tier().values()))
        m.gauge("CapacityUsed", lambda: sum(self.store.used_by_tier().values()))
        m.gauge("CapacityFree", lambda: sum(self.store.capacity_by_tier().values()) -
                sum(self.store.used_by_tier().values()))
        m.gauge("BlocksCached", lambda: len(self.native.block_ids(-1)))
        hbm = [i for i, a in enumerate(self.store.arenas) if a is not None and a.kind == "hbm"]
        if hbm:
            ps = self.conf.get_bytes("alluxio.worker.hbm.page.size")
            m.gauge("HbmPagesTotal", lambda: sum(self.native.dir_capacity(i) for i in hbm) // ps)
            m.gauge("HbmPagesFree", lambda: sum(self.native.dir_available(i) for i in hbm) // ps)

    def ingest_pool(self):
        from .ingest import IngestPool
        with self._staging_lock:
            if self._ingest is None:
                self._ingest = IngestPool(
                    self, self.conf.get_bytes("alluxio.worker.ufs.ingest.chunk.size", "8MB"),
                    self.conf.get_int("alluxio.worker.ufs.ingest.depth", "3"),
                    self.conf.get_int("alluxio.worker.network.async.cache.manager.threads.max") + 4)
            return self._ingest

    def staging(self) -> _Staging:
        with self._staging_lock:
            if self._staging is None:
                self._staging = _Staging(self.conf.get_bytes("alluxio.worker.network.reader.max.chunk.size.bytes") * 4)
            return self._staging

    # ---- sessions -----------------------------------------------------------------------------
    def session_heartbeat(self, session_id: int) -> None:
        with self._session_lock:
            self._sessions[session_id] = time.time()

    def renew_sessions(self, session_ids) -> list[int]:
        """Heartbeat of sessions a client holds open across calls (short-circuit device reads and
        writes); returns the ids this worker no longer knows (already cleaned up)."""
        now = time.time()
        unknown = []
        with self._session_lock:
            for s in session_ids:
                if s in self._sessions:
                    self._sessions[s] = now
                else:
                    unknown.append(s)
        return unknown

    def cleanup_session(self, session_id: int) -> None:
        with self._session_lock:
            self._sessions.pop(session_id, None)
        with native_errors():
            self.native.cleanup_session(session_id)

    def cleanup_expired_sessions(self, timeout_s: float | None = None) -> list[int]:
        timeout_s = timeout_s if timeout_s is not None else \
            self.conf.get_ms("alluxio.worker.session.timeout") / 1000.0
        now = time.time()
        with self._session_lock:
            dead = [s for s, t in self._sessions.items() if now - t > timeout_s]
        for s in dead:
            self.cleanup_session(s)
        return dead

    # ---- writes -------------------------------------------------------------------------------
    def create_block(self, session_id: int, block_id: int, tier: int = 0, medium: str = "",
                     initial_bytes: int | None = None, pin: bool = False) -> int:
        if initial_bytes is None:
            initial_bytes = self.conf.get_bytes("alluxio.worker.file.buffer.size", "1MB")
        self.session_heartbeat(session_id)
        with native_errors():
            return self.native.create_block(session_id, block_id, tier, medium, max(1, initial_bytes), True, pin)

    def request_space(self, session_id: int, block_id: int, additional: int) -> None:
        with native_errors():
            self.native.request_space(session_id, block_id, additional)

    def write_ptr(self, session_id: int, block_id: int, offset: int, ptr: int, length: int, kind: int,
                  stream: int = 0, sync: bool = True) -> None:
        with native_errors():
            self.native.write(session_id, block_id, offset, ptr, length, kind, stream, sync)

    def write_bytes(self, session_id: int, block_id: int, offset: int, data) -> None:
        import numpy as np
        arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        if arr.nbytes == 0:
            return
        with native_errors():
            self.native.write(session_id, block_id, offset, arr.ctypes.data, arr.nbytes, HOST, 0, True)
        self.metrics.counter("BytesWrittenAlluxio").inc(arr.nbytes)

    def write_tensor(self, session_id: int, block_id: int, offset: int, t, stream: int = 0) -> None:
        kind = DEVICE if t.is_cuda else HOST
        t = t.contiguous()
        self.write_ptr(session_id, block_id, offset, t.data_ptr(), t.numel() * t.element_size(), kind, stream, True)
        self.metrics.counter("BytesWrittenAlluxio").inc(t.numel() * t.element_size())

    def commit_block(self, session_id: int, block_id: int, pin: bool = False, hold: bool = False,
                     crc=None) -> None:
        """Commit a temp block and report it to the master.  ``hold``: a CACHE_THROUGH tee block --
        keep it from eviction until the file's UFS stream has appended it (BlockStore::hold_block,
        released by the AppendBlock copy).  ``crc``: its (piece bytes, CRC32Cs) when the caller
        already computed them (a verified peer pull), so they are not computed twice."""
        with native_errors():
            self.native.commit_block(session_id, block_id, pin)
            if hold:
                self.native.hold_block(block_id)
        # the commit's added-event is reported by CommitBlock already
        self._report_commit(block_id, crc)

    def verify_block_crc(self, block_id: int, src_crcs: list[int], src_piece: int) -> None:
        """Compare the block's bytes against CRC32Cs of ``src_piece``-byte pieces computed by its
        source (its page size, which may differ from ours): both sides are folded into one
        whole-block CRC with crc32c_combine."""
        from ..ops.native import lib
        from ..utils.exceptions import DataLossException
        with native_errors():
            mine = self.native.checksum(block_id, 0)
            length = self.native.block_info(block_id).length
            ps = self.native.block_pages(block_id)[2]
        combine = lib().crc32c_combine

        def fold(crcs, piece):
            acc, left = 0, length
            for i, c in enumerate(crcs):
                n = min(piece, left)
                acc = c if i == 0 else combine(acc, c, n)
                left -= n
            return acc

        if len(src_crcs) != -(-length // src_piece) or fold(src_crcs, src_piece) != fold(mine, ps):
            self.metrics.counter("Crc32cMismatches").inc()
            raise DataLossException(f"block {block_id}: CRC32C mismatch after transfer")
        self.metrics.counter("Crc32cVerifiedBytes").inc(length)
        return ps, list(mine)

    def abort_block(self, session_id: int, block_id: int) -> None:
        with native_errors():
            self.native.abort_block(session_id, block_id)

    # ---- locks / reads ------------------------------------------------------------------------
    def lock_block(self, session_id: int, block_id: int, timeout_ms: int = 30_000, write: bool = False) -> int:
        self.session_heartbeat(session_id)
        with native_errors():
            lid = self.native.lock_block(session_id, block_id, write, timeout_ms)
        if lid < 0:
            raise DeadlineExceededException(f"timed out locking block {block_id}")
        return lid

    def unlock(self, lock_id: int) -> None:
        with native_errors():
            self.native.unlock(lock_id)

    def has_block(self, block_id: int) -> bool:
        return self.native.has_block(block_id)

    def block_info(self, block_id: int):
        with native_errors():
            return self.native.block_info(block_id)

    def access_block(self, session_id: int, block_id: int) -> None:
        with native_errors():
            self.native.access_block(session_id, block_id)

    def read(self, block_id: int, offset: int, length: int, dst_ptr: int, dst_kind: int,
             stream: int = 0, sync: bool = True) -> None:
        with native_errors():
            self.native.read(block_id, offset, length, dst_ptr, dst_kind, stream, sync)
        self._count_read(length, dst_kind)

    def read_batch(self, reqs, stream: int = 0, sync: bool = True) -> int:
        """``reqs`` = [(block_id, offset, length, dst_ptr, dst_kind)]; one gather launch."""
        with native_errors():
            self.native.read_batch(reqs, stream, sync)
        total = sum(r[2] for r in reqs)
        self._count_read(total, reqs[0][4] if reqs else DEVICE)
        return total

    def _count_read(self, n: int, kind: int) -> None:
        self.metrics.counter("BytesReadAlluxio").inc(n)
        if kind == DEVICE:
            self.metrics.counter("BytesReadDevice").inc(n)

    def read_bytes(self, block_id: int, offset: int, length: int) -> bytes:
        """Byte-stream read: the block bytes land directly in a new ``bytes`` object (one copy)."""
        with native_errors():
            out = self.native.read_frame(block_id, offset, length, b"")
        self._count_read(length, HOST)
        return out

    def read_frame(self, block_id: int, offset: int, length: int):
        """One zero-copy ``ReadResponse`` frame of block bytes for the gRPC data server
        (rpc/marshal.py; reference ReadResponseMarshaller)."""
        hdr = marshal.read_response_header(length)
        with native_errors():
            frame = self.native.read_frame(block_id, offset, length, hdr)
        self._count_read(length, HOST)
        return marshal.DataFrame(frame, len(hdr))

    # ---- management ---------------------------------------------------------------------------
    def remove_block(self, session_id: int, block_id: int) -> None:
        with native_errors():
            self.native.remove_block(session_id, block_id)
        self.crc.pop(block_id, None)
        self.metrics.counter("BlocksRemoved").inc()

    def move_block(self, session_id: int, block_id: int, medium: str = "", tier: int = -1) -> int:
        with native_errors():
            return self.native.move_block(session_id, block_id, tier, medium, True)

    def free_space(self, session_id: int, nbytes: int, tier: int = -1) -> list[int]:
        with native_errors():
            return self.native.free_space(session_id, nbytes, tier, -1)

    def checksum(self, block_id: int, piece: int = 0) -> list[int]:
        with native_errors():
            out = self.native.checksum(block_id, piece)
        self.metrics.counter("Crc32cBytes").inc(self.native.block_info(block_id).length)
        return out

    def update_pinned(self, file_ids) -> None:
        self.pinned_files = set(file_ids)
        with native_errors():
            self.native.set_pinned_files(sorted(self.pinned_files))

    # ---- UFS: cold reads + caching ------------------------------------------------------------
    def _ufs_for(self, opts):
        if self._ufs_resolver is not None:
            return self._ufs_resolver(opts.mountId, opts.ufs_path)
        from ..underfs import registry
        u = self._ufs_cache.get(opts.mountId)
        if u is None:
            props = {}
            fsm = self._fsm()
            if fsm is not None and opts.mountId:
                info = fsm.GetUfsInfo(pb.file.GetUfsInfoPRequest(mountId=opts.mountId)).ufsInfo
                props = dict(info.properties.properties)
                if info.uri:
                    self._ufs_uris[opts.mountId] = info.uri
            u = registry.create(opts.ufs_path, self.conf, props)
            self._ufs_cache[opts.mountId] = u
        return u

    def note_ufs_mount(self, mount_id: int, ufs) -> None:
        """After a UFS call served in Python: a mount whose UFS the native data server can reach
        by itself is registered with it, so later calls of that mount stay on its I/O threads --
        a plain local directory (UFS_FILE writes: csrc/data_server.cpp UfsFileWriteStream; cold
        reads: pread) or a plain-HTTP S3 endpoint (cold reads: signed ranged GETs)."""
        from ..underfs.local import LocalUnderFileSystem
        from ..underfs.s3 import S3UnderFileSystem
        roots = self.native_ufs_roots
        if roots is None or not mount_id:
            return
        if type(ufs) is LocalUnderFileSystem:
            uri = self._ufs_uris.get(mount_id)
            if uri is not None and roots.resolve(mount_id, uri.rstrip("/") + "/x") is None:
                roots.set(mount_id, uri)
        elif isinstance(ufs, S3UnderFileSystem) and ufs._native_on and \
                self.conf.get_bool("alluxio.worker.data.server.native.ufs.read.enabled", "true"):
            import urllib.parse
            u = urllib.parse.urlsplit(ufs.client.endpoint)
            if roots.resolve_s3(mount_id, f"s3://{ufs.bucket}/x") is None:
                part, inflight = ufs.upload_shape()
                roots.set_s3(mount_id, u.hostname, u.port or 80, ufs.bucket, ufs.client.access_key,
                             ufs.client.secret_key, ufs.client.region, ufs._parallel, ufs._part, part, inflight,
                             **ufs.http_limits())

    note_local_ufs = note_ufs_mount

    def ufs_block_target(self, mount_id: int, block_id: int):
        """(UFS, path) of the UFS block file of ``block_id`` under mount ``mount_id``
        (BlockUtils.getUfsBlockPath)."""
        from ..underfs import registry
        from .ufs_fallback import ufs_block_path
        fsm = self._fsm()
        if fsm is None:
            raise NotFoundException("no master connection to resolve the UFS of mount %d" % mount_id)
        info = fsm.GetUfsInfo(pb.file.GetUfsInfoPRequest(mountId=mount_id)).ufsInfo
        path = ufs_block_path(info.uri, block_id)
        if self._ufs_resolver is not None:
            return self._ufs_resolver(mount_id, path), path
        return registry.create(path, self.conf, dict(info.properties.properties)), path

    def commit_block_in_ufs(self, block_id: int, length: int) -> None:
        bm = self._bm()
        if bm is not None:
            bm.CommitBlockInUfs(pb.block.CommitBlockInUfsPRequest(blockId=block_id, length=length))
        self.metrics.counter("BlocksCommittedInUfs").inc()

    def read_ufs_range(self, opts, offset: int, length: int, block_id: int = 0) -> bytes:
        from ..underfs.base import OpenOptions
        from .ufs_fallback import resolve_ufs_block_opts
        opts = resolve_ufs_block_opts(self, block_id, opts)
        ufs = self._ufs_for(opts)
        with ufs.open(opts.ufs_path, OpenOptions(offset=opts.offset_in_file + offset)) as f:
            data = f.read(length)
        self.metrics.counter("BytesReadUfsAll").inc(len(data))
        return data

    @traced("Worker.cache_block_from_ufs")
    def cache_block_from_ufs(self, block_id: int, opts, session_id: int | None = None, on_chunk=None,
                             offset: int = 0) -> bool:
        """UFS -> pinned staging ring -> block (async H2D on a side stream for the HBM tier,
        overlapped with the next UFS read: worker/ingest.py) -> commit.  Idempotent.
        ``on_chunk`` sees every chunk as it is ingested (read-through streaming to a client)."""
        if self.native.has_block(block_id):
            return True
        session_id = session_id if session_id is not None else ids.CACHE_UFS_SESSION_ID
        from ..underfs.base import OpenOptions
        from .ufs_fallback import resolve_ufs_block_opts
        opts = resolve_ufs_block_opts(self, block_id, opts)
        ufs = self._ufs_for(opts)
        length = opts.block_size
        try:
            self.create_block(session_id, block_id, 0, "", length or 1)
        except Exception as e:  # noqa: BLE001
            if self.native.has_block(block_id) or self.native.has_temp_block(block_id):
                return self.native.has_block(block_id)
            raise e
        from ..underfs.lz4frame import Lz4FrameUnderFileSystem
        if isinstance(ufs, Lz4FrameUnderFileSystem) and has_gpu() and on_chunk is None:
            idx = ufs.frame_index(opts.ufs_path)
            start = opts.offset_in_file + offset
            if idx is not None and start % idx.block_max == 0:
                try:
                    self._ingest_lz4_frame(session_id, block_id, ufs, opts.ufs_path, idx, start, length)
                    self.commit_block(session_id, block_id)
                    return True
                except Exception:
                    try:
                        self.abort_block(session_id, block_id)
                    except Exception:  # noqa: BLE001
                        pass
                    raise
        pool = self.ingest_pool()
        pipe = pool.acquire()
        try:
            t0 = time.perf_counter()
            with ufs.open(opts.ufs_path, OpenOptions(offset=opts.offset_in_file + offset)) as f:
                pos = pipe.run(session_id, block_id, f, length, on_chunk)
            if pos != length:
                raise IOError(f"short UFS read for block {block_id}: {pos} of {length}")
            self.metrics.counter("BytesReadUfsAll").inc(length)
            self.metrics.counter("UfsIngestBytes").inc(length)
            self.metrics.timer("UfsIngestBlock").update(time.perf_counter() - t0)
            self.commit_block(session_id, block_id)
            return True
        except Exception:
            try:
                self.abort_block(session_id, block_id)
            except Exception:  # noqa: BLE001
                pass
            raise
        finally:
            pool.release(pipe)

    @traced("Worker.ingest_lz4_frame")
    def _ingest_lz4_frame(self, session_id: int, block_id: int, ufs, path: str, idx, start: int,
                          length: int) -> None:
        """Cache decompressed bytes [start, start+length) of an LZ4 frame: the compressed span of
        the frame blocks covering them is read from the UFS in one request, copied to the GPU,
        and decoded by one K11 launch (stored blocks by one batched copy) into a device buffer
        that is then written into the temp block (underfs/lz4frame.py)."""
        import torch

        from ..ops.native import lib
        from ..underfs.base import OpenOptions
        from ..utils.exceptions import DataLossException
        bm = idx.block_max
        j0, j1 = start // bm, -(-(start + length) // bm)
        blocks = idx.blocks[j0:j1]
        lo = blocks[0][0]
        hi = blocks[-1][0] + blocks[-1][1]
        t0 = time.perf_counter()
        host = torch.empty(hi - lo, dtype=torch.uint8, pin_memory=True)
        mv = memoryview(host.numpy())
        got = 0
        with ufs.inner.open(path, OpenOptions(offset=lo)) as f:
            while got < hi - lo:
                n = f.readinto(mv[got:])
                if not n:
                    break
                got += n
        if got != hi - lo:
            raise IOError(f"short read of the LZ4 frame span of block {block_id}: {got} of {hi - lo}")
        dev = torch.device("cuda", self.store.device)
        comp = host.to(dev, non_blocking=True)
        out = torch.empty((j1 - j0) * bm, dtype=torch.uint8, device=dev)
        C = lib()
        chunks, raws, want = [], [], []
        for k, (off, n, raw) in enumerate(blocks):
            src = comp.data_ptr() + off - lo
            dst = out.data_ptr() + k * bm
            want.append(idx.block_len(j0 + k))
            if raw:
                raws.append((src, dst, n))
            else:
                chunks.append((src, dst, n, bm))
        stream = torch.cuda.current_stream(dev).cuda_stream
        if raws:
            C.batched_copy(raws, stream)
        sizes = C.lz4_device(chunks, False, stream) if chunks else []
        it = iter(sizes)
        for k, (off, n, raw) in enumerate(blocks):
            got = n if raw else next(it)
            if got != want[k]:
                raise DataLossException(f"LZ4 frame block {j0 + k} of {path} decoded to {got} bytes, "
                                        f"expected {want[k]}")
        self.write_ptr(session_id, block_id, 0, out.data_ptr() + (start - j0 * bm), length, DEVICE, stream, True)
        self.metrics.counter("BytesReadUfsAll").inc(hi - lo)
        self.metrics.counter("UfsIngestBytes").inc(length)
        self.metrics.counter("Lz4DecodedBytes").inc(length)
        self.metrics.timer("UfsIngestBlock").update(time.perf_counter() - t0)

    @traced("Worker.cache_blocks_from_ufs")
    def cache_blocks_from_ufs(self, items, session_id: int | None = None) -> int:
        """Bulk form of :meth:`cache_block_from_ufs` for many small blocks (``items`` =
        [(block id, OpenUfsBlockOptions)]): blocks of a local UFS are read by the native store's
        thread pool straight into a pinned staging buffer and copied into HBM in batches
        (BlockStore::ingest_files), one Python call for the lot; other UFSes take the per-block
        pipeline.  Returns the number of blocks newly cached."""
        from ..underfs.local import LocalUnderFileSystem, strip_scheme
        from .ufs_fallback import resolve_ufs_block_opts
        session_id = session_id if session_id is not None else ids.CACHE_UFS_SESSION_ID
        native_ids, paths, offs, lens, slow = [], [], [], [], []
        local_mount: dict = {}          # mount id -> is a local UFS (one resolution per mount, not per block)
        for bid, opts in items:
            opts = resolve_ufs_block_opts(self, bid, opts)
            is_local = local_mount.get(opts.mountId)
            if is_local is None or not opts.mountId:
                u = self._ufs_for(opts)
                # local files, or a UFS that names a local file to pread per path (synthetic)
                is_local = (strip_scheme if isinstance(u, LocalUnderFileSystem)
                            else getattr(u, "native_path", None)) or False
                if opts.mountId:
                    local_mount[opts.mountId] = is_local
            npath = is_local(opts.ufs_path) if is_local else None
            if npath and opts.block_size > 0:
                native_ids.append(bid)
                paths.append(npath)
                offs.append(opts.offset_in_file)
                lens.append(opts.block_size)
            else:
                slow.append((bid, opts))
        done = 0
        if native_ids:
            staging, sbytes = self._bulk_staging(max(lens))
            t0 = time.perf_counter()
            with self._bulk_lock, native_errors():
                status = self.native.ingest_files(session_id, native_ids, paths, offs, lens, staging.data_ptr(),
                                                  sbytes, self._bulk_threads, 0)
                if self.page_check:
                    self.check_page_accounting("bulk ingest")
            t1 = time.perf_counter()
            self.metrics.timer("UfsIngestBulk").update(t1 - t0)
            ok = [b for b, st in zip(native_ids, status) if st == 0]
            crcs = self._crcs_of(ok)
            t2 = time.perf_counter()
            committed = []
            for bid, st, n in zip(native_ids, status, lens):
                if st == 0:
                    done += 1
                    self.metrics.counter("BytesReadUfsAll").inc(n)
                    self.metrics.counter("UfsIngestBytes").inc(n)
                    committed.append(bid)
                elif st == 2:
                    LOG.warning("bulk cache: UFS read of block %d failed", bid)
                elif st == 3:
                    slow.append((bid, None))      # no space in one go: leave it to the slow path below
            self._report_commits(committed, crcs)
            bs = self.bulk_stats
            bs["native_s"] += t1 - t0
            bs["crc_s"] += t2 - t1
            bs["report_s"] += time.perf_counter() - t2
        for bid, opts in slow:
            if opts is None:
                continue
            try:
                done += bool(self.cache_block_from_ufs(bid, opts, session_id))
            except Exception:  # noqa: BLE001
                LOG.debug("cache of block %d failed", bid, exc_info=True)
        return done

    def check_page_accounting(self, where: str = "") -> list[str]:
        """Debug check of every arena dir's page accounting (host pool + K7 magazine + block
        pages); returns the violations, each also logged and counted."""
        errs = []
        for i in range(len(self.store.dirs)):
            e = self.native.check_pages(i)
            if e:
                errs.append(f"dir {i}: {e}")
                LOG.error("page accounting violated after %s: dir %d: %s", where or "?", i, e)
        if errs:
            self.metrics.counter("PageAccountingErrors").inc(len(errs))
        return errs

    def _bulk_staging(self, min_item: int):
        import torch
        want = max(self.conf.get_bytes("alluxio.worker.ufs.ingest.bulk.staging.size", "64MB"), 2 * min_item)
        with self._staging_lock:
            if self._bulk_buf is None or self._bulk_buf.numel() < want:
                self._bulk_buf = torch.empty(want, dtype=torch.uint8, pin_memory=has_gpu())
            return self._bulk_buf, self._bulk_buf.numel()

    def _crcs_of(self, block_ids) -> dict:
        """{block id: (piece bytes, per-page CRC32Cs)} of freshly committed blocks that keep CRCs,
        computed by one gathered kernel launch for the HBM ones (BlockStore::checksum_blocks)."""
        if not block_ids or not (self.crc_enabled or self.crc_device):
            return {}
        with native_errors():
            crcs = self.native.checksum_blocks(block_ids, not self.crc_enabled)
        return {bid: (piece, crc) for bid, (piece, crc) in zip(block_ids, crcs) if piece}

    def _report_commit(self, block_id: int, crc=None) -> None:
        """Tell the master about a block committed by the native store (CommitBlock)."""
        info = self.native.block_info(block_id)
        if crc is not None:
            self.crc[block_id] = crc
            self.metrics.counter("Crc32cBytes").inc(info.length)
        elif self.crc_enabled or (self.crc_device and info.medium == "HBM"):
            t0 = time.perf_counter()
            self.crc[block_id] = (self.native.block_pages(block_id)[2], self.native.checksum(block_id, 0))
            self.metrics.timer("Crc32cCommit").update(time.perf_counter() - t0)
            self.metrics.counter("Crc32cBytes").inc(info.length)
        bm = self._bm()
        if bm is not None and self.worker_id != ids.INVALID_WORKER_ID:
            bm.CommitBlock(pb.block.CommitBlockPRequest(
                workerId=self.worker_id, usedBytesOnTier=self.store.used_by_tier().get(info.tier_alias, 0),
                tierAlias=info.tier_alias, blockId=block_id, length=info.length, mediumType=info.medium))
        self.metrics.counter("BlocksCommitted").inc()

    def report_native_commits(self, block_ids, crcs: dict) -> None:
        """Master report of blocks the native committer committed (worker/services.py
        NativeCommitBatch): ``_report_commits`` with the CommitBlocks call retried -- exponential
        back-off from alluxio.user.rpc.retry.base.sleep up to .max.sleep, for at most
        alluxio.user.rpc.retry.max.duration (the reference master client's RetryPolicy) -- before
        the failure goes back to the committer."""
        self._report_commits(block_ids, crcs, retry=True)

    def _commit_rpc(self, call, retry: bool):
        if not retry:
            return call()
        import random
        base = self.conf.get_ms("alluxio.user.rpc.retry.base.sleep") / 1000.0
        cap = self.conf.get_ms("alluxio.user.rpc.retry.max.sleep") / 1000.0
        deadline = time.monotonic() + self.conf.get_ms("alluxio.user.rpc.retry.max.duration") / 1000.0
        attempt = 0
        while True:
            try:
                return call()
            except Exception as e:  # noqa: BLE001
                msg = str(e).upper()
                if "UNIMPLEMENTED" in msg or "UNKNOWN METHOD" in msg:
                    raise                        # not transient: the per-block fallback handles it
                attempt += 1
                pause = min(cap, base * (2 ** (attempt - 1)))
                pause = pause / 2 + random.random() * pause / 2
                if time.monotonic() + pause > deadline:
                    raise
                LOG.warning("block commit report to the master failed (attempt %d), retrying: %s", attempt, e)
                time.sleep(pause)

    def _report_commits(self, block_ids, crcs: dict, retry: bool = False) -> None:
        """``_report_commit`` for a batch of freshly committed blocks: one CommitBlocks call per
        16384 blocks with parallel arrays (falls back to per-block CommitBlock against a master
        without the extension)."""
        if not block_ids:
            return
        native = self.native
        ids_, lens, tix, tiers, mediums, index = [], [], [], [], [], {}
        crc_bytes = 0
        for bid in block_ids:
            info = native.block_info(bid)
            key = (info.tier_alias, info.medium)
            k = index.get(key)
            if k is None:
                k = index[key] = len(tiers)
                tiers.append(info.tier_alias)
                mediums.append(info.medium)
            ids_.append(bid)
            lens.append(info.length)
            tix.append(k)
            crc = crcs.get(bid)
            if crc is not None:
                self.crc[bid] = crc
                crc_bytes += info.length
            elif self.crc_enabled or (self.crc_device and info.medium == "HBM"):
                self.crc[bid] = (native.block_pages(bid)[2], native.checksum(bid, 0))
                crc_bytes += info.length
        if crc_bytes:
            self.metrics.counter("Crc32cBytes").inc(crc_bytes)
        bm = self._bm()
        if bm is not None and self.worker_id != ids.INVALID_WORKER_ID:
            used = self.store.used_by_tier()
            step = 16384
            for i in range(0, len(ids_), step):
                req = pb.block.CommitBlocksPRequest(workerId=self.worker_id, blockIds=ids_[i:i + step],
                                                    lengths=lens[i:i + step], tierIndex=tix[i:i + step],
                                                    tiers=tiers, mediums=mediums, usedBytesOnTiers=used)
                try:
                    self._commit_rpc(lambda: bm.CommitBlocks(req), retry)
                except Exception as e:  # noqa: BLE001 - a master without the extension RPC
                    if "UNIMPLEMENTED" not in str(e).upper() and "unknown method" not in str(e).lower():
                        raise
                    for bid, n, k in zip(ids_[i:i + step], lens[i:i + step], tix[i:i + step]):
                        bm.CommitBlock(pb.block.CommitBlockPRequest(
                            workerId=self.worker_id, usedBytesOnTier=used.get(tiers[k], 0), tierAlias=tiers[k],
                            blockId=bid, length=n, mediumType=mediums[k]))
        self.metrics.counter("BlocksCommitted").inc(len(ids_))

    def async_cache(self, block_id: int, opts=None, source=None, length: int | None = None) -> bool:
        """Deduplicated background caching; returns False if already queued/cached."""
        if self.native.has_block(block_id):
            return False
        with self._async_lock:
            if block_id in self._async_inflight:
                return False
            self._async_inflight.add(block_id)

        def run():
            try:
                if source is not None:
                    source(block_id)
                elif opts is not None:
                    self.cache_block_from_ufs(block_id, opts, ids.ASYNC_CACHE_UFS_SESSION_ID)
                self.metrics.counter("AsyncCacheSucceededBlocks").inc()
            except Exception:  # noqa: BLE001
                LOG.debug("async cache of %d failed", block_id, exc_info=True)
                self.metrics.counter("AsyncCacheFailedBlocks").inc()
            finally:
                with self._async_lock:
                    self._async_inflight.discard(block_id)
        self.metrics.counter("AsyncCacheRequests").inc()
        self._async_pool.submit(run)
        return True

    def wait_async_idle(self, timeout: float = 30.0) -> bool:
        deadline = time.time() + timeout
        while time.time() < deadline:
            with self._async_lock:
                if not self._async_inflight:
                    return True
            time.sleep(0.01)
        return False

    # ---- heartbeat report ---------------------------------------------------------------------
    def drain_report(self):
        """(removed block ids, {(tier alias, medium): [added ids]}) since the last report."""
        removed, added = [], {}
        for ev in self.native.drain_events():
            if ev.kind == 1:
                removed.append(ev.block_id)
                self.crc.pop(ev.block_id, None)   # evicted: its CRCs go with it
                for k in list(added):
                    if ev.block_id in added[k]:
                        added[k].remove(ev.block_id)
            else:
                added.setdefault((ev.tier_alias, ev.medium), []).append(ev.block_id)
        return removed, added

    def current_blocks(self) -> dict:
        out: dict = {}
        for bid in self.native.block_ids(-1):
            info = self.native.block_info(bid)
            out.setdefault((info.tier_alias, info.medium), []).append(bid)
        return out

    def close(self) -> None:
        self._async_pool.shutdown(wait=False, cancel_futures=True)


def not_found(block_id: int) -> NotFoundException:
    return BlockDoesNotExistException(f"Block {block_id} does not exist")
