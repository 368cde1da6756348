"""File and block streams.

Parity: core/client/fs/src/main/java/alluxio/client/file/AlluxioFileInStream.java:66-434 (block
switching, failed-worker retry, positioned read, passive/async caching trigger :386-420),
AlluxioFileOutStream.java:56-319 (per-block out streams, UFS stream for THROUGH types,
completeFile + async persist on close), block/AlluxioBlockStore.java (source selection :149-224:
local -> remote -> UFS via policy; replicated out streams :281-339), block/stream/
{BlockInStream,BlockOutStream,GrpcDataReader,GrpcDataWriter,LocalFileDataReader}.java.

Readers fill caller buffers: ``bytes`` / ``bytearray`` / numpy / torch tensors.  When the
block's worker lives in this process and the destination is a device tensor, the copy is one
page-gather kernel launch from HBM pages into the tensor (no host round trip).

Host reads (``readinto`` / ``read``) go through the native chunk-buffered reader
(``_C.HostInStream``, csrc/block_source.cpp; the LocalFileDataReader analogue of
LocalFileDataReader.java:58-70): each block reader hands it a native *source* -- the in-process
store, a HIP-IPC-mapped HBM arena (chunks DMA'd D2H into a pinned buffer), a shared DRAM arena, or
a native gRPC ReadBlock stream to the worker's data port -- and a ``read(buf)`` inside the current
chunk is a memcpy with no Python frame, device tensor or RPC per call.
"""
from __future__ import annotations

import io
import logging
import queue
import random
import sys
import threading
import time

import numpy as np

from ..proto import enum_name, pb
from ..rpc import marshal
from ..utils import ids
from ..utils.exceptions import (AlluxioStatusException, NotFoundException, ResourceExhaustedException,
                                UnavailableException)
from .context import SVC_WORKER, FileSystemContext, worker_address_str

LOG = logging.getLogger(__name__)

HOST, DEVICE = 0, 1


def _buffer_ptr(buf):
    """(pointer, nbytes, kind, keepalive) of a writable/readable buffer."""
    # a tensor can only exist once torch is imported: never import it here (a multi-second
    # first import under the module lock would stall every writer thread)
    torch = sys.modules.get("torch")
    if torch is not None and isinstance(buf, torch.Tensor):
        if not buf.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return buf.data_ptr(), buf.numel() * buf.element_size(), DEVICE if buf.is_cuda else HOST, buf
    if isinstance(buf, np.ndarray):
        return buf.ctypes.data, buf.nbytes, HOST, buf
    arr = np.frombuffer(buf, dtype=np.uint8)
    return arr.ctypes.data, arr.nbytes, HOST, arr


# ----------------------------------------------------------------------------------------------
# block readers
class BlockReader:
    length: int

    def read_into(self, offset: int, length: int, ptr: int, kind: int, stream: int = 0) -> None:
        raise NotImplementedError

    def read_bytes(self, offset: int, length: int) -> bytes:
        out = np.empty(length, dtype=np.uint8)
        self.read_into(offset, length, out.ctypes.data, HOST)
        return out.tobytes()

    def native_source(self):
        """A ``_C.BlockSource`` over this block for the native host reader, or None (the reader
        then calls :meth:`read_into` through ``_C.PySource``)."""
        return None

    def close(self) -> None:
        pass


class LocalBlockReader(BlockReader):
    """Reads a block held by a worker in this process (lock for the reader's lifetime)."""

    source = "local"

    def __init__(self, worker, block_id: int, session: int):
        self.w = worker
        self.block_id = block_id
        self.session = session
        self.lock_id = worker.lock_block(session, block_id)
        self.length = worker.block_info(block_id).length
        worker.access_block(session, block_id)

    def read_into(self, offset, length, ptr, kind, stream=0):
        self.w.read(self.block_id, offset, length, ptr, kind, stream, sync=True)

    def native_source(self):
        from ..ops.native import lib
        C = lib()
        info = self.w.native.block_info(self.block_id)
        device = self.w.native.dir_spec(info.dir).kind == C.DirKind.DEVICE
        self._src = C.StoreSource(self.w.native, self.block_id, self.length, device)
        return self._src

    def close(self):
        src, self._src = getattr(self, "_src", None), None
        if src is not None and src.bytes:
            self.w._count_read(src.bytes, 0)      # reads served natively still count as worker I/O
        if self.lock_id is not None:
            try:
                self.w.unlock(self.lock_id)
            finally:
                self.lock_id = None


class _AckQueue:
    """Request iterator for a bidi stream that the reader feeds with acks."""

    def __init__(self, first):
        self.q: queue.Queue = queue.Queue()
        self.q.put(first)

    def __iter__(self):
        while True:
            item = self.q.get()
            if item is None:
                return
            yield item

    def put(self, r):
        self.q.put(r)

    def close(self):
        self.q.put(None)


def _native_call(ctx, address: str, data_address):
    """(host, port, channel id, user, timeout ms, domain socket) for a native gRPC call to a
    worker's data port, or None when the worker is in this process (no socket to skip)."""
    host, port = data_address or tuple(address.rsplit(":", 1))
    ch = ctx.worker_channel(address)
    if ch.is_local:
        return None
    cid = ""
    if ch.auth is not None:
        ch._channel()                 # SASL handshake once per channel; its id authorizes the call
        cid = ch.channel_id or ""
    timeout = int(ctx.conf.get_ms("alluxio.user.streaming.data.timeout", "30sec"))
    from ..rpc import domain_socket_for
    uds = domain_socket_for(address) or ""       # a same-node worker's domain socket
    return host, int(port), cid, ch.user or "", timeout, uds


class GrpcBlockReader(BlockReader):
    """Sequential chunked ReadBlock stream with ``offset_received`` acks (GrpcDataReader)."""

    source = "remote"

    def __init__(self, ctx: FileSystemContext, address: str, block_id: int, length: int, ufs_opts=None,
                 chunk: int | None = None, promote: bool = False, data_address: tuple | None = None):
        self.ctx = ctx
        self.address = address
        # (host, port) of the worker's data server (WorkerNetAddress.dataPort)
        self.data_address = data_address
        self.block_id = block_id
        self.length = length
        self.ufs_opts = ufs_opts
        self.chunk = chunk or ctx.conf.get_bytes("alluxio.user.network.reader.chunk.size.bytes", "1MB")
        self.promote = promote
        self._stream = None
        self._reqs = None
        self._pos = None
        self._buf = b""
        self._buf_off = 0
        self._nsrc = None               # native GrpcBlockSource for large reads (False: unavailable)

    def _open(self, offset):
        self._close_stream()
        req = pb.block.ReadRequest(block_id=self.block_id, offset=offset, length=self.length - offset,
                                   chunk_size=self.chunk, promote=self.promote)
        if self.ufs_opts is not None:
            req.open_ufs_block_options.CopyFrom(self.ufs_opts)
        self._reqs = _AckQueue(req)
        call = self.ctx.worker_channel(self.address).raw_stream(SVC_WORKER, "ReadBlock")
        self._stream = iter(call(iter(self._reqs)))
        self._pos = offset
        self._buf = b""
        self._buf_off = offset

    def _next_chunk(self):
        try:
            resp = next(self._stream)
        except StopIteration:
            return b""
        except Exception as e:  # grpc errors
            import grpc
            if isinstance(e, grpc.RpcError):
                raise AlluxioStatusException.from_status(e.code().value[0], e.details()) from None
            raise
        data = resp.chunk.data
        self._pos += len(data)
        self._reqs.put(pb.block.ReadRequest(offset_received=self._pos))
        return data

    def read_bytes(self, offset, length):
        if self._stream is None or offset < self._buf_off or offset > self._pos:
            self._open(offset)
        out = bytearray()
        while len(out) < length:
            rel = offset + len(out) - self._buf_off
            if rel < len(self._buf):
                take = self._buf[rel:rel + (length - len(out))]
                out += take
                continue
            data = self._next_chunk()
            if not data:
                break
            self._buf_off += len(self._buf)
            self._buf = data
        return bytes(out)

    def read_into(self, offset, length, ptr, kind, stream=0):
        # large reads (a GPU consumer's batch, a host buffer) go through the native client: frames
        # parsed straight into the destination (host) or into pinned chunks DMA'd H2D (device)
        if length >= (1 << 20) and self._nsrc is not False:
            if self._nsrc is None:
                try:
                    self._nsrc = self.native_source() or False
                except Exception:  # noqa: BLE001 - fall back to the grpcio stream
                    LOG.debug("native ReadBlock client unavailable", exc_info=True)
                    self._nsrc = False
            if self._nsrc is not False:
                from ..ops.native import lib, native_errors
                dev = 0
                if kind == DEVICE:
                    import torch
                    dev = torch.cuda.current_device()
                    # the H2D copies run on the native reader's own stream: work queued on the
                    # caller's stream (e.g. the fill of a fresh torch.zeros buffer) finishes first
                    (torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()).synchronize()
                with native_errors():
                    lib().source_read(self._nsrc, offset, length, ptr, kind, dev)
                return
        data = self.read_bytes(offset, length)
        if len(data) != length:
            raise UnavailableException(f"short read of block {self.block_id}: {len(data)}/{length}")
        _copy_bytes_to(data, ptr, kind)

    def native_source(self):
        """The same ReadBlock call made by the native gRPC client (HTTP/2 with libnghttp2, frames
        parsed straight into the reader's buffer; csrc/block_source.cpp) against the data port."""
        conf = self.ctx.conf
        if not conf.get_bool("alluxio.user.native.reader.enabled", "true"):
            return None
        from ..ops.native import lib
        if not lib().FrameRpcServer.grpc_available():
            return None
        call = _native_call(self.ctx, self.address, self.data_address)
        if call is None:
            return None
        host, port, cid, user, timeout, uds = call
        ufs = self.ufs_opts.SerializeToString() if self.ufs_opts is not None else b""
        return lib().GrpcBlockSource(host, port, self.block_id, self.length, self.chunk, ufs, self.promote,
                                     cid, user, timeout, uds)

    def _close_stream(self):
        if self._reqs is not None:
            self._reqs.close()
        if self._stream is not None:
            try:
                for _ in self._stream:
                    pass
            except Exception:  # noqa: BLE001
                pass
        self._stream = None
        self._reqs = None

    def close(self):
        self._close_stream()
        if self._nsrc:
            self._nsrc.close()
        self._nsrc = None


class IpcBlockReader(BlockReader):
    """Short-circuit read of a block held by a same-node worker process: its HBM arena mapped via
    HIP IPC, or its shared DRAM arena mapped via memfd (the analogue of LocalFileDataReader's
    mmap; see alluxio_amd/parallel/ipc.py)."""

    source = "ipc"

    def __init__(self, ctx: FileSystemContext, address: str, block_id: int, session: int):
        import torch
        self.ctx = ctx
        self.address = address
        self.block_id = block_id
        self.session = session
        self.stub = ctx.worker_stub(address)
        self.h = self.stub.OpenDeviceBlock(pb.block.OpenDeviceBlockRequest(block_id=block_id, session_id=session))
        ctx.session_keeper().add(address, session)     # the read lock lives as long as the handle
        from ..ops.native import has_gpu
        self.device = torch.cuda.current_device() if has_gpu() else 0
        try:
            from ..parallel.ipc import map_handle
            map_handle(self.h, self.device)
        except Exception as e:
            self.close()
            raise UnavailableException(f"worker {address} did not share block {block_id}: {e}") from e
        if ctx.conf.get_bool("alluxio.user.short.circuit.verify.crc", "false") and self.h.crc32c:
            from ..parallel.ipc import verify_handle_crc
            try:
                verify_handle_crc(self.h, self.device)
            except Exception:
                self.close()
                raise
        self.length = self.h.length

    def read_into(self, offset, length, ptr, kind, stream=0):
        from ..ops.native import has_gpu
        from ..parallel.ipc import gather_block, map_handle, page_segments
        if kind == DEVICE:
            gather_block(self.h, offset, length, ptr, self.device, stream)
            return
        import ctypes
        if self.h.arena_kind != "dram" and not has_gpu():
            # an HBM arena's mapping is a device address: never memcpy it on the host
            raise UnavailableException(f"block {self.block_id}: HBM arena needs a visible GPU")
        if self.h.arena_kind == "dram":
            # shared host arena -> host buffer: plain memcpy of the page runs
            base = map_handle(self.h, self.device)
            for src, dst, n in page_segments(base, list(self.h.pages), self.h.page_size, offset, length, ptr):
                ctypes.memmove(dst, src, n)
            return
        import torch
        tmp = torch.empty(length, dtype=torch.uint8, device=torch.device("cuda", self.device))
        gather_block(self.h, offset, length, tmp.data_ptr(), self.device, stream)
        host = tmp.cpu()
        ctypes.memmove(ptr, host.data_ptr(), length)

    def native_source(self):
        from ..ops.native import has_gpu, lib
        from ..parallel.ipc import map_handle
        C = lib()
        if self.h.arena_kind == "dram":
            return C.HostArenaSource(map_handle(self.h, self.device), list(self.h.pages), self.h.page_size,
                                     self.h.length)
        if not has_gpu():
            return None
        return C.DeviceArenaSource(map_handle(self.h, self.device), list(self.h.pages), self.h.page_size,
                                   self.h.length, self.device)

    def close(self):
        if self.h is not None:
            try:
                self.stub.UnlockDeviceBlock(pb.block.UnlockDeviceBlockRequest(
                    block_id=self.block_id, lock_id=self.h.lock_id, session_id=self.session))
            except Exception:  # noqa: BLE001
                LOG.debug("unlock of device block %d failed", self.block_id, exc_info=True)
            self.ctx.session_keeper().remove(self.address, self.session)
            self.h = None


def _native_opener(stream: "FileInStream"):
    """opener(idx, failed) for ``_C.HostInStream`` holding only a weak reference to the stream
    (the native object must not keep its FileInStream alive)."""
    import weakref
    ref = weakref.ref(stream)

    def opener(idx: int, failed: bool):
        s = ref()
        if s is None:
            raise ValueError("I/O operation on closed file")
        return s._open_native(idx, failed)
    return opener


def _copy_bytes_to(data: bytes, ptr: int, kind: int) -> None:
    import ctypes
    if kind == HOST:
        ctypes.memmove(ptr, data, len(data))
        return
    import torch
    src = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy())
    from ..ops.native import lib
    pinned = src.pin_memory()
    dst = torch.cuda.current_stream()
    # H2D via the runtime copy engine into the raw device pointer
    tmp = torch.empty(len(data), dtype=torch.uint8, device="cuda")
    tmp.copy_(pinned)
    lib().batched_copy([(tmp.data_ptr(), ptr, len(data))], int(dst.cuda_stream))


# ----------------------------------------------------------------------------------------------
class FileInStream(io.RawIOBase):
    def __init__(self, ctx: FileSystemContext, status, read_type: str = "CACHE", options=None):
        super().__init__()
        self.ctx = ctx
        self.status = status
        self.read_type = read_type
        self.length = status.length
        self.block_size = status.blockSizeBytes or (64 << 20)
        self._pos = 0
        self.session = ids.create_session_id()
        self._reader: BlockReader | None = None
        self._reader_idx = -1
        self._failed: dict[str, int] = {}
        self.passive_cache = ctx.conf.get_bool("alluxio.user.file.passive.cache.enabled")
        self.bytes_read = 0
        # native host reader (see module docstring): owns the position while it is active
        self._nat = None
        self._nreader: BlockReader | None = None
        if self.length > 0 and ctx.conf.get_bool("alluxio.user.native.reader.enabled", "true"):
            from ..ops.native import lib
            self._nat = lib().HostInStream(self.length, self.block_size,
                                           ctx.conf.get_bytes("alluxio.user.native.reader.buffer.size", "4MB"),
                                           _native_opener(self),
                                           ctx.conf.get_bool("alluxio.user.native.reader.prefetch.enabled", "true"),
                                           ctx.conf.get_bool("alluxio.user.native.reader.next.block.start.enabled",
                                                             "false"))
            # instance attribute: read(buf) loops call the C entry point directly
            self.readinto = self._nat.fast_readinto

    # ---- io.RawIOBase -------------------------------------------------------------------------
    def readable(self):
        return True

    def seekable(self):
        return True

    @property
    def pos(self) -> int:
        return self._nat.pos if self._nat is not None else self._pos

    @pos.setter
    def pos(self, v: int) -> None:
        if self._nat is not None:
            self._nat.pos = v
        else:
            self._pos = v

    def tell(self):
        return self.pos

    def seek(self, off, whence=io.SEEK_SET):
        new = {io.SEEK_SET: off, io.SEEK_CUR: self.pos + off, io.SEEK_END: self.length + off}[whence]
        if new < 0:
            raise ValueError("negative seek position")
        self.pos = min(new, self.length)
        return self.pos

    def readinto(self, b) -> int:
        mv = memoryview(b).cast("B")
        n = min(len(mv), self.length - self.pos)
        if n <= 0:
            return 0
        arr = np.frombuffer(mv, dtype=np.uint8, count=n)
        self._read_range(self.pos, n, arr.ctypes.data, HOST)
        self.pos += n
        return n

    def read(self, size=-1) -> bytes:
        if size is None or size < 0:
            size = self.length - self.pos
        size = min(size, self.length - self.pos)
        if size <= 0:
            return b""
        if self._nat is not None:
            return self._nat.read(size)
        out = np.empty(size, dtype=np.uint8)
        self._read_range(self.pos, size, out.ctypes.data, HOST)
        self.pos += size
        return out.tobytes()

    def readall(self):
        return self.read(-1)

    # ---- buffer API ---------------------------------------------------------------------------
    def read_into(self, buf, nbytes: int | None = None, stream: int = 0) -> int:
        """Read up to ``len(buf)`` bytes at the current position into a host/device buffer."""
        ptr, cap, kind, _keep = _buffer_ptr(buf)
        n = min(cap if nbytes is None else nbytes, self.length - self.pos)
        if n <= 0:
            return 0
        if kind == HOST and self._nat is not None:
            if n > self.block_size and self._read_blocks_parallel(self.pos, n, ptr, HOST, stream):
                self.pos += n
                return n
            return self._nat.read_ptr(ptr, n)
        self._read_range(self.pos, n, ptr, kind, stream)
        self.pos += n
        return n

    def pread(self, position: int, buf, nbytes: int | None = None) -> int:
        """Positioned read that does not move the stream position."""
        ptr, cap, kind, _keep = _buffer_ptr(buf)
        n = min(cap if nbytes is None else nbytes, self.length - position)
        if n <= 0:
            return 0
        self._read_range(position, n, ptr, kind)
        return n

    # ---- internals ----------------------------------------------------------------------------
    def _read_range(self, pos: int, n: int, ptr: int, kind: int, stream: int = 0) -> None:
        if n > self.block_size and self._read_blocks_parallel(pos, n, ptr, kind, stream):
            return
        done = 0
        while done < n:
            idx = (pos + done) // self.block_size
            off = (pos + done) - idx * self.block_size
            reader = self._reader_for(idx)
            take = min(n - done, reader.length - off)
            if take <= 0:
                raise UnavailableException(f"block {idx} of {self.status.path} is shorter than expected")
            reader.read_into(off, take, ptr + done, kind, stream)
            done += take
        self.bytes_read += n
        self.ctx.metrics.counter("BytesReadClient").inc(n)
        if kind == DEVICE:
            self.ctx.metrics.counter("BytesReadDevice").inc(n)

    def _read_blocks_parallel(self, pos: int, n: int, ptr: int, kind: int, stream: int) -> bool:
        """A read into host or device memory spanning several blocks of remote workers: each
        block is its own ReadBlock stream on the native client (host: frames parsed into the
        destination; device: into pinned chunks DMA'd H2D), up to
        ``alluxio.user.device.read.parallelism`` of them at once, so one consumer is not bound by
        a single stream.  False (nothing read) when the first block is not remote."""
        par = self.ctx.conf.get_int("alluxio.user.device.read.parallelism", "4")
        if par <= 1:
            return False
        pieces = []
        done = 0
        while done < n:
            idx = (pos + done) // self.block_size
            off = (pos + done) - idx * self.block_size
            take = min(n - done, self.block_size - off)
            pieces.append((idx, off, take, done))
            done += take
        first = self._reader_for(pieces[0][0])
        if not isinstance(first, GrpcBlockReader):
            return False
        from concurrent.futures import ThreadPoolExecutor
        dev = None
        if kind == DEVICE:
            import torch
            dev = torch.cuda.current_device()
            # work queued on the caller's stream may still write the buffer (see GrpcBlockReader)
            (torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()).synchronize()

        def one(piece):
            idx, off, take, at = piece
            if dev is not None:
                import torch
                torch.cuda.set_device(dev)
            r = first if idx == pieces[0][0] else self._open_block(self.status.fileBlockInfos[idx], idx)
            try:
                if off + take > r.length:
                    raise UnavailableException(f"block {idx} of {self.status.path} is shorter than expected")
                r.read_into(off, take, ptr + at, kind, 0)
            finally:
                if r is not first:
                    r.close()
        with ThreadPoolExecutor(max_workers=min(par, len(pieces)), thread_name_prefix="block-read") as ex:
            for f in [ex.submit(one, p) for p in pieces]:
                f.result()
        self.bytes_read += n
        self.ctx.metrics.counter("BytesReadClient").inc(n)
        if kind == DEVICE:
            self.ctx.metrics.counter("BytesReadDevice").inc(n)
        return True

    def _reader_for(self, idx: int) -> BlockReader:
        if self._reader is not None and self._reader_idx == idx:
            return self._reader
        self._close_reader()
        fbi = self.status.fileBlockInfos[idx]
        self._reader = self._open_block(fbi, idx)
        self._reader_idx = idx
        return self._reader

    def _open_block(self, fbi, idx: int) -> BlockReader:
        bi = fbi.blockInfo
        block_len = bi.length if bi.length else min(self.block_size, self.length - idx * self.block_size)
        locs = [l for l in bi.locations if worker_address_str(l.workerAddress) not in self._failed]
        inproc = [l for l in locs if self.ctx.in_process_worker(l.workerAddress) is not None]
        last_err = None
        # 1) a worker in this process holding the block
        for l in inproc:
            w = self.ctx.in_process_worker(l.workerAddress)
            try:
                return LocalBlockReader(w, bi.blockId, self.session)
            except NotFoundException as e:
                last_err = e
                self._failed[worker_address_str(l.workerAddress)] = 1
        # 2) a remote (or same-node, other process) worker over the data server
        others = [l for l in locs if l not in inproc]
        others.sort(key=lambda l: 0 if self.ctx.is_local(l.workerAddress) else 1)
        for l in others:
            addr = worker_address_str(l.workerAddress)
            if self.ctx.is_local(l.workerAddress) and self._ipc_enabled(l.workerAddress):
                try:
                    return IpcBlockReader(self.ctx, addr, bi.blockId, self.session)
                except Exception:  # noqa: BLE001 - not in the HBM tier / IPC unsupported: use gRPC
                    LOG.debug("IPC read of block %d from %s unavailable", bi.blockId, addr, exc_info=True)
            if self.ctx.is_local(l.workerAddress):
                self.ctx._note_domain_socket(l.workerAddress)
            try:
                # CACHE_PROMOTE: the worker moves the block to its top tier first (reference
                # BlockInStream: ReadRequest.promote = the read type's isPromote())
                r = GrpcBlockReader(self.ctx, addr, bi.blockId, block_len,
                                    data_address=(l.workerAddress.host,
                                                  l.workerAddress.dataPort or l.workerAddress.rpcPort),
                                    promote=self.read_type == "CACHE_PROMOTE")
                self._maybe_passive_cache(bi.blockId, l.workerAddress, block_len)
                return r
            except Exception as e:  # noqa: BLE001
                last_err = e
                self._failed[addr] = 1
        # 3) UFS through a worker chosen by the UFS read policy: the file in the UFS, or -- for a
        # not yet persisted file whose block went to the UFS tier -- the block's UFS block file
        opts = None
        if self.status.persisted and self.status.ufsPath:
            opts = pb.dataserver.OpenUfsBlockOptions(
                ufs_path=self.status.ufsPath, offset_in_file=idx * self.block_size, block_size=block_len,
                mountId=self.status.mountId, no_cache=self.read_type == "NO_CACHE")
        elif not self.status.persisted and not locs and block_len > 0:
            opts = pb.dataserver.OpenUfsBlockOptions(block_in_ufs_tier=True, block_size=block_len,
                                                     mountId=self.status.mountId,
                                                     no_cache=self.read_type == "NO_CACHE")
        if opts is not None:
            from .policy import create_policy
            pol = create_policy(self.ctx.conf.get("alluxio.user.ufs.block.read.location.policy"), self.ctx.conf)
            workers = self.ctx.workers()
            w = pol.get_worker(workers, bi.blockId, block_len, self.ctx) if workers else None
            if w is not None:
                lw = self.ctx.in_process_worker(w.address)
                if lw is not None and not opts.no_cache:
                    lw.cache_block_from_ufs(bi.blockId, opts, self.session)
                    self.ctx.metrics.counter("BytesReadUfs").inc(block_len)
                    return LocalBlockReader(lw, bi.blockId, self.session)
                return GrpcBlockReader(self.ctx, worker_address_str(w.address), bi.blockId, block_len, ufs_opts=opts,
                                       data_address=(w.address.host, w.address.dataPort or w.address.rpcPort))
        raise UnavailableException(f"Block {bi.blockId} of {self.status.path} is not available "
                                   f"(no live location{'' if self.status.persisted else ', not persisted'})"
                                   + (f": {last_err}" if last_err else ""))

    def _ipc_enabled(self, addr=None) -> bool:
        """The IPC short circuit for a same-node worker: on when short circuit is enabled and either
        the worker has no domain socket or short circuit is preferred over it (reference
        BlockInStream.java:116-124)."""
        conf = self.ctx.conf
        if not conf.get_bool("alluxio.worker.ipc.enabled", "true") or \
                not conf.get_bool("alluxio.user.short.circuit.enabled", "true"):
            return False
        if addr is not None and addr.domainSocketPath and \
                not conf.get_bool("alluxio.user.short.circuit.preferred", "false"):
            return False
        return True

    def _maybe_passive_cache(self, block_id: int, source_addr, length: int) -> None:
        if not self.passive_cache or self.read_type == "NO_CACHE":
            return
        for w in self.ctx.workers():
            if self.ctx.is_local(w.address) and worker_address_str(w.address) != worker_address_str(source_addr):
                try:
                    self.ctx.worker_stub(worker_address_str(w.address)).AsyncCache(pb.block.AsyncCacheRequest(
                        block_id=block_id, source_host=source_addr.host, source_port=source_addr.rpcPort,
                        length=length))
                except Exception:  # noqa: BLE001
                    LOG.debug("passive cache request failed", exc_info=True)
                return

    def _open_native(self, idx: int, failed: bool):
        """Source of block ``idx`` for the native reader (``failed``: its previous source broke,
        so that worker is skipped like a failed location of the Python path)."""
        if failed and self._nreader is not None:
            addr = getattr(self._nreader, "address", None)
            if addr:
                self._failed[addr] = 1
        self._close_nreader()
        reader = self._open_block(self.status.fileBlockInfos[idx], idx)
        self._nreader = reader
        src = None
        try:
            src = reader.native_source()
        except Exception:  # noqa: BLE001 - e.g. no data port: the Python reader serves the bytes
            LOG.debug("native source of block %d unavailable", idx, exc_info=True)
        if src is None:
            from ..ops.native import lib
            src = lib().PySource(reader, reader.length)
        return src

    def _close_nreader(self) -> None:
        if self._nreader is not None:
            try:
                self._nreader.close()
            finally:
                self._nreader = None

    def _close_reader(self) -> None:
        if self._reader is not None:
            try:
                self._reader.close()
            finally:
                self._reader = None
                self._reader_idx = -1

    def close(self) -> None:
        if not self.closed:
            self._close_reader()
            if self._nat is not None:
                n = self._nat.bytes_read
                if n:
                    self.bytes_read += n
                    self.ctx.metrics.counter("BytesReadClient").inc(n)
                pos = self._nat.pos
                self._nat.close()
                self.__dict__.pop("readinto", None)
                self._nat = None
                self._pos = pos
            self._close_nreader()
        super().close()


# ----------------------------------------------------------------------------------------------
# writers
class BlockWriter:
    def write_ptr(self, offset, ptr, length, kind) -> None:
        raise NotImplementedError

    def commit(self, hold_for_append: bool = False) -> None:
        """Commit the block.  ``hold_for_append``: the worker keeps it from eviction until the
        file's UFS stream appends it (CACHE_THROUGH tee)."""
        raise NotImplementedError

    def cancel(self) -> None:
        raise NotImplementedError


class LocalBlockWriter(BlockWriter):
    def __init__(self, worker, block_id, session, tier=0, medium="", initial=1 << 20, pin=False):
        self.w = worker
        self.block_id = block_id
        self.session = session
        worker.create_block(session, block_id, tier, medium, initial, pin)
        self.pin = pin

    def write_ptr(self, offset, ptr, length, kind):
        self.w.write_ptr(self.session, self.block_id, offset, ptr, length, kind)

    def commit(self, hold_for_append=False):
        self.w.commit_block(self.session, self.block_id, self.pin, hold_for_append)

    def cancel(self):
        try:
            self.w.abort_block(self.session, self.block_id)
        except Exception:  # noqa: BLE001
            pass


class LocalUfsFallbackWriter(BlockWriter):
    """In-process worker write with the UFS tier (worker/ufs_fallback.py)."""

    def __init__(self, worker, block_id, session, mount_id, tier=0, medium="", initial=1 << 20):
        from ..worker.ufs_fallback import UfsFallbackBlockWriter
        self._w = UfsFallbackBlockWriter(worker, session, block_id, mount_id, tier, medium, initial)

    def write_ptr(self, offset, ptr, length, kind):
        self._w.write_ptr(offset, ptr, length, kind)

    def commit(self, hold_for_append=False):
        self._w.commit()

    def cancel(self):
        self._w.cancel()


class IpcBlockWriter(BlockWriter):
    """Short-circuit write into a same-node worker process (the analogue of the reference's
    LocalFileDataWriter over CreateLocalBlock): the worker creates the temp block with its pages
    reserved (``OpenDeviceWrite``), this process maps the arena -- HBM through HIP IPC, DRAM through
    the memfd -- and copies into the pages itself (csrc/block_source.cpp ``ArenaSink``: pinned
    staging + H2D DMA), then ``CommitDeviceWrite`` records the length and commits."""

    def __init__(self, ctx, address, block_id, capacity, tier=0, medium="", pin=False):
        from ..ops.native import has_gpu, lib
        from ..parallel.ipc import map_handle
        self.ctx = ctx
        self.block_id = block_id
        self.pin = pin
        self.address = address
        self.stub = ctx.worker_stub(address)
        self.h = self.stub.OpenDeviceWrite(pb.block.OpenDeviceWriteRequest(
            block_id=block_id, length=capacity, tier=tier, medium_type=medium, pin_on_create=pin))
        self.session = self.h.lock_id
        # renewed until commit/cancel: an expired session would hand the reserved pages, which this
        # process keeps writing through its mapping, to another block
        ctx.session_keeper().add(address, self.session)
        try:
            if self.h.arena_kind != "dram" and not has_gpu():
                raise UnavailableException("HBM arena needs a visible GPU")
            import torch
            self.device = torch.cuda.current_device() if has_gpu() else 0
            base = map_handle(self.h, self.device)
            self.sink = lib().ArenaSink(base, list(self.h.pages), self.h.page_size, self.h.length, self.device,
                                        self.h.arena_kind == "dram")
        except Exception:
            self.cancel()
            raise

    def write_ptr(self, offset, ptr, length, kind):
        from ..ops.native import native_errors
        keep = None
        if kind == DEVICE:
            import torch
            from ..ops.native import lib
            tmp = torch.empty(length, dtype=torch.uint8, device="cuda")
            lib().batched_copy([(ptr, tmp.data_ptr(), length)], 0)
            keep = tmp.cpu()
            ptr = keep.data_ptr()
        with native_errors():
            self.sink.write_ptr(offset, ptr, length)

    def commit(self, hold_for_append=False):
        if self.h is None:
            return
        h, self.h = self.h, None
        try:
            self.stub.CommitDeviceWrite(pb.block.CommitDeviceWriteRequest(
                block_id=self.block_id, session_id=self.session, length=self.sink.length, pin_on_create=self.pin,
                hold_for_append=hold_for_append))
        finally:
            self.ctx.session_keeper().remove(self.address, self.session)

    def cancel(self):
        if self.h is None:
            return
        self.h = None
        try:
            self.stub.CommitDeviceWrite(pb.block.CommitDeviceWriteRequest(
                block_id=self.block_id, session_id=self.session, abort=True))
        except Exception:  # noqa: BLE001 - the session expires on the worker
            LOG.debug("abort of short-circuit write of block %d failed", self.block_id, exc_info=True)
        self.ctx.session_keeper().remove(self.address, self.session)


class GrpcBlockWriter(BlockWriter):
    """WriteBlock stream (GrpcDataWriter): command, chunks, then half-close -> commit."""

    def __init__(self, ctx, address, block_id, tier=0, medium="", reserve=1 << 20, pin=False,
                 chunk: int | None = None, ufs_fallback_mount: int | None = None, data_address: tuple | None = None):
        self.chunk = chunk or ctx.conf.get_bytes("alluxio.user.network.writer.chunk.size.bytes", "1MB")
        self._sink = None
        self.address = address
        if ufs_fallback_mount is None and ctx.conf.get_bool("alluxio.user.native.writer.enabled", "true"):
            # the same WriteBlock call made by the native gRPC client (csrc/block_source.cpp
            # GrpcBlockSink): chunks framed around the caller's bytes, GIL released while sending
            from ..ops.native import lib, native_errors
            if lib().FrameRpcServer.grpc_available():
                call = _native_call(ctx, address, data_address)
                if call is not None:
                    host, port, cid, user, timeout, uds = call
                    with native_errors():
                        self._sink = lib().GrpcBlockSink(host, port, block_id, tier, medium, reserve, pin,
                                                         self.chunk, cid, user, timeout, uds)
                    return
        cmd = pb.block.WriteRequestCommand(type=0, id=block_id, offset=0, tier=tier, medium_type=medium,
                                           space_to_reserve=reserve, pin_on_create=pin)
        if ufs_fallback_mount is not None:
            # UFS_FALLBACK_BLOCK: the worker spills the block to the UFS when it is out of space
            cmd.type = 2
            cmd.create_ufs_block_options.mount_id = ufs_fallback_mount
        self._reqs = _AckQueue(pb.block.WriteRequest(command=cmd))
        call = ctx.worker_channel(address).raw_stream(SVC_WORKER, "WriteBlock")
        self._resp = call(iter(self._reqs))
        self._result = []
        self._err = []

        def drain():
            try:
                for r in self._resp:
                    self._result.append(r)
            except Exception as e:  # noqa: BLE001
                self._err.append(e)
        self._t = threading.Thread(target=drain, daemon=True)
        self._t.start()

    def write_ptr(self, offset, ptr, length, kind):
        if self._sink is not None:
            from ..ops.native import native_errors
            from ..utils import optiming
            keep = None
            if kind == DEVICE:
                import torch
                from ..ops.native import lib
                tmp = torch.empty(length, dtype=torch.uint8, device="cuda")
                lib().batched_copy([(ptr, tmp.data_ptr(), length)], 0)
                keep = tmp.cpu()
                ptr = keep.data_ptr()
            t0 = time.perf_counter() if optiming.ENABLED else 0.0
            with native_errors():
                self._sink.write_ptr(ptr, length)
            if optiming.ENABLED:
                optiming.add("client.sink_write", time.perf_counter() - t0)
            return
        if kind == DEVICE:
            import torch
            from ..ops.native import lib
            tmp = torch.empty(length, dtype=torch.uint8, device="cuda")
            lib().batched_copy([(ptr, tmp.data_ptr(), length)], 0)
            data = tmp.cpu().numpy().tobytes()
        else:
            data = _host_view(ptr, length)      # frames copy the bytes, so a view suffices
        mv = memoryview(data)
        for i in range(0, len(data), self.chunk):
            self._reqs.put(marshal.write_request_frame(mv[i:i + self.chunk]))

    def commit(self, hold_for_append=False):
        if self._sink is not None:
            from ..ops.native import native_errors
            sink, self._sink = self._sink, None
            with native_errors():
                sink.commit(hold_for_append)
            return
        if hold_for_append:
            self._reqs.put(pb.block.WriteRequest(command=pb.block.WriteRequestCommand(hold_for_append=True)))
        self._reqs.close()
        self._t.join()
        if self._err:
            e = self._err[0]
            import grpc
            if isinstance(e, grpc.RpcError):
                raise AlluxioStatusException.from_status(e.code().value[0], e.details())
            raise e

    def cancel(self):
        if self._sink is not None:
            sink, self._sink = self._sink, None
            sink.cancel()
            return
        if not hasattr(self, "_reqs"):
            return                      # a native stream already committed or cancelled
        try:
            self._resp.cancel()
        except Exception:  # noqa: BLE001
            pass
        self._reqs.close()


def _host_view(ptr: int, n: int) -> memoryview:
    """A byte memoryview over host memory at ``ptr`` (no copy); valid while the owner lives."""
    import ctypes
    return memoryview((ctypes.c_ubyte * n).from_address(ptr)).cast("B")


class UfsWriter:
    """THROUGH / CACHE_THROUGH UFS stream (via the local worker's UFS client or a WriteBlock
    UFS_FILE stream to a worker — reference UfsFileWriteHandler).  The remote stream is the
    native gRPC client (``GrpcBlockSink`` with the UFS_FILE command) unless
    ``alluxio.user.native.writer.enabled`` is off."""

    def __init__(self, ctx, status, worker_addr=None, local_worker=None, worker=None):
        self.length = 0
        self.worker_addr = worker_addr
        self._local = None
        self._grpc = None
        self._sink = None
        opts = pb.dataserver.CreateUfsFileOptions(ufs_path=status.ufsPath, owner=status.owner, group=status.group,
                                                  mode=status.mode, mount_id=status.mountId)
        if local_worker is not None:
            from ..underfs.base import CreateOptions
            ufs = local_worker._ufs_for(pb.dataserver.OpenUfsBlockOptions(ufs_path=status.ufsPath,
                                                                          mountId=status.mountId))
            self._local = ufs.create(status.ufsPath, CreateOptions(create_parent=True, ensure_atomic=True,
                                                                   mode=status.mode or 0o644))
            self._ufs = ufs
            self._path = status.ufsPath
            return
        cmd = pb.block.WriteRequestCommand(type=1, id=status.fileId, create_ufs_file_options=opts)
        if worker is not None and ctx.conf.get_bool("alluxio.user.native.writer.enabled", "true"):
            from ..ops.native import lib, native_errors
            if lib().FrameRpcServer.grpc_available():
                call = _native_call(ctx, worker_addr, (worker.host, worker.dataPort or worker.rpcPort))
                if call is not None:
                    host, port, cid, user, timeout, uds = call
                    chunk = ctx.conf.get_bytes("alluxio.user.network.writer.chunk.size.bytes", "1MB")
                    with native_errors():
                        self._sink = lib().GrpcBlockSink(host, port, status.fileId, chunk=chunk, channel_id=cid,
                                                         user=user, timeout_ms=timeout, unix_path=uds,
                                                         command=cmd.SerializeToString())
                    return
        self._q = _AckQueue(pb.block.WriteRequest(command=cmd))
        call = ctx.worker_channel(worker_addr).raw_stream(SVC_WORKER, "WriteBlock")
        self._grpc = call(iter(self._q))
        self._err = []
        self._t = threading.Thread(target=self._drain, daemon=True)
        self._t.start()

    def _drain(self):
        try:
            for _ in self._grpc:
                pass
        except Exception as e:  # noqa: BLE001
            self._err.append(e)

    def write(self, data) -> None:
        n = len(data)
        self.length += n
        if self._local is not None:
            self._local.write(data)
        elif self._sink is not None:
            from ..ops.native import native_errors
            ptr, n, _, keep = _buffer_ptr(data)
            with native_errors():
                self._sink.write_ptr(ptr, n)
            del keep
        else:
            mv = memoryview(data)
            for i in range(0, n, 1 << 20):
                self._q.put(marshal.write_request_frame(mv[i:i + (1 << 20)]))

    def append_block(self, block_id: int, length: int) -> None:
        """The next ``length`` bytes of the file are block ``block_id``, which this stream's
        worker holds: the worker copies them from its store (CACHE_THROUGH tee)."""
        from ..ops.native import native_errors
        with native_errors():
            self._sink.append_block(block_id, length)
        self.length += length

    def close(self) -> None:
        if self._local is not None:
            self._local.close()
        elif self._sink is not None:
            from ..ops.native import native_errors
            sink, self._sink = self._sink, None
            with native_errors():
                sink.commit()
        else:
            self._q.close()
            self._t.join()
            if self._err:
                raise UnavailableException(f"UFS write failed: {self._err[0]}")

    def cancel(self) -> None:
        try:
            if self._local is not None:
                self._local.close()
                self._ufs.delete_file(self._path)
            elif self._sink is not None:
                sink, self._sink = self._sink, None
                sink.cancel()
            elif self._grpc is not None:
                self._grpc.cancel()
        except Exception:  # noqa: BLE001
            pass


class FileOutStream(io.RawIOBase):
    """Writes a file block by block to the chosen worker(s) and/or the UFS.

    Replicated writes (reference AlluxioBlockStore.getOutStream, AlluxioBlockStore.java:281-339,
    and BlockOutStream.createReplicatedBlockOutStream, BlockOutStream.java:109-134): the number of
    initial copies is ``replication_durable`` for ASYNC_THROUGH (when above ``replication_min``),
    else ``replication_min``.  The reference streams every byte to each replica.  Here, when the
    replicas share a node with the first (primary) worker, only the primary receives the bytes and
    the other replicas *pull* each finished block out of the primary's arena at commit — over xGMI
    between GPU workers (``PeerTransfer`` -> :func:`alluxio_amd.parallel.peer.pull_block`), all
    replicas in parallel.  Replicas on other nodes get their own gRPC block stream, as before.
    """

    # CACHE_THROUGH streams open in this process.  The UFS copy overlaps the cache copy only
    # while there are few: with more, the streams already overlap each other and the helper
    # threads only add contention (profiles/r4_worker_write_cache_through_ab.jsonl: one writer
    # 3.1 -> 4.5 GB/s with the overlap, four writers 11.9 -> 8.6).
    _ct_open = 0
    _ct_lock = threading.Lock()
    _OVERLAP_MAX_STREAMS = 2

    def __init__(self, ctx: FileSystemContext, status, write_type: str, replication_durable: int = 1,
                 write_tier: int = 0, medium: str = "", persistence_wait_ms: int = 0, replication_min: int = 0):
        super().__init__()
        self.ctx = ctx
        self.status = status
        self.path = status.path
        self.write_type = write_type
        self.block_size = status.blockSizeBytes
        self.session = ids.create_session_id()
        self.write_tier = write_tier
        self.medium = medium
        self.persistence_wait_ms = persistence_wait_ms
        self.cache = write_type in ("MUST_CACHE", "CACHE_THROUGH", "ASYNC_THROUGH", "TRY_CACHE")
        self.through = write_type in ("CACHE_THROUGH", "THROUGH")
        rmin = max(1, replication_min or 0)
        self.replicas = (replication_durable if write_type == "ASYNC_THROUGH" and replication_durable > rmin
                         else rmin)
        self._fanout: list[str] = []        # same-node replicas that pull each block from the primary
        self._primary_addr = None
        self._block_id = None
        from .policy import create_policy
        self.policy = create_policy(ctx.conf.get("alluxio.user.block.write.location.policy.class"), ctx.conf)
        self._writers: list[BlockWriter] = []
        self._block_written = 0
        self._pos = 0
        self._ufs = None
        self._beside = None          # helper thread of CACHE_THROUGH's UFS writes
        self._overlap_min = ctx.conf.get_bytes("alluxio.user.file.cache.through.overlap.min", "256KB")
        self._ct_counted = False
        self._canceled = False
        self._tee_block = False      # CACHE_THROUGH: the current block's UFS bytes come from the worker
        self._tee = ctx.conf.get_bool("alluxio.user.file.cache.through.tee.enabled", "true")
        up = status.ufsPath or ""
        self._object_store = "://" in up and not up.startswith("file://")
        # object stores: with few writers two streams win (S3 parts upload while the bytes
        # arrive), with many the tee does (the client sends each byte once); auto picks per block
        self._tee_os = str(ctx.conf.get("alluxio.user.file.cache.through.tee.object.store.enabled", "auto")).lower()
        self._tee_os_min = int(ctx.conf.get("alluxio.user.file.cache.through.tee.object.store.min.streams", "8"))
        if self._object_store and self._tee_os == "false":
            self._tee = False
        self._failed: BaseException | None = None    # a parallel block write failed: no completion
        self._workers = None
        if self.through:
            workers = ctx.workers()
            w = self.policy.get_worker(workers, 0, 0, ctx) if workers else None
            lw = ctx.in_process_worker(w.address) if w is not None else None
            if w is None:
                raise UnavailableException("no worker available for the UFS stream")
            self._ufs = UfsWriter(ctx, status, worker_address_str(w.address), lw, w.address)
            if self.cache:
                with FileOutStream._ct_lock:
                    FileOutStream._ct_open += 1
                self._ct_counted = True

    def writable(self):
        return True

    def tell(self):
        return self._pos

    def write(self, data) -> int:
        if self._failed is not None:
            raise IOError(f"output stream of {self.path} failed earlier: {self._failed}") from self._failed
        ptr, n, kind, keep = _buffer_ptr(data)
        if n == 0:
            return 0
        if self.through:
            if kind == DEVICE:
                import torch
                host = keep.detach().reshape(-1).view(torch.uint8).cpu().numpy()
            else:
                host = _host_view(ptr, n)        # zero-copy view of the caller's buffer
            if self.cache and self._tee_write(ptr, n, kind):
                self._pos += n
                return n
            if self.cache and kind != DEVICE and self._pair_write(ptr, n):
                self._pos += n
                return n
            if self.cache and n >= self._overlap_min and kind != DEVICE and \
                    FileOutStream._ct_open <= self._OVERLAP_MAX_STREAMS:
                # CACHE_THROUGH: the UFS write (a native stream or a syscall, both without the
                # GIL) runs on this stream's helper thread beside the copy into the cache tier;
                # both finish before write() returns, so the caller's buffer is not used afterwards
                if self._beside is None:
                    from concurrent.futures import ThreadPoolExecutor
                    self._beside = ThreadPoolExecutor(max_workers=1, thread_name_prefix="ufs-write")
                fut = self._beside.submit(self._ufs.write, host)
                try:
                    self._write_cache(ptr, n, kind)
                finally:
                    err = fut.exception()
                if err is not None:
                    raise err
                self._pos += n
                return n
            self._ufs.write(host)
        if self.cache:
            self._write_cache(ptr, n, kind)
        self._pos += n
        return n

    def _tee_eligible(self) -> bool:
        """The current block goes to exactly one native block stream on the worker that also runs
        this file's native UFS stream: its UFS bytes can be copied by that worker."""
        if len(self._writers) != 1:
            return False
        w = self._writers[0]
        return (isinstance(w, GrpcBlockWriter) and w._sink is not None
                and getattr(self._ufs, "_sink", None) is not None and w.address == self._ufs.worker_addr)

    def _tee_write(self, ptr: int, n: int, kind) -> bool:
        """CACHE_THROUGH with the cache block and the UFS file on one worker: the bytes travel
        once, to the block stream; when the block is committed the UFS stream is told to append it
        (``AppendBlock``) and the worker copies it from its store into the file.  Blocks that are
        not eligible (another worker, replicas, an in-process worker) take the general path."""
        if not self._tee or self.replicas != 1 or getattr(self._ufs, "_sink", None) is None:
            return False
        done = 0
        while done < n:
            if not self._writers or self._block_written >= self.block_size:
                self._next_block()
            if not self._tee_block:
                if done == 0:
                    return False             # this block takes the general path
                # (cannot happen mid-call: eligibility is fixed per block and checked at its start)
                raise IOError("CACHE_THROUGH tee changed within one write")
            take = min(n - done, self.block_size - self._block_written)
            self._writers[0].write_ptr(self._block_written, ptr + done, take, kind)
            self._block_written += take
            done += take
        return True

    def _pair_write(self, ptr: int, n: int) -> bool:
        """CACHE_THROUGH host write inside one block whose cache writer and UFS writer are both
        native gRPC streams: both get the bytes in one native call (GIL released once; the UFS
        stream's write on a pooled helper thread).  False = not that shape (the caller writes them
        the general way)."""
        us = getattr(self._ufs, "_sink", None)
        if us is None or self.replicas != 1:
            return False
        if not self._writers or self._block_written >= self.block_size:
            self._next_block()
        if n > self.block_size - self._block_written or len(self._writers) != 1:
            return False
        w = self._writers[0]
        cs = getattr(w, "_sink", None) if isinstance(w, GrpcBlockWriter) else None
        if cs is None:
            return False
        from ..ops.native import lib, native_errors
        from ..utils import optiming
        t0 = time.perf_counter() if optiming.ENABLED else 0.0
        with native_errors():
            lib().sink_write_pair(cs, us, ptr, n)
        if optiming.ENABLED:
            optiming.add("client.pair_write", time.perf_counter() - t0)
        self._ufs.length += n
        self._block_written += n
        return True

    def _write_cache(self, ptr, n, kind):
        done = 0
        while done < n:
            if (kind == HOST and n - done >= 2 * self.block_size and self.replicas == 1 and
                    (not self._writers or self._block_written >= self.block_size)):
                k = self._write_blocks_parallel(ptr + done, n - done)
                if k:
                    done += k
                    continue
            if not self._writers or self._block_written >= self.block_size:
                self._next_block()
            take = min(n - done, self.block_size - self._block_written)
            for w in self._writers:
                w.write_ptr(self._block_written, ptr + done, take, kind)
            self._block_written += take
            done += take

    def _write_blocks_parallel(self, ptr: int, n: int) -> int:
        """Whole blocks of one large host write to remote workers: up to
        ``alluxio.user.device.read.parallelism`` blocks at once, each its own WriteBlock (or
        short-circuit) stream, committed as it completes.  Block ids are taken in file order first.
        Returns the bytes written; 0 when the next block's writer is not remote (an in-process
        worker): that block is then left open as the current block, as _next_block would."""
        par = self.ctx.conf.get_int("alluxio.user.device.read.parallelism", "4")
        if par <= 1:
            return 0
        self._next_block()
        if self._fanout or not all(isinstance(w, (GrpcBlockWriter, IpcBlockWriter)) for w in self._writers):
            return 0
        opened = [self._writers]
        self._writers = []
        try:
            for _ in range(min(n // self.block_size, par) - 1):
                _, ws, _ = self._open_writers()
                opened.append(ws)
        except Exception:
            for ws in opened:
                for w in ws:
                    w.cancel()
            raise
        from concurrent.futures import ThreadPoolExecutor
        bs = self.block_size

        def fill(j):
            for w in opened[j]:
                w.write_ptr(0, ptr + j * bs, bs, HOST)

        def commit(j):
            for w in opened[j]:
                w.commit()
        # every block's bytes first, commits only once all of them landed: a failed block never
        # leaves a committed block after it, and the stream is marked failed so later writes and
        # close() raise (close cancels the file) instead of completing a file with a hole
        committed = [False] * len(opened)
        err = None
        with ThreadPoolExecutor(max_workers=len(opened), thread_name_prefix="block-write") as ex:
            errs = [f.exception() for f in [ex.submit(fill, j) for j in range(len(opened))]]
            err = next((e for e in errs if e is not None), None)
            if err is None:
                futs = [ex.submit(commit, j) for j in range(len(opened))]
                for j, f in enumerate(futs):
                    e = f.exception()
                    committed[j] = e is None
                    err = err or e
        if err is not None:
            for j, ws in enumerate(opened):
                if not committed[j]:
                    for w in ws:
                        try:
                            w.cancel()
                        except Exception:  # noqa: BLE001
                            LOG.debug("cancel of block writer failed", exc_info=True)
            self._failed = err
            raise err
        self._block_written = 0
        return len(opened) * bs

    def _next_block(self) -> None:
        from ..utils import optiming
        t0 = time.perf_counter() if optiming.ENABLED else 0.0
        self._finish_block()
        t1 = time.perf_counter() if optiming.ENABLED else 0.0
        bid, self._writers, self._fanout = self._open_writers()
        self._block_written = 0
        self._tee_block = bool(self.through and self.cache and self._tee and self._ufs is not None
                               and self.replicas == 1 and self._tee_eligible())
        if self._tee_block and self._object_store and self._tee_os == "auto":
            self._tee_block = FileOutStream._ct_open >= self._tee_os_min
        if optiming.ENABLED:
            optiming.add("client.finish_block", t1 - t0)
            optiming.add("client.open_writers", time.perf_counter() - t1)

    def _open_writers(self):
        """Allocates the file's next block id and opens its writer(s): (id, writers, same-node
        replicas that pull the block from the primary)."""
        writers = []
        bid = self.ctx.fs_master().GetNewBlockIdForFile(pb.file.GetNewBlockIdForFilePRequest(path=self.path)).id
        workers = self._workers if self._workers is not None else self.ctx.workers(refresh=self._workers is None)
        self._workers = workers
        chosen = []
        cands = list(workers)
        for _ in range(self.replicas):
            w = self.policy.get_worker(cands, bid, self.block_size, self.ctx)
            if w is None:
                break
            chosen.append(w)
            cands = [c for c in cands if worker_address_str(c.address) != worker_address_str(w.address)]
        if not chosen:
            raise UnavailableException("no worker available to write the block")
        if self.replicas > 1 and len(chosen) < self.replicas:
            raise ResourceExhaustedException(f"Not enough workers for replications, {len(chosen)} workers "
                                             f"selected but {self.replicas} required")
        reserve = min(self.block_size, self.ctx.conf.get_bytes("alluxio.user.file.buffer.bytes", "8MB"))
        fanout = []
        self._primary_addr = worker_address_str(chosen[0].address)
        self._block_id = bid
        if len(chosen) > 1 and self.ctx.conf.get_bool("alluxio.user.block.replication.peer.pull.enabled", "true"):
            prim_host = chosen[0].address.host
            pullers = [w for w in chosen[1:] if w.address.host == prim_host and self.ctx.is_local(w.address)]
            fanout = [worker_address_str(w.address) for w in pullers]
            chosen = [chosen[0]] + [w for w in chosen[1:] if w not in pullers]
        # ASYNC_THROUGH with the UFS tier: a worker out of space spills the block to a UFS block
        # file instead of failing the write (alluxio.user.file.ufs.tier.enabled)
        ufs_tier = self.write_type == "ASYNC_THROUGH" and \
            self.ctx.conf.get_bool("alluxio.user.file.ufs.tier.enabled", "false")
        for w in chosen:
            lw = self.ctx.in_process_worker(w.address)
            if lw is not None and ufs_tier:
                writers.append(LocalUfsFallbackWriter(lw, bid, self.session, self.status.mountId,
                                                            self.write_tier, self.medium, max(1, reserve)))
            elif lw is not None:
                writers.append(LocalBlockWriter(lw, bid, self.session, self.write_tier, self.medium,
                                                      max(1, reserve)))
            elif self._ipc_write(w) and not ufs_tier:
                addr = worker_address_str(w.address)
                try:
                    writers.append(IpcBlockWriter(self.ctx, addr, bid, self.block_size, self.write_tier,
                                                        self.medium))
                except Exception:  # noqa: BLE001 - no shared arena (file tier, no GPU): the data port
                    LOG.debug("short-circuit write to %s unavailable", addr, exc_info=True)
                    writers.append(GrpcBlockWriter(self.ctx, addr, bid, self.write_tier, self.medium, reserve,
                                                         data_address=(w.address.host,
                                                                       w.address.dataPort or w.address.rpcPort)))
            else:
                writers.append(GrpcBlockWriter(self.ctx, worker_address_str(w.address), bid,
                                                     self.write_tier, self.medium, reserve,
                                                     ufs_fallback_mount=self.status.mountId if ufs_tier else None,
                                                     data_address=(w.address.host,
                                                                   w.address.dataPort or w.address.rpcPort)))
        return bid, writers, fanout

    def _ipc_write(self, w) -> bool:
        """Short-circuit (shared-arena) writes to a same-node worker in another process."""
        conf = self.ctx.conf
        return conf.get_bool("alluxio.user.short.circuit.enabled", "true") and \
            conf.get_bool("alluxio.user.short.circuit.write.enabled", "true") and \
            conf.get_bool("alluxio.worker.ipc.enabled", "true") and self.ctx.is_local(w.address)

    def _finish_block(self) -> None:
        hold = bool(self._writers) and self._tee_block and self._block_written > 0
        for w in self._writers:
            w.commit(hold) if hold else w.commit()
        had = bool(self._writers)
        if had and self._tee_block and self._block_written:
            # committed on the worker that runs the UFS stream: it appends the block to the file
            self._ufs.append_block(self._block_id, self._block_written)
        self._tee_block = False
        self._writers = []
        if had and self._fanout:
            # replicas pull the committed block while this stream writes the next one (the pulls
            # are peer DMAs plus a few RPCs each: serialising them behind every block doubled the
            # time of a replicated write); close() waits for all of them and raises their errors
            from ..parallel.peer import fan_out
            import concurrent.futures as cf
            if getattr(self, "_fan_exec", None) is None:
                self._fan_exec = cf.ThreadPoolExecutor(2, thread_name_prefix="replica-fanout")
                self._fan_futs = []
            bid = self._block_id
            self._fan_futs.append((bid, self._fan_exec.submit(
                fan_out, self._primary_addr, list(self._fanout), bid, self._block_written, self.ctx.worker_stub)))
            self._fanout = []

    def _wait_fanouts(self) -> None:
        futs = getattr(self, "_fan_futs", None) or []
        self._fan_futs = []
        errors = []
        t0 = time.perf_counter()
        for bid, f in futs:
            try:
                e = f.result()
            except Exception as ex_:  # noqa: BLE001
                e = [("?", str(ex_))]
            if e:
                errors.append((bid, e))
        if futs:
            # how long close() waited for replica pulls still running after the last block
            from ..parallel.peer import _add_time
            _add_time("fan_close_wait", time.perf_counter() - t0)
        ex = getattr(self, "_fan_exec", None)
        if ex is not None:
            ex.shutdown(wait=False)
            self._fan_exec = None
        if errors:
            raise UnavailableException(f"replicating blocks failed: {errors}")

    def _stop_beside(self) -> None:
        if self._beside is not None:
            self._beside.shutdown(wait=False)
            self._beside = None
        if self._ct_counted:
            self._ct_counted = False
            with FileOutStream._ct_lock:
                FileOutStream._ct_open -= 1

    def cancel(self) -> None:
        self._canceled = True
        self._stop_beside()
        try:
            self._wait_fanouts()        # no replica pull of this file is left running
        except Exception:  # noqa: BLE001
            pass
        for w in self._writers:
            w.cancel()
        self._writers = []
        if self._ufs is not None:
            self._ufs.cancel()
        try:
            self.ctx.fs_master().Remove(pb.file.DeletePRequest(path=self.path, options=pb.file.DeletePOptions(
                alluxioOnly=True, unchecked=True)))
        except Exception:  # noqa: BLE001
            pass
        super().close()

    def close(self) -> None:
        if self.closed:
            return
        if self._canceled:
            return
        if self._failed is not None:
            err = self._failed
            self.cancel()
            raise IOError(f"output stream of {self.path} failed; the file was cancelled: {err}") from err
        self._stop_beside()
        from ..utils import optiming
        ufs_closed = False
        try:
            t0 = time.perf_counter() if optiming.ENABLED else 0.0
            self._finish_block()
            self._wait_fanouts()
            t1 = time.perf_counter() if optiming.ENABLED else 0.0
            opts = pb.file.CompleteFilePOptions()
            if self._ufs is not None:
                self._ufs.close()
                ufs_closed = True
                opts.ufsLength = self._ufs.length
            t2 = time.perf_counter() if optiming.ENABLED else 0.0
            if self.write_type == "ASYNC_THROUGH":
                opts.asyncPersistOptions.persistenceWaitTime = self.persistence_wait_ms
            self.ctx.fs_master().CompleteFile(pb.file.CompleteFilePRequest(path=self.path, options=opts))
            if optiming.ENABLED:
                optiming.add("client.close.finish_block", t1 - t0)
                optiming.add("client.close.ufs_commit", t2 - t1)
                optiming.add("client.close.complete_file", time.perf_counter() - t2)
        except Exception:
            for w in self._writers:
                try:
                    w.cancel()
                except Exception:  # noqa: BLE001 - keep the original error
                    pass
            if self._ufs is not None and not ufs_closed:
                self._ufs.cancel()      # e.g. an object-store upload is aborted now, not at GC
            raise
        finally:
            super().close()
        self.ctx.metrics.counter("BytesWrittenClient").inc(self._pos)


__all__ = ["FileInStream", "FileOutStream", "LocalBlockReader", "GrpcBlockReader", "LocalBlockWriter",
           "GrpcBlockWriter", "HOST", "DEVICE", "random", "enum_name"]
