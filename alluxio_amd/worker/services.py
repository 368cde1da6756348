"""gRPC ``BlockWorker`` service of a worker (the data server).

Parity: core/server/worker/src/main/java/alluxio/worker/grpc/BlockWorkerImpl.java:61-210,
AbstractReadHandler.java (chunked streaming, flow control: pause while more than the window is
un-acked by ``offset_received`` — :74-77, :113-140, :170-172, :336-439), BlockReadHandler.java
(openBlock: lock -> reader, UFS fallback :159-235), AbstractWriteHandler / BlockWriteHandler
(:36-149: reserve, append, flush acks, commit on close), UfsFileWriteHandler (CACHE_THROUGH's UFS
stream), ShortCircuitBlock{Read,Write}Handler (lock/create local block for the stream lifetime).

MI355X extension RPCs: ``OpenDeviceBlock`` hands out the block's page list plus a HIP IPC handle
of the HBM arena so a same-node process can gather the bytes with its own kernel (the device
analogue of short-circuit mmap); ``UnlockDeviceBlock`` releases it.
"""
from __future__ import annotations

import logging
import os
import threading
import time

from ..ops.native import native_errors
from ..proto import enum_name, pb
from ..rpc import marshal
from ..utils import ids
from ..utils.exceptions import (BlockDoesNotExistException, InvalidArgumentException,
                                UnavailableException)

LOG = logging.getLogger(__name__)
_SLOW_READ_LOG = None   # SamplingLogger: one slow-read warning per 5 minutes (BlockReadHandler.java:63)

SVC_BLOCK_WORKER = "alluxio.grpc.block.BlockWorker"


class BlockWorkerService:
    def __init__(self, worker, conf):
        self.w = worker
        self.conf = conf
        self.max_chunk = conf.get_bytes("alluxio.worker.network.reader.max.chunk.size.bytes")
        self.window = conf.get_bytes("alluxio.worker.network.reader.buffer.size")
        self.slow_read_s = conf.get_ms("alluxio.worker.remote.io.slow.threshold") / 1000.0
        global _SLOW_READ_LOG
        if _SLOW_READ_LOG is None:
            from ..utils.pause_monitor import SamplingLogger
            _SLOW_READ_LOG = SamplingLogger(LOG, 300.0)
        self._device_locks: dict[int, tuple[int, int]] = {}
        self._lock = threading.Lock()

    # ------------------------------------------------------------------------------------------
    def ReadBlock(self, request_iter, ctx):
        it = iter(request_iter)
        first = next(it, None)
        if first is None:
            return
        session = ids.create_session_id()
        acked = [first.offset]
        done = threading.Event()
        cond = threading.Condition()

        def ack_reader():
            try:
                for r in it:
                    if r.HasField("offset_received"):
                        with cond:
                            acked[0] = max(acked[0], r.offset_received)
                            cond.notify_all()
            except Exception:  # noqa: BLE001
                pass
            finally:
                done.set()
                with cond:
                    cond.notify_all()
        t = threading.Thread(target=ack_reader, daemon=True, name="read-acks")
        t.start()
        chunk = min(first.chunk_size or (1 << 20), self.max_chunk)
        lock_id = None
        try:
            bid = first.block_id
            if not self.w.has_block(bid):
                if first.HasField("open_ufs_block_options") and (first.open_ufs_block_options.ufs_path or
                                                                 first.open_ufs_block_options.block_in_ufs_tier):
                    from .ufs_fallback import resolve_ufs_block_opts
                    opts = resolve_ufs_block_opts(self.w, bid, first.open_ufs_block_options)
                    if not first.open_ufs_block_options.block_in_ufs_tier:
                        # the native data server reads later cold blocks of this mount itself
                        self.w.note_ufs_mount(opts.mountId, self.w._ufs_for(opts))
                    if opts.no_cache or first.offset != 0 or self.w.native.has_temp_block(bid):
                        # partial / uncached reads (or another reader is caching it): plain stream
                        yield from self._stream_ufs(opts, first.offset, first.length, chunk, acked, cond, done)
                        return
                    # read-through: stream each UFS chunk to the client as it is cached
                    # (UnderFileSystemBlockReader.java:205-243)
                    yield from self._stream_ufs_caching(bid, opts, first.length, chunk, acked, cond, done,
                                                        session)
                    return
                else:
                    raise BlockDoesNotExistException(f"Block {bid} does not exist on this worker")
            if first.promote:
                # before the read lock (a locked block does not move): BlockReadHandler.openBlock
                try:
                    self.w.move_block(session, bid, tier=0)
                except Exception:  # noqa: BLE001
                    pass
            lock_id = self.w.lock_block(session, bid)
            info = self.w.block_info(bid)
            length = first.length if first.length > 0 else info.length - first.offset
            end = min(info.length, first.offset + length)
            pos = first.offset
            self.w.access_block(session, bid)
            # BytesReadDomain vs BytesReadRemote (DefaultBlockWorker metrics by transport)
            peer = ctx.peer() if hasattr(ctx, "peer") else ""
            read_counter = self.w.metrics.counter(
                "BytesReadDomain" if str(peer).startswith("unix:") else "BytesReadRemote")
            while pos < end:
                with cond:
                    while pos - acked[0] >= self.window and not done.is_set():
                        cond.wait(0.5)
                n = min(chunk, end - pos)
                t_buf = time.monotonic()
                frame = self.w.read_frame(bid, pos, n)      # header + bytes, sent as-is
                took = time.monotonic() - t_buf
                if took >= self.slow_read_s:                # BlockReadHandler.java:136-150
                    _SLOW_READ_LOG.warning("Getting buffer for remote read took longer than %d ms. "
                                           "block=%d offset=%d length=%d took=%d ms", int(self.slow_read_s * 1000),
                                           bid, pos, n, int(took * 1000), key="slow-read")
                pos += n
                read_counter.inc(n)
                yield frame
        finally:
            if lock_id is not None:
                try:
                    self.w.unlock(lock_id)
                except Exception:  # noqa: BLE001
                    pass
            self.w.cleanup_session(session)

    def _stream_ufs_caching(self, bid, opts, length, chunk, acked, cond, done, session):
        """Cache the block from the UFS on a background thread (K3 pipeline) and stream every
        ingested chunk to the client as it lands, respecting the flow-control window; bytes past
        the requested length are cached but not sent."""
        import queue
        end = length if length > 0 else opts.block_size
        q: queue.Queue = queue.Queue(maxsize=8)
        err: list = []

        def on_chunk(mv):
            q.put(bytes(mv))            # copy out of the staging buffer before it is reused

        def run():
            try:
                self.w.cache_block_from_ufs(bid, opts, session, on_chunk=on_chunk)
            except Exception as e:  # noqa: BLE001
                err.append(e)
            finally:
                q.put(None)
        t = threading.Thread(target=run, daemon=True, name=f"ufs-read-through-{bid}")
        t.start()
        pos = 0
        while True:
            data = q.get()
            if data is None:
                break
            if pos >= end:
                continue               # keep draining: the rest of the block is still cached
            with cond:
                while pos - acked[0] >= self.window and not done.is_set():
                    cond.wait(0.5)
            n = min(len(data), end - pos)
            mv = memoryview(data)               # frames join header + slice: one copy, not two
            for off in range(0, n, chunk):
                yield marshal.read_response_frame(mv[off:min(n, off + chunk)])
            pos += n
        t.join()
        if err and pos < end:
            raise err[0]
        self.w.metrics.counter("BytesReadUfsThrough").inc(pos)

    def _stream_ufs(self, opts, offset, length, chunk, acked, cond, done):
        end = offset + (length if length > 0 else opts.block_size - offset)
        pos = offset
        while pos < end:
            with cond:
                while pos - acked[0] >= self.window and not done.is_set():
                    cond.wait(0.5)
            n = min(chunk, end - pos)
            data = self.w.read_ufs_range(opts, pos, n)
            if not data:
                break
            pos += len(data)
            yield marshal.read_response_frame(data)

    # ------------------------------------------------------------------------------------------
    def NativeWriteCommit(self, req, ctx):
        """Commit of a WriteBlock whose chunks the native data server wrote (csrc/data_server.cpp
        BlockWriteStream): CRC32C and the master's CommitBlock, as WriteBlock's end does.  Only the
        server itself posts it; a client calling it is refused."""
        if not getattr(ctx, "internal", False):
            from ..utils.exceptions import PermissionDeniedException
            raise PermissionDeniedException("NativeWriteCommit is internal to the worker's data server")
        if not req.ufs_read:
            self.w.commit_block(req.session_id, req.block_id, req.pin, req.hold_for_append)
            return pb.block.WriteResponse(offset=req.length)
        # a cold ReadBlock the native server read through from the UFS: posted by its reader once
        # the whole block is in the store (the call itself may be gone); the session is ours now
        try:
            self.w.commit_block(req.session_id, req.block_id, req.pin)
            self.w.metrics.counter("BytesReadUfsAll").inc(req.length)
            self.w.metrics.counter("BytesReadUfsThrough").inc(req.length)
        finally:
            self.w.cleanup_session(req.session_id)    # aborts the temp block if the commit failed
        return pb.block.WriteResponse(offset=req.length)

    def NativeCommitBatch(self, req, ctx):
        """The master report of the blocks the native committer (csrc/data_server.cpp
        BlockCommitter) committed since its last report: their streamed CRCs are kept and ONE
        CommitBlocks call tells the master about all of them (retried for
        alluxio.user.rpc.retry.max.duration).  A failure fails every block of the batch: the
        committer removes them again and fails their streams.  Internal to the data server."""
        if not getattr(ctx, "internal", False):
            from ..utils.exceptions import PermissionDeniedException
            raise PermissionDeniedException("NativeCommitBatch is internal to the worker's data server")
        import numpy as np
        ids = list(req.block_id)
        crcs = {}
        for bid, piece, c in zip(ids, req.crc_piece, req.crc):
            if piece and c:
                crcs[bid] = (int(piece), np.frombuffer(c, dtype="<u4").tolist())
        self.w.report_native_commits(ids, crcs)
        ufs = [n for n, u in zip(req.length, req.ufs_read) if u]
        if ufs:
            self.w.metrics.counter("BytesReadUfsAll").inc(sum(ufs))
            self.w.metrics.counter("BytesReadUfsThrough").inc(sum(ufs))
        return pb.block.NativeCommitBatchResponse()

    def ResolveUfsMount(self, req, ctx):
        """A cold read of a mount the native data server has not seen: resolve its UFS the way the
        reference worker does on demand (WorkerUfsManager.java:56-65 asks the master's GetUfsInfo)
        and register it with the data server when its I/O threads can reach it (note_ufs_mount).
        Internal to the data server; the cold read then runs natively."""
        if not getattr(ctx, "internal", False):
            from ..utils.exceptions import PermissionDeniedException
            raise PermissionDeniedException("ResolveUfsMount is internal to the worker's data server")
        opts = pb.dataserver.OpenUfsBlockOptions(ufs_path=req.ufs_path, mountId=req.mount_id)
        self.w.note_ufs_mount(req.mount_id, self.w._ufs_for(opts))
        roots = self.w.native_ufs_roots
        native = roots is not None and (roots.resolve(req.mount_id, req.ufs_path) is not None or
                                        roots.resolve_s3(req.mount_id, req.ufs_path) is not None)
        self.w.metrics.counter("UfsMountsResolvedNatively").inc()
        return pb.block.ResolveUfsMountResponse(native=native)

    def ReadUfsRange(self, req, ctx):
        """Bytes of a UFS file the data server's threads cannot read themselves (the first cold read
        of a mount that resolved to a Python-only UFS).  Internal to the data server."""
        if not getattr(ctx, "internal", False):
            from ..utils.exceptions import PermissionDeniedException
            raise PermissionDeniedException("ReadUfsRange is internal to the worker's data server")
        opts = pb.dataserver.OpenUfsBlockOptions(ufs_path=req.ufs_path, mountId=req.mount_id, offset_in_file=0,
                                                 block_size=req.offset + req.length)
        return pb.block.ReadUfsRangeResponse(data=self.w.read_ufs_range(opts, req.offset, req.length))

    def WriteBlock(self, request_iter, ctx):
        it = iter(request_iter)
        first = next(it, None)
        if first is None or not first.HasField("command"):
            raise InvalidArgumentException("WriteBlock stream must start with a command")
        cmd = first.command
        rtype = enum_name(pb.block.RequestType, cmd.type)
        session = ids.create_session_id()
        pos = cmd.offset
        if rtype == "UFS_FILE":
            yield from self._write_ufs_file(cmd, it)
            return
        if rtype == "UFS_FALLBACK_BLOCK":
            yield from self._write_ufs_fallback(cmd, it, session)
            return
        bid = cmd.id
        tier = cmd.tier if cmd.HasField("tier") else 0
        medium = cmd.medium_type
        reserve = cmd.space_to_reserve or self.conf.get_bytes("alluxio.worker.file.buffer.size", "1MB")
        self.w.create_block(session, bid, tier if not medium else -1, medium, reserve, cmd.pin_on_create)
        committed = False
        hold = cmd.hold_for_append
        try:
            for req in it:
                if req.HasField("chunk"):
                    data = req.chunk.data
                    self.w.write_bytes(session, bid, pos, data)
                    pos += len(data)
                elif req.HasField("command"):
                    hold = hold or req.command.hold_for_append
                    if req.command.flush:
                        yield pb.block.WriteResponse(offset=pos)
            self.w.commit_block(session, bid, cmd.pin_on_create, hold)
            committed = True
            yield pb.block.WriteResponse(offset=pos)
        finally:
            if not committed:
                try:
                    self.w.abort_block(session, bid)
                except Exception:  # noqa: BLE001
                    pass
            self.w.cleanup_session(session)

    def _write_ufs_fallback(self, cmd, it, session):
        """UfsFallbackBlockWriteHandler: local block, spilling to a UFS block file when the worker
        runs out of space (worker/ufs_fallback.py)."""
        from .ufs_fallback import UfsFallbackBlockWriter
        o = cmd.create_ufs_block_options
        if o.fallback and o.bytes_in_block_store:
            raise InvalidArgumentException("short-circuit UFS fallback with bytes already in the block store is "
                                           "not supported; write the block through this stream from offset 0")
        reserve = cmd.space_to_reserve or self.conf.get_bytes("alluxio.worker.file.buffer.size", "1MB")
        w = UfsFallbackBlockWriter(self.w, session, cmd.id, o.mount_id, cmd.tier if cmd.HasField("tier") else 0,
                                   cmd.medium_type, reserve, local=not o.fallback, pin=cmd.pin_on_create)
        done = False
        try:
            for req in it:
                if req.HasField("chunk"):
                    w.write(req.chunk.data)
                elif req.HasField("command") and req.command.flush:
                    yield pb.block.WriteResponse(offset=w.pos)
            w.commit()
            done = True
            yield pb.block.WriteResponse(offset=w.pos)
        finally:
            if not done:
                w.cancel()
            self.w.cleanup_session(session)

    def _write_ufs_file(self, cmd, it):
        from ..underfs.base import CreateOptions
        o = cmd.create_ufs_file_options
        ufs = self.w._ufs_for(pb.dataserver.OpenUfsBlockOptions(ufs_path=o.ufs_path, mountId=o.mount_id))
        pos = 0
        out = ufs.create(o.ufs_path, CreateOptions(create_parent=True, ensure_atomic=True, owner=o.owner,
                                                   group=o.group, mode=o.mode or 0o644))
        ok = False
        try:
            for req in it:
                if req.HasField("chunk"):
                    out.write(req.chunk.data)
                    pos += len(req.chunk.data)
                elif req.HasField("append_block"):
                    # CACHE_THROUGH tee: the next bytes are a block this worker holds
                    pos += self._append_block(out, req.append_block.block_id, req.append_block.length)
                elif req.HasField("command") and req.command.flush:
                    yield pb.block.WriteResponse(offset=pos)
            ok = True
        finally:
            if ok:
                out.close()
            else:
                try:
                    cancel = getattr(out, "cancel", None)
                    if cancel is not None:        # object stores: abort the upload, write nothing
                        cancel()
                    else:
                        out.close()
                        ufs.delete_file(o.ufs_path)
                except Exception:  # noqa: BLE001
                    pass
        self.w.metrics.counter("BytesWrittenUfsAll").inc(pos)
        self.w.note_ufs_mount(o.mount_id, ufs)
        yield pb.block.WriteResponse(offset=pos)

    def _append_block(self, out, block_id: int, length: int) -> int:
        """Copy [0, length) of a block this worker holds into a UFS output stream (read-locked,
        8 MiB at a time through a host buffer)."""
        import numpy as np
        session = ids.create_session_id()
        lock_id = self.w.lock_block(session, block_id)
        self.w.native.release_hold(block_id)      # the commit's append hold: our lock keeps it now
        try:
            buf = np.empty(min(length, 8 << 20), dtype=np.uint8)
            off = 0
            while off < length:
                k = min(len(buf), length - off)
                self.w.native.read(block_id, off, k, buf.ctypes.data, 0)
                out.write(memoryview(buf)[:k])
                off += k
        finally:
            self.w.unlock(lock_id)
        return length

    # ------------------------------------------------------------------------------------------
    def OpenLocalBlock(self, request_iter, ctx):
        it = iter(request_iter)
        first = next(it, None)
        if first is None:
            return
        session = ids.create_session_id()
        lock_id = self.w.lock_block(session, first.block_id)
        try:
            info = self.w.block_info(first.block_id)
            path = ""
            spec = self.w.native.dir_spec(info.dir)
            if spec.path:
                path = os.path.join(spec.path, str(first.block_id))
            yield pb.block.OpenLocalBlockResponse(path=path)
            for _ in it:  # hold the lock until the client closes the stream
                pass
        finally:
            self.w.unlock(lock_id)
            self.w.cleanup_session(session)

    def CreateLocalBlock(self, request_iter, ctx):
        it = iter(request_iter)
        first = next(it, None)
        if first is None:
            return
        session = ids.create_session_id()
        self.w.create_block(session, first.block_id, first.tier, first.medium_type,
                            first.space_to_reserve or (1 << 20), first.pin_on_create)
        ok = False
        try:
            yield pb.block.CreateLocalBlockResponse(path="")
            for req in it:
                if req.space_to_reserve:
                    self.w.request_space(session, first.block_id, req.space_to_reserve)
                    yield pb.block.CreateLocalBlockResponse(path="")
            if not first.only_reserve_space:
                self.w.commit_block(session, first.block_id, first.pin_on_create)
            ok = True
        finally:
            if not ok and first.cleanup_on_failure:
                try:
                    self.w.abort_block(session, first.block_id)
                except Exception:  # noqa: BLE001
                    pass

    def AsyncCache(self, req, ctx):
        src = None
        if req.source_host and (req.source_host, req.source_port) != (self.w.address.host, self.w.address.rpcPort):
            src = self.w.peer_fetcher(req.source_host, req.source_port, req.length)
        opts = req.open_ufs_block_options if req.HasField("open_ufs_block_options") else None
        if opts is not None and not opts.block_size and req.length:
            opts.block_size = req.length
        self.w.async_cache(req.block_id, opts=opts, source=src, length=req.length)
        return pb.block.AsyncCacheResponse()

    def RemoveBlock(self, req, ctx):
        self.w.remove_block(ids.create_session_id(), req.block_id)
        return pb.block.RemoveBlockResponse()

    def MoveBlock(self, req, ctx):
        self.w.move_block(ids.create_session_id(), req.block_id, medium=req.medium_type)
        return pb.block.MoveBlockResponse()

    def ClearMetrics(self, req, ctx):
        self.w.metrics.registry.clear()
        return pb.block.ClearMetricsResponse()

    # ---- MI355X extensions ---------------------------------------------------------------------
    def OpenDeviceBlock(self, req, ctx):
        """Read-lock a block and describe where its pages live for a same-node reader: HBM arenas
        are exported as a HIP IPC handle, shared DRAM arenas as (pid, memfd).  The reader maps the
        arena once and copies the pages itself (``parallel.ipc.map_handle``)."""
        session = req.session_id or ids.create_session_id()
        lock_id = self.w.lock_block(session, req.block_id)
        try:
            pages, d, ps, base = self.w.native.block_pages(req.block_id)
            info = self.w.block_info(req.block_id)
            arena = self.w.store.arena_for_dir(d)
            if arena is None:
                raise UnavailableException("block is in a file tier: no shared memory view")
            h = pb.block.DeviceBlockHandle(block_id=req.block_id, length=info.length, page_size=ps, pages=pages,
                                           arena_bytes=arena.nbytes, device=arena.device, lock_id=lock_id,
                                           pid=os.getpid(), arena_kind=arena.kind, host_fd=-1)
            if arena.kind == "hbm":
                try:
                    h.arena_ipc_handle, h.arena_offset = arena.ipc_handle()
                except Exception:  # noqa: BLE001
                    LOG.debug("IPC export unavailable", exc_info=True)
            else:
                share = arena.share_handle()
                if share is None:
                    raise UnavailableException("DRAM arena is not shareable")
                h.host_fd = share[1]
            piece, crcs = self.w.crc.get(req.block_id, (0, None))
            if crcs and piece == ps:     # CRCs are per page of the handle's page size
                h.crc32c.extend(crcs)
            with self._lock:
                self._device_locks[lock_id] = (session, req.block_id)
            self.w.access_block(session, req.block_id)
            # reader_gpu = reading device + 1: a reader on another GPU pulls these bytes over xGMI
            if arena.kind == "hbm" and req.reader_gpu and req.reader_gpu - 1 != arena.device:
                self.w.metrics.counter("XgmiBytesSent").inc(info.length)
            return h
        except Exception:
            self.w.unlock(lock_id)
            raise

    def OpenDeviceWrite(self, req, ctx):
        """Short-circuit write for a same-node writer process (the analogue of CreateLocalBlock,
        whose writer fills a temp block file): create the temp block with ``length`` bytes of
        pages reserved and describe them like :meth:`OpenDeviceBlock`; the writer maps the arena
        and copies into the pages itself, then calls :meth:`CommitDeviceWrite`.  The client renews
        the session while the write is open (:meth:`SessionHeartbeat`); an abandoned write is
        reclaimed with its session (``alluxio.worker.session.timeout``)."""
        session = req.session_id or ids.create_session_id()
        length = max(int(req.length), 1)
        self.w.create_block(session, req.block_id, req.tier if not req.medium_type else -1, req.medium_type,
                            length, req.pin_on_create)
        try:
            pages, d, ps, _base = self.w.native.block_pages(req.block_id)
            arena = self.w.store.arena_for_dir(d)
            if arena is None:
                raise UnavailableException("block is in a file tier: no shared memory view")
            h = pb.block.DeviceBlockHandle(block_id=req.block_id, length=length, page_size=ps, pages=pages,
                                           arena_bytes=arena.nbytes, device=arena.device, lock_id=session,
                                           pid=os.getpid(), arena_kind=arena.kind, host_fd=-1)
            if arena.kind == "hbm":
                h.arena_ipc_handle, h.arena_offset = arena.ipc_handle()
            else:
                share = arena.share_handle()
                if share is None:
                    raise UnavailableException("DRAM arena is not shareable")
                h.host_fd = share[1]
            return h
        except Exception:
            self.w.abort_block(session, req.block_id)
            self.w.cleanup_session(session)
            raise

    def CommitDeviceWrite(self, req, ctx):
        """End of a short-circuit write: record the written length and commit (CRC, master
        report), or abort."""
        try:
            if req.abort:
                self.w.abort_block(req.session_id, req.block_id)
            else:
                with native_errors():
                    self.w.native.external_write(req.session_id, req.block_id, 0, req.length)
                self.w.commit_block(req.session_id, req.block_id, req.pin_on_create, req.hold_for_append)
                self.w.metrics.counter("BytesWrittenAlluxio").inc(req.length)
                self.w.metrics.counter("BytesWrittenDomain").inc(req.length)
        finally:
            self.w.cleanup_session(req.session_id)
        return pb.block.CommitDeviceWriteResponse()

    def SessionHeartbeat(self, req, ctx):
        """Keeps the sessions of open short-circuit handles alive (client/session_keeper.py): an
        IPC-mapped write or read outlives any one RPC, so without renewals the session cleaner
        would reclaim its pages under the client after ``alluxio.worker.session.timeout``."""
        return pb.block.SessionHeartbeatResponse(unknown_session_ids=self.w.renew_sessions(list(req.session_ids)))

    def UnlockDeviceBlock(self, req, ctx):
        with self._lock:
            self._device_locks.pop(req.lock_id, None)
        self.w.unlock(req.lock_id)
        return pb.block.UnlockDeviceBlockResponse()

    def PeerTransfer(self, req, ctx):
        from .remote import peer_transfer
        ok, msg = peer_transfer(self.w, req)
        return pb.block.PeerTransferResponse(ok=ok, message=msg)
