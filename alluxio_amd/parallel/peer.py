"""Worker-to-worker block pulls on one node, with failure handling.

Reference: a worker caches a block held by another worker by streaming it through the peer's
``ReadBlock`` gRPC service (core/server/worker/src/main/java/alluxio/worker/block/RemoteBlockReader.java,
AsyncCacheRequestManager.java:213-240); replicated writes stream the bytes to every replica
(core/client/fs/src/main/java/alluxio/client/block/stream/BlockOutStream.java:109-134).

Here the destination worker *pulls* the block straight out of the source worker's memory:

1. ``OpenDeviceBlock`` on the source read-locks the block and returns its page list plus a way to
   map the arena — a HIP IPC handle for HBM, ``(pid, memfd)`` for a shared DRAM arena;
2. the destination reserves its own pages (``BlockStore.external_write``) and runs the batched
   copy kernel on ITS GPU, reading the peer's HBM over xGMI (or host memory; memcpy on CPU builds);
3. commit, then ``UnlockDeviceBlock``.

No payload crosses the RPC channel.  Failures are handled the way SURVEY §5.3 asks for the GPU
plane: every control RPC has a deadline, a peer whose mapped pull failed is marked for a cooldown
(``alluxio.worker.peer.failure.cooldown``) during which its blocks come through the gRPC block
stream instead, and an aborted pull always releases both the destination's temp block and the
source's read lock.
"""
from __future__ import annotations

import logging
import os
import threading
import time

from ..proto import pb
from ..utils import ids

LOG = logging.getLogger(__name__)

_fail_lock = threading.Lock()
_failed_until: dict[tuple[int, str], float] = {}   # (worker id, peer address) -> monotonic deadline

# Wall time of the steps of the mapped pulls of this process (seconds, and pulls): the replica
# fan-out breakdown bench.py's replicate phase reports (profiles/r6_replica_fanout.md).
_times_lock = threading.Lock()
PULL_TIMES: dict[str, float] = {}


def _add_time(step: str, dt: float) -> None:
    with _times_lock:
        PULL_TIMES[step] = PULL_TIMES.get(step, 0.0) + dt


def pull_times() -> dict[str, float]:
    with _times_lock:
        return dict(PULL_TIMES)


def _cooldown_s(worker) -> float:
    return worker.conf.get_ms("alluxio.worker.peer.failure.cooldown", "30sec") / 1000.0


def _rpc_timeout_s(worker) -> float:
    return worker.conf.get_ms("alluxio.worker.peer.rpc.timeout", "30sec") / 1000.0


def mark_failed(worker, addr: str) -> None:
    with _fail_lock:
        _failed_until[(id(worker), addr)] = time.monotonic() + _cooldown_s(worker)
    worker.metrics.counter("PeerPullFailures").inc()


def peer_failed(worker, addr: str) -> bool:
    with _fail_lock:
        t = _failed_until.get((id(worker), addr))
        if t is None:
            return False
        if time.monotonic() >= t:
            del _failed_until[(id(worker), addr)]
            return False
        return True


def clear_failures(worker=None) -> None:
    with _fail_lock:
        if worker is None:
            _failed_until.clear()
        else:
            for k in [k for k in _failed_until if k[0] == id(worker)]:
                del _failed_until[k]


def _my_gpu(worker) -> int:
    """This worker's device index + 1 (0 = no GPU): the ``reader_gpu`` of OpenDeviceBlock."""
    from ..ops.native import has_gpu
    return (int(worker.store.device) + 1) if has_gpu() else 0


def mapped_pull(worker, block_id: int, addr: str, tier: int = 0, medium: str = "", handle=None) -> int:
    """Pull ``block_id`` from same-node worker ``addr`` by mapping its arena; returns bytes.
    ``handle``: the source's DeviceBlockHandle, opened (read-locked) once by the writer for all
    replicas (fan_out) -- then this pull neither opens nor unlocks it."""
    from ..ops.native import has_gpu, lib
    from .ipc import map_handle
    from .transfer import cross_page_segments
    if worker.conf.get_bool("alluxio.test.peer.mapped.pull.fail", "false"):
        raise RuntimeError("mapped pull failure injected (alluxio.test.peer.mapped.pull.fail)")
    clock = time.perf_counter
    t0 = clock()
    session = ids.create_session_id()
    timeout = _rpc_timeout_s(worker)
    stub = None
    if handle is not None:
        h = handle
    else:
        stub = worker.peer_stub(addr)
        h = stub.OpenDeviceBlock(pb.block.OpenDeviceBlockRequest(block_id=block_id, session_id=session,
                                                                 reader_gpu=_my_gpu(worker)), timeout=timeout)
    t1 = clock()
    _add_time("open_rpc", t1 - t0)
    try:
        n = h.length
        dev = int(worker.store.device)
        src_base = map_handle(h, dev)
        t2 = clock()
        _add_time("map", t2 - t1)
        worker.create_block(session, block_id, tier, medium, max(n, 1))
        try:
            dst_pages = worker.native.external_write(session, block_id, 0, n)
            _p, _d, dps, dbase = worker.native.block_pages(block_id)
            segs = cross_page_segments(src_base, list(h.pages), h.page_size, dbase, list(dst_pages), dps, 0, n)
            t3 = clock()
            _add_time("create_and_plan", t3 - t2)
            if has_gpu():
                import torch
                with torch.cuda.device(dev):   # the copy kernel runs on THIS worker's GPU, reading the peer
                    lib().batched_copy(segs, 0, True)
            else:
                lib().batched_copy(segs, 0, True)
            t4 = clock()
            _add_time("copy", t4 - t3)
            crc = None
            if h.crc32c and worker.conf.get_bool("alluxio.worker.peer.verify.crc", "true"):
                # the destination's CRCs, compared with the source's, are also the ones it keeps
                crc = worker.verify_block_crc(block_id, list(h.crc32c), h.page_size)
            t5 = clock()
            _add_time("verify_crc", t5 - t4)
            worker.commit_block(session, block_id, crc=crc)
            _add_time("commit_and_report", clock() - t5)
        except Exception:
            worker.abort_block(session, block_id)
            raise
    finally:
        t6 = clock()
        if stub is not None:
            # the source's read lock goes off the critical path: nothing here waits for the unlock
            # (a lost one expires with the session on the source)
            req = pb.block.UnlockDeviceBlockRequest(block_id=block_id, lock_id=h.lock_id, session_id=session)

            def unlock():
                try:
                    stub.UnlockDeviceBlock(req, timeout=timeout)
                except Exception:  # noqa: BLE001 - the source expires the session's locks itself
                    LOG.warning("unlock of block %d on %s failed", block_id, addr, exc_info=True)
            _control_pool().submit(unlock)
        _add_time("unlock_rpc", clock() - t6)
        _add_time("pulls", 1.0)
        _add_time("total", clock() - t0)
    cross_gpu = h.arena_kind != "dram" and has_gpu() and int(h.device) != dev
    worker.metrics.counter("XgmiBytesReceived" if cross_gpu else "PeerSharedBytesReceived").inc(n)
    return n


def pull_block(worker, block_id: int, addr: str, length: int, tier: int = 0, medium: str = "",
               same_node: bool = True, handle=None) -> int:
    """Copy ``block_id`` from worker ``addr`` into ``worker``; returns the bytes moved (0 when it
    already holds the block).  Same-node peers: mapped pull, falling back to the gRPC block
    stream (and marking the peer) when that fails; other nodes: the gRPC block stream."""
    if worker.has_block(block_id):
        return 0
    mapped_ok = (same_node and worker.conf.get_bool("alluxio.worker.ipc.enabled", "true")
                 and not peer_failed(worker, addr))
    if mapped_ok:
        try:
            return mapped_pull(worker, block_id, addr, tier, medium, handle)
        except Exception as e:  # noqa: BLE001
            if worker.has_block(block_id):
                return 0   # a concurrent pull won the race
            LOG.warning("mapped pull of block %d from %s failed (%s); using the block stream", block_id, addr, e)
            mark_failed(worker, addr)
    from ..worker.remote import remote_block_fetcher
    host, port = addr.rsplit(":", 1)
    remote_block_fetcher(worker, host, int(port), length or None)(block_id)
    worker.metrics.counter("PeerStreamBytesReceived").inc(length)
    return length


_pool_lock = threading.Lock()
_pool = None


def _control_pool():
    """Threads for the fan-out's control calls (PeerTransfer to the replicas, deferred unlocks):
    created once per process, not a thread per call."""
    global _pool
    with _pool_lock:
        if _pool is None:
            from concurrent.futures import ThreadPoolExecutor
            _pool = ThreadPoolExecutor(16, thread_name_prefix="peer-control")
        return _pool


def fan_out(src_worker_addr: str, replica_addrs: list[str], block_id: int, length: int, stub_for,
            timeout_s: float = 60.0, share_handle: bool = True) -> list[tuple[str, str]]:
    """Ask every replica to pull ``block_id`` from ``src_worker_addr`` (``PeerTransfer``), all in
    flight at once; returns ``[(replica, error)]`` for the ones that failed.

    The block is opened on the source ONCE for all replicas (``OpenDeviceBlock``: read lock + page
    list + arena handle) and the handle rides in each PeerTransfer, so a replica's pull costs no
    control call to the source; the lock goes when the last replica is done (one unlock per
    block instead of an open and an unlock per replica)."""
    errors: list[tuple[str, str]] = []
    lock = threading.Lock()
    handle, session = None, 0
    t0 = time.perf_counter()
    if share_handle and replica_addrs:
        session = ids.create_session_id()
        try:
            handle = stub_for(src_worker_addr).OpenDeviceBlock(
                pb.block.OpenDeviceBlockRequest(block_id=block_id, session_id=session), timeout=timeout_s)
        except Exception:  # noqa: BLE001 - not shareable (file tier, ...): each replica opens itself
            LOG.debug("shared open of block %d on %s failed", block_id, src_worker_addr, exc_info=True)
            handle = None
    t1 = time.perf_counter()
    _add_time("fan_open_rpc", t1 - t0)

    def one(addr: str) -> None:
        try:
            req = pb.block.PeerTransferRequest(block_id=block_id, length=length, src_address=src_worker_addr)
            if handle is not None:
                req.handle.CopyFrom(handle)
            tc = time.perf_counter()
            _add_time("fan_call_start", tc - t1)       # queued on the control pool
            r = stub_for(addr).PeerTransfer(req, timeout=timeout_s)
            _add_time("fan_call", time.perf_counter() - tc)
            _add_time("fan_calls", 1.0)
            if not r.ok:
                raise RuntimeError(r.message)
        except Exception as e:  # noqa: BLE001
            with lock:
                errors.append((addr, str(e)))

    try:
        futs = [_control_pool().submit(one, a) for a in replica_addrs[1:]]
        if replica_addrs:
            one(replica_addrs[0])
        for f in futs:
            f.result()
    finally:
        t2 = time.perf_counter()
        _add_time("fan_transfers", t2 - t1)
        if handle is not None:
            try:
                stub_for(src_worker_addr).UnlockDeviceBlock(pb.block.UnlockDeviceBlockRequest(
                    block_id=block_id, lock_id=handle.lock_id, session_id=session), timeout=timeout_s)
            except Exception:  # noqa: BLE001 - the source expires the session's locks itself
                LOG.warning("unlock of block %d on %s failed", block_id, src_worker_addr, exc_info=True)
        t3 = time.perf_counter()
        _add_time("fan_unlock_rpc", t3 - t2)
        _add_time("fan_total", t3 - t0)
        _add_time("fans", 1.0)
    return errors


def is_same_node(worker, host: str) -> bool:
    import socket
    mine = getattr(worker.address, "host", "127.0.0.1")
    return host in ("127.0.0.1", "localhost", mine, socket.gethostname(), os.environ.get("ALLUXIO_NODE_HOST", "\0"))
