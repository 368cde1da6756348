"""Inode last-access-time updates (reference
core/server/master/src/main/java/alluxio/master/file/AccessTimeUpdater.java, 168 lines).

``getStatus`` with a READ/WRITE access mode and ``updateTimestamps`` (what a client's open sends)
and ``listStatus`` (every listed directory) call :meth:`AccessTimeUpdater.update` with the
operation time (DefaultFileSystemMaster.java:882, :1103).  An access less than
``alluxio.master.file.access.time.update.precision`` after the recorded one is ignored.  With
``alluxio.master.file.access.time.journal.flush.interval`` > 0 the new time is applied to the inode
at once and journaled in a batch -- one journal context per flush interval for every inode touched
meanwhile, as the reference's scheduled ``flushUpdates`` does; with 0 each update is journaled
synchronously.  Pending updates are flushed on stop (``beforeShutdown``).  Replay applies the same
``UpdateInodeEntry{last_access_time_ms}`` with max() semantics, so a batch that lands after a newer
synchronous update never moves the time backwards.
"""
from __future__ import annotations

import logging
import threading

from ..proto import pb
from .inode import now_ms

LOG = logging.getLogger(__name__)


class AccessTimeUpdater:
    def __init__(self, fsm, flush_interval_ms: int, precision_ms: int, shutdown_timeout_ms: int = 1000):
        self.fsm = fsm
        self.flush_interval_ms = flush_interval_ms
        self.precision_ms = precision_ms
        self.shutdown_timeout_s = max(0.0, shutdown_timeout_ms / 1000.0)
        self._pending: dict[int, int] = {}
        self._lock = threading.Lock()
        self._timer: threading.Timer | None = None
        self._running = False
        self.flushes = 0
        self.updates = 0

    def start(self) -> None:
        self._running = self.flush_interval_ms > 0

    def stop(self) -> None:
        with self._lock:
            t, self._timer = self._timer, None
        if t is not None:
            t.cancel()
        if self._running:
            self.flush()
        self._running = False

    def update(self, inode, op_time_ms: int | None = None) -> None:
        """Record an access of ``inode`` (callers hold at least the tree read lock, never the
        write lock: a synchronous update takes it)."""
        op = op_time_ms if op_time_ms is not None else now_ms()
        if op - inode.last_access_time_ms <= self.precision_ms:
            return
        self.updates += 1
        if not self._running:
            self._journal({inode.id: op})
            return
        # applied now, journaled with the next flush (updateInodeAccessTimeNoJournal)
        inode.last_access_time_ms = max(inode.last_access_time_ms, op)
        self.fsm.tree._bump_epoch()          # cached FileInfos carry the old time
        with self._lock:
            self._pending[inode.id] = max(op, self._pending.get(inode.id, 0))
            if self._timer is None:
                self._timer = threading.Timer(self.flush_interval_ms / 1000.0, self._scheduled_flush)
                self._timer.daemon = True
                self._timer.start()

    def _scheduled_flush(self) -> None:
        with self._lock:
            self._timer = None
        try:
            self.flush()
        except Exception:  # noqa: BLE001 -- journal unavailable (lost primacy): dropped like the reference
            LOG.debug("Failed to flush access time updates.", exc_info=True)

    def flush(self) -> int:
        with self._lock:
            pending, self._pending = self._pending, {}
        if pending:
            self._journal(pending)
            self.flushes += 1
        return len(pending)

    def _journal(self, updates: dict[int, int]) -> None:
        from .file_system_master import RpcContext
        fsm = self.fsm
        with RpcContext(fsm) as rpc, fsm.tree.lock.write():
            for iid, t in updates.items():
                if iid not in fsm.tree.inodes:
                    continue       # deleted meanwhile
                fsm._apply(rpc, pb.journal.JournalEntry(update_inode=pb.journal.UpdateInodeEntry(
                    id=iid, last_access_time_ms=t)))
