"""Client-side renewal of worker sessions that outlive a single RPC.

A short-circuit handle (``IpcBlockReader`` / ``IpcBlockWriter``) maps the worker's arena and works
on its pages for as long as the caller keeps it open, but the worker only knows the handle through
its session, which ``cleanup_expired_sessions`` reclaims after ``alluxio.worker.session.timeout``
without a heartbeat.  Reclaiming an open write hands its reserved pages to another block while the
client is still DMA-ing into them.  The reference ties that lifetime to the CreateLocalBlock /
OpenLocalBlock stream instead (core/server/worker/src/main/java/alluxio/worker/grpc/
ShortCircuitBlockWriteHandler.java: the temp block lives until the stream completes or fails);
here one daemon thread per client context renews every open session, grouped per worker, with one
``SessionHeartbeat`` call each ``interval`` -- a dead client stops renewing and its sessions expire
as before.
"""
from __future__ import annotations

import logging
import threading

from ..proto import pb

LOG = logging.getLogger(__name__)


class SessionKeeper:
    def __init__(self, ctx, interval_s: float):
        self.ctx = ctx
        self.interval = max(0.05, interval_s)
        self._open: dict[str, dict[int, int]] = {}     # worker address -> session -> open handles
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._stop = False
        self._thread: threading.Thread | None = None
        self.renewals = 0
        self.lost: set[int] = set()                    # sessions a worker no longer knew

    def add(self, address: str, session: int) -> None:
        with self._lock:
            per = self._open.setdefault(address, {})
            per[session] = per.get(session, 0) + 1
            if self._thread is None and not self._stop:
                self._thread = threading.Thread(target=self._run, daemon=True, name="session-keeper")
                self._thread.start()

    def remove(self, address: str, session: int) -> None:
        with self._lock:
            per = self._open.get(address)
            if not per or session not in per:
                return
            per[session] -= 1
            if per[session] <= 0:
                del per[session]
            if not per:
                del self._open[address]

    def open_sessions(self) -> dict[str, list[int]]:
        with self._lock:
            return {a: sorted(s) for a, s in self._open.items()}

    def renew_now(self) -> int:
        """One renewal round (also run by the thread); returns the sessions renewed."""
        n = 0
        for address, sessions in self.open_sessions().items():
            try:
                r = self.ctx.worker_stub(address).SessionHeartbeat(
                    pb.block.SessionHeartbeatRequest(session_ids=sessions))
            except Exception:  # noqa: BLE001 -- the worker is down or busy: retried next round
                LOG.debug("session heartbeat to %s failed", address, exc_info=True)
                continue
            gone = set(r.unknown_session_ids)
            if gone:
                LOG.warning("worker %s lost short-circuit sessions %s", address, sorted(gone))
                self.lost |= gone
            n += len(sessions) - len(gone)
        self.renewals += 1
        return n

    def _run(self) -> None:
        while not self._stop:
            self._wake.wait(self.interval)
            self._wake.clear()
            if self._stop:
                break
            try:
                self.renew_now()
            except Exception:  # noqa: BLE001
                LOG.debug("session renewal round failed", exc_info=True)

    def close(self) -> None:
        self._stop = True
        self._wake.set()
