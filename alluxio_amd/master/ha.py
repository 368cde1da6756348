"""Primary election for HA masters.

Parity: core/server/common/src/main/java/alluxio/master/PrimarySelector.java (state PRIMARY /
SECONDARY + listeners), ZkMasterInquireClient / PrimarySelectorClient.java:286 (Curator
LeaderSelector on a ZooKeeper path) and FaultTolerantAlluxioMasterProcess.java:59-194 (standby
tails the journal; on election it gains primacy and starts serving; on loss it steps down).

ZooKeeper is not part of this stack; masters of an HA group share the UFS journal directory, so
election is an exclusive ``flock`` on a lock file in that shared directory: whoever holds it is
primary, and the kernel releases it when the holder dies (the ZK ephemeral-node property).
"""
from __future__ import annotations

import fcntl
import logging
import os
import threading

LOG = logging.getLogger(__name__)


class PrimarySelector:
    PRIMARY, SECONDARY = "PRIMARY", "SECONDARY"

    def start(self, on_primary, on_secondary=None) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def stop(self) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    @property
    def state(self) -> str:  # pragma: no cover - interface
        raise NotImplementedError


class AlwaysPrimarySelector(PrimarySelector):
    """Single-master deployments (UfsJournalSingleMasterPrimarySelector)."""

    def __init__(self):
        self._state = self.SECONDARY

    def start(self, on_primary, on_secondary=None) -> None:
        self._state = self.PRIMARY
        on_primary()

    def stop(self) -> None:
        self._state = self.SECONDARY

    @property
    def state(self) -> str:
        return self._state


class FileLockPrimarySelector(PrimarySelector):
    def __init__(self, lock_path: str, poll_s: float = 0.1):
        self.lock_path = lock_path
        self.poll_s = poll_s
        self._fd = None
        self._state = self.SECONDARY
        self._stop = threading.Event()
        self._t = None

    @property
    def state(self) -> str:
        return self._state

    def _try_acquire(self) -> bool:
        fd = os.open(self.lock_path, os.O_CREAT | os.O_RDWR, 0o644)
        try:
            fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError:
            os.close(fd)
            return False
        os.ftruncate(fd, 0)
        os.write(fd, f"{os.getpid()}\n".encode())
        self._fd = fd
        return True

    def start(self, on_primary, on_secondary=None) -> None:
        os.makedirs(os.path.dirname(self.lock_path) or ".", exist_ok=True)
        self._stop.clear()

        def run():
            while not self._stop.is_set():
                if self._try_acquire():
                    self._state = self.PRIMARY
                    LOG.info("elected primary (lock %s)", self.lock_path)
                    try:
                        on_primary()
                    except Exception:  # noqa: BLE001
                        LOG.exception("gaining primacy failed; releasing the lock")
                        self._release()
                        self._state = self.SECONDARY
                        if on_secondary is not None:
                            on_secondary()
                        continue
                    return
                self._stop.wait(self.poll_s)
        self._t = threading.Thread(target=run, name="primary-selector", daemon=True)
        self._t.start()

    def wait_primary(self, timeout: float) -> bool:
        if self._t is not None:
            self._t.join(timeout)
        return self._state == self.PRIMARY

    def _release(self) -> None:
        if self._fd is not None:
            try:
                fcntl.flock(self._fd, fcntl.LOCK_UN)
            finally:
                os.close(self._fd)
                self._fd = None

    def halt(self) -> None:
        """Stop contending for primacy but keep a held lock (shutdown closes the journal first)."""
        self._stop.set()
        if self._t is not None and self._t is not threading.current_thread():
            self._t.join(timeout=5)

    def stop(self) -> None:
        self.halt()
        self._release()
        self._state = self.SECONDARY
