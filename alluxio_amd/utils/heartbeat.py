"""Heartbeat threads with a pluggable timer.

Parity: core/common/src/main/java/alluxio/heartbeat/HeartbeatThread.java:30-129 (thread that
calls ``executor.heartbeat()`` each tick), ``SleepingTimer`` (production: sleep the interval,
warn when a tick overran), ``ScheduledTimer`` + ``HeartbeatScheduler`` (tests tick a named
heartbeat by hand: HeartbeatScheduler.java:35-165).  Tests use :class:`ManualHeartbeat` to drive
master/worker background executors deterministically, exactly like the reference's
``ManuallyScheduleHeartbeat`` JUnit rule.
"""
from __future__ import annotations

import contextlib
import logging
import threading
import time

LOG = logging.getLogger(__name__)

# Names used by masters / workers (reference HeartbeatContext.java).
MASTER_LOST_WORKER_DETECTION = "Master Lost Worker Detection"
MASTER_TTL_CHECK = "Master TTL Check"
MASTER_REPLICATION_CHECK = "Master Replication Check"
MASTER_PERSISTENCE_SCHEDULER = "Master Persistence Scheduler"
MASTER_PERSISTENCE_CHECKER = "Master Persistence Checker"
MASTER_LOST_FILES_DETECTION = "Master Lost Files Detection"
MASTER_BLOCK_INTEGRITY_CHECK = "Master Block Integrity Check"
MASTER_METRICS_TIME_SERIES = "Master Metrics Time Series"
MASTER_UFS_CLEANUP = "Master Ufs Cleanup"
MASTER_DAILY_BACKUP = "Master Daily Backup"
MASTER_LOST_MASTER_DETECTION = "Master Lost Master Detection"
MASTER_ACTIVE_UFS_SYNC = "Master Active UFS Sync"
MASTER_CHECKPOINT_SCHEDULING = "Master Checkpoint Scheduling"
WORKER_BLOCK_SYNC = "Worker Block Sync"
WORKER_PIN_LIST_SYNC = "Worker Pin List Sync"
WORKER_SESSION_CLEANER = "Worker Session Cleaner"
WORKER_STORAGE_HEALTH = "Worker Storage Health"
WORKER_FILESYSTEM_MASTER_SYNC = "Worker FileSystemMaster Sync"
WORKER_TIER_MANAGEMENT = "Worker Tier Management"
JOB_MASTER_LOST_WORKER_DETECTION = "Job Master Lost Worker Detection"
JOB_WORKER_COMMAND_HANDLING = "Job Worker Command Handling"
META_MASTER_SYNC = "Meta Master Sync"
CLIENT_METRICS_SYNC = "Client Metrics Sync"


class HeartbeatExecutor:
    def heartbeat(self) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def close(self) -> None:
        pass


class FunctionExecutor(HeartbeatExecutor):
    def __init__(self, fn):
        self.fn = fn

    def heartbeat(self) -> None:
        self.fn()


class SleepingTimer:
    def __init__(self, name: str, interval_ms: int):
        self.name = name
        self.interval = interval_ms / 1000.0
        self._last = None
        self._stop = threading.Event()

    def tick(self) -> bool:
        if self._last is not None:
            elapsed = time.monotonic() - self._last
            if elapsed > self.interval:
                LOG.debug("%s last execution took %.1f ms, longer than the interval %.1f ms",
                          self.name, elapsed * 1e3, self.interval * 1e3)
            else:
                if self._stop.wait(self.interval - elapsed):
                    return False
        self._last = time.monotonic()
        return not self._stop.is_set()

    def stop(self) -> None:
        self._stop.set()


class ScheduledTimer:
    """A timer that only fires when :func:`HeartbeatScheduler.execute` releases it."""

    def __init__(self, name: str, interval_ms: int = 0):
        self.name = name
        self._cond = threading.Condition()
        self._scheduled = False
        self._stopped = False
        HeartbeatScheduler.add_timer(self)

    def tick(self) -> bool:
        with self._cond:
            HeartbeatScheduler.timer_waiting(self)
            while not self._scheduled and not self._stopped:
                self._cond.wait()
            self._scheduled = False
            return not self._stopped

    def schedule(self) -> None:
        with self._cond:
            self._scheduled = True
            self._cond.notify_all()

    def stop(self) -> None:
        with self._cond:
            self._stopped = True
            self._cond.notify_all()
        HeartbeatScheduler.remove_timer(self)


class HeartbeatScheduler:
    _lock = threading.Condition()
    _timers: dict[str, ScheduledTimer] = {}
    _waiting: set[str] = set()

    @classmethod
    def add_timer(cls, timer: ScheduledTimer) -> None:
        with cls._lock:
            cls._timers[timer.name] = timer
            cls._lock.notify_all()

    @classmethod
    def remove_timer(cls, timer: ScheduledTimer) -> None:
        with cls._lock:
            if cls._timers.get(timer.name) is timer:
                cls._timers.pop(timer.name, None)
            cls._waiting.discard(timer.name)

    @classmethod
    def timer_waiting(cls, timer: ScheduledTimer) -> None:
        with cls._lock:
            cls._waiting.add(timer.name)
            cls._lock.notify_all()

    @classmethod
    def await_ready(cls, name: str, timeout: float = 10.0) -> bool:
        deadline = time.monotonic() + timeout
        with cls._lock:
            while name not in cls._waiting:
                rem = deadline - time.monotonic()
                if rem <= 0:
                    return False
                cls._lock.wait(rem)
            return True

    @classmethod
    def schedule(cls, name: str) -> None:
        with cls._lock:
            timer = cls._timers.get(name)
            cls._waiting.discard(name)
        if timer is None:
            raise KeyError(f"no scheduled heartbeat named {name!r}")
        timer.schedule()

    @classmethod
    def execute(cls, name: str, timeout: float = 10.0) -> None:
        """Run one heartbeat of ``name`` and wait until it has completed."""
        if not cls.await_ready(name, timeout):
            raise TimeoutError(f"heartbeat {name!r} never became ready")
        cls.schedule(name)
        if not cls.await_ready(name, timeout):
            raise TimeoutError(f"heartbeat {name!r} did not finish")


class _ManualRegistry:
    names: set[str] = set()
    lock = threading.Lock()


@contextlib.contextmanager
def manual_heartbeat(*names: str):
    """Context manager: heartbeat threads created inside use :class:`ScheduledTimer`."""
    with _ManualRegistry.lock:
        _ManualRegistry.names.update(names)
    try:
        yield HeartbeatScheduler
    finally:
        with _ManualRegistry.lock:
            _ManualRegistry.names.difference_update(names)


def make_timer(name: str, interval_ms: int):
    with _ManualRegistry.lock:
        manual = name in _ManualRegistry.names
    return ScheduledTimer(name, interval_ms) if manual else SleepingTimer(name, interval_ms)


class HeartbeatThread(threading.Thread):
    def __init__(self, name: str, executor, interval_ms: int):
        super().__init__(name=f"heartbeat-{name}", daemon=True)
        if callable(executor) and not isinstance(executor, HeartbeatExecutor):
            executor = FunctionExecutor(executor)
        self.hb_name = name
        self.executor = executor
        self.timer = make_timer(name, interval_ms)
        self._stopped = False

    def run(self) -> None:
        try:
            while not self._stopped and self.timer.tick():
                if self._stopped:
                    break
                try:
                    self.executor.heartbeat()
                except Exception:  # noqa: BLE001
                    LOG.exception("uncaught exception in heartbeat %s", self.hb_name)
        finally:
            try:
                self.executor.close()
            except Exception:  # noqa: BLE001
                LOG.exception("heartbeat %s close failed", self.hb_name)

    def shutdown(self, join: bool = True) -> None:
        self._stopped = True
        self.timer.stop()
        if join and self.is_alive() and threading.current_thread() is not self:
            self.join(timeout=5)
