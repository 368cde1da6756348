"""Process pause monitor and sampling logger (SURVEY §5.1 slow-path observability).

Parity:
- core/common/src/main/java/alluxio/util/JvmPauseMonitor.java (started by AlluxioMasterProcess.java:
  265-273 and AlluxioWorkerProcess.java:244-251 when ``alluxio.{master,worker}.jvm.monitor.enabled``):
  a thread sleeps ``alluxio.jvm.monitor.sleep.interval`` and measures how much longer the sleep took;
  extra time above ``alluxio.jvm.monitor.info.threshold`` logs at INFO, above
  ``alluxio.jvm.monitor.warn.threshold`` at WARN, with the counters the reference exports
  (total extra time, info / warn threshold exceedances).  In a Python server a pause is a GIL hog,
  a long GC cycle or host memory pressure; the report names the threads that were running.
- core/common/src/main/java/alluxio/util/logging/SamplingLogger.java: at most one message per key
  per interval (used for the slow remote-read log of BlockReadHandler.java:63-65,136-150).
"""
from __future__ import annotations

import gc
import logging
import sys
import threading
import time

LOG = logging.getLogger(__name__)


class PauseMonitor:
    def __init__(self, sleep_s: float = 1.0, info_s: float = 1.0, warn_s: float = 10.0, metrics=None,
                 prefix: str = "Process"):
        self.sleep_s, self.info_s, self.warn_s = sleep_s, info_s, warn_s
        self.metrics = metrics
        self.prefix = prefix
        self.total_extra_s = 0.0
        self.info_exceeded = 0
        self.warn_exceeded = 0
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def start(self) -> "PauseMonitor":
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="pause-monitor", daemon=True)
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=self.sleep_s + 1)
            self._thread = None

    def is_started(self) -> bool:
        return self._thread is not None

    def _run(self) -> None:
        gc_before = sum(s.get("collections", 0) for s in gc.get_stats())
        while not self._stop.is_set():
            t0 = time.monotonic()
            if self._stop.wait(self.sleep_s):
                return
            extra = time.monotonic() - t0 - self.sleep_s
            gc_now = sum(s.get("collections", 0) for s in gc.get_stats())
            self.check(extra, gc_now - gc_before)
            gc_before = gc_now

    def check(self, extra_s: float, gc_collections: int = 0) -> str | None:
        """Account one measured pause; returns the level it was logged at (or None)."""
        if extra_s <= 0:
            return None
        self.total_extra_s += extra_s
        if self.metrics is not None:
            self.metrics.counter(f"{self.prefix}.TotalExtraTime").inc(int(extra_s * 1000))
        level = None
        if extra_s > self.warn_s:
            self.warn_exceeded += 1
            level = "WARN"
        elif extra_s > self.info_s:
            self.info_exceeded += 1
            level = "INFO"
        if level is None:
            return None
        if self.metrics is not None:
            self.metrics.counter(f"{self.prefix}.{'Warn' if level == 'WARN' else 'Info'}TimeExceeded").inc()
        msg = (f"Detected pause in process (e.g. a GIL hog or GC): approximately {extra_s * 1000:.0f}ms; "
               f"{gc_collections} GC collections meanwhile; running threads: {self._threads()}")
        (LOG.warning if level == "WARN" else LOG.info)(msg)
        return level

    @staticmethod
    def _threads() -> str:
        names = {t.ident: t.name for t in threading.enumerate()}
        out = []
        for tid, frame in sys._current_frames().items():
            name = names.get(tid, str(tid))
            if name == "pause-monitor":
                continue
            out.append(f"{name}@{frame.f_code.co_name}")
        return ", ".join(sorted(out)[:12])


def from_conf(conf, role: str, metrics=None) -> PauseMonitor | None:
    """The monitor configured for ``role`` ("master" / "worker"), or None when disabled."""
    if not conf.get_bool(f"alluxio.{role}.jvm.monitor.enabled", "true"):
        return None
    return PauseMonitor(conf.get_ms("alluxio.jvm.monitor.sleep.interval") / 1000.0,
                        conf.get_ms("alluxio.jvm.monitor.info.threshold") / 1000.0,
                        conf.get_ms("alluxio.jvm.monitor.warn.threshold") / 1000.0,
                        metrics, prefix=role.capitalize())


class SamplingLogger:
    """Log at most once per ``interval_s`` per message key (reference SamplingLogger)."""

    def __init__(self, logger: logging.Logger, interval_s: float):
        self.logger = logger
        self.interval_s = interval_s
        self._last: dict = {}
        self._lock = threading.Lock()
        self.suppressed = 0

    def _ok(self, key) -> bool:
        now = time.monotonic()
        with self._lock:
            last = self._last.get(key)
            if last is not None and now - last < self.interval_s:
                self.suppressed += 1
                return False
            self._last[key] = now
            return True

    def warning(self, msg: str, *args, key=None) -> bool:
        if not self._ok(key if key is not None else msg):
            return False
        self.logger.warning(msg, *args)
        return True

    def info(self, msg: str, *args, key=None) -> bool:
        if not self._ok(key if key is not None else msg):
            return False
        self.logger.info(msg, *args)
        return True
