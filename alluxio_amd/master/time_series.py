"""Cluster metrics time series kept by the primary master for the web UI.

Parity: the TimeSeriesRecorder heartbeat of
core/server/master/src/main/java/alluxio/master/file/DefaultFileSystemMaster.java:670-674,4087-4160
(every ``alluxio.master.metrics.time.series.interval`` it records % Alluxio space used, % UFS space
used and the cluster read / write throughputs), stored by
core/server/master/src/main/java/alluxio/master/metrics/TimeSeriesStore.java and served by the
master REST handler as ``MasterWebUIMetrics.timeSeriesMetrics``
(core/common/src/main/java/alluxio/wire/MasterWebUIMetrics.java:334; TimeSeries / DataPoint of
core/common/src/main/java/alluxio/metrics/TimeSeries.java).  Throughputs are the growth of the
cluster byte counters since the previous sample, in bytes per minute (the reference's
``*Throughput`` gauges are per-minute meters).  Each series keeps its last ``max_points`` samples.
"""
from __future__ import annotations

import collections
import threading
import time

READ_SERIES = (("Cluster.BytesReadLocalThroughput", "Cluster.BytesReadLocal"),
               ("Cluster.BytesReadDomainThroughput", "Cluster.BytesReadDomain"),
               ("Cluster.BytesReadAlluxioThroughput", "Cluster.BytesReadAlluxio"),
               ("Cluster.BytesReadUfsThroughput", "Cluster.BytesReadUfsAll"))
WRITE_SERIES = (("Cluster.BytesWrittenLocalThroughput", "Cluster.BytesWrittenLocal"),
                ("Cluster.BytesWrittenAlluxioThroughput", "Cluster.BytesWrittenAlluxio"),
                ("Cluster.BytesWrittenDomainThroughput", "Cluster.BytesWrittenDomain"),
                ("Cluster.BytesWrittenUfsThroughput", "Cluster.BytesWrittenUfsAll"))


class TimeSeriesStore:
    def __init__(self, max_points: int = 1440):
        self.max_points = max_points
        self._series: dict[str, collections.deque] = {}
        self._lock = threading.Lock()

    def record(self, name: str, value: float, ts_ms: int | None = None) -> None:
        ts = int(time.time() * 1000) if ts_ms is None else ts_ms
        with self._lock:
            d = self._series.get(name)
            if d is None:
                d = self._series[name] = collections.deque(maxlen=self.max_points)
            d.append((ts, float(value)))

    def series(self) -> list[dict]:
        """[{"name", "dataPoints": [{"timeStamp", "value"}]}] (the reference's JSON shape)."""
        with self._lock:
            return [{"name": n, "dataPoints": [{"timeStamp": t, "value": v} for t, v in d]}
                    for n, d in sorted(self._series.items())]


class TimeSeriesRecorder:
    def __init__(self, block_master, metrics_master, root_ufs_space=None, store: TimeSeriesStore | None = None):
        self.bm = block_master
        self.mm = metrics_master
        self.root_ufs_space = root_ufs_space      # () -> (total, used) bytes, or None
        self.store = store or TimeSeriesStore()
        self._last: tuple[float, dict] | None = None

    def heartbeat(self) -> None:
        s = self.store
        cap, used = self.bm.capacity_bytes(), self.bm.used_bytes()
        s.record("% Alluxio Space Used", int(100 * used / cap) if cap > 0 else 0)
        ufs_pct = 0
        if self.root_ufs_space is not None:
            try:
                total, u = self.root_ufs_space()
                ufs_pct = int(100 * u / total) if total > 0 else 0
            except Exception:  # noqa: BLE001 -- a UFS without space reporting
                ufs_pct = 0
        s.record("% UFS Space Used", ufs_pct)
        now = time.monotonic()
        cluster = self.mm.get_metrics() if self.mm is not None else {}
        counters = {c: float(cluster.get(c, 0)) for _, c in READ_SERIES + WRITE_SERIES}
        prev = self._last
        self._last = (now, counters)
        for name, c in READ_SERIES + WRITE_SERIES:
            if prev is None or now <= prev[0]:
                rate = 0.0
            else:
                rate = max(0.0, counters[c] - prev[1].get(c, 0.0)) * 60.0 / (now - prev[0])
            s.record(name, int(rate))
