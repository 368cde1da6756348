"""Metrics system: registry, instruments, sinks.

Parity: core/common/src/main/java/alluxio/metrics/MetricsSystem.java (registry keyed by
``<Instance>.<Name>.<tags>``, counters/meters/timers/gauges, client & worker metrics shipped to
the master in heartbeats), metrics sinks (console/CSV/JSON servlet/Prometheus servlet:
core/server/common/.../metrics/sink/{MetricsServlet,PrometheusMetricsServlet}.java).
"""
from __future__ import annotations

import bisect
import collections
import csv
import json
import logging
import math
import os
import re
import threading
import time

from .keys import CATALOG, TYPES  # noqa: F401


class Counter:
    """LongAdder-style counter: ``inc`` is one GIL-atomic deque append (no lock, so hot RPC paths
    never convoy on it); pending increments are folded in under a lock when read or every 4096."""

    __slots__ = ("_v", "_pending", "_lock", "_sources")

    def __init__(self):
        self._v = 0
        self._pending = collections.deque()
        self._lock = threading.Lock()
        self._sources = ()

    def add_source(self, fn) -> None:
        """Count ``fn()`` too: a monotonic counter kept elsewhere (a native server's bytes)."""
        self._sources = self._sources + (fn,)

    def inc(self, n: int = 1) -> None:
        self._pending.append(n)
        if len(self._pending) > 4096:
            self._fold()

    def dec(self, n: int = 1) -> None:
        self.inc(-n)

    def _fold(self) -> int:
        with self._lock:
            q = self._pending
            s = 0
            for _ in range(len(q)):
                s += q.popleft()
            self._v += s
            v = self._v
        for fn in self._sources:
            v += fn()
        return v

    @property
    def count(self) -> int:
        return self._fold()

    def value(self):
        return self._fold()


class Meter:
    """Exponentially-weighted 1/5/15-minute rates + mean rate (Codahale semantics: marks go to an
    uncounted adder, folded into the rates on 5 s ticks)."""

    _TICK = 5.0

    def __init__(self):
        self._lock = threading.Lock()
        self._count = Counter()
        self._start = time.monotonic()
        self._last_tick = self._start
        self._uncounted = Counter()
        self._rates = [0.0, 0.0, 0.0]
        self._init = [False, False, False]
        self._alphas = [1 - math.exp(-self._TICK / 60.0 / m) for m in (1, 5, 15)]

    def mark(self, n: int = 1) -> None:
        if time.monotonic() - self._last_tick >= self._TICK:
            with self._lock:
                self._tick()
        self._count.inc(n)
        self._uncounted.inc(n)

    def _tick(self):
        now = time.monotonic()
        while now - self._last_tick >= self._TICK:
            with self._uncounted._lock:
                q = self._uncounted._pending
                pend = sum(q.popleft() for _ in range(len(q))) + self._uncounted._v
                self._uncounted._v = 0
            inst = pend / self._TICK
            for i, a in enumerate(self._alphas):
                if self._init[i]:
                    self._rates[i] += a * (inst - self._rates[i])
                else:
                    self._rates[i] = inst
                    self._init[i] = True
            self._last_tick += self._TICK

    @property
    def count(self) -> int:
        return self._count.count

    def one_minute_rate(self) -> float:
        with self._lock:
            self._tick()
            return self._rates[0]

    def mean_rate(self) -> float:
        el = time.monotonic() - self._start
        return self.count / el if el > 0 else 0.0

    def value(self):
        return self.one_minute_rate()


class Timer:
    """Duration histogram (reservoir of the last 1028 samples) + meter; ``update`` is lock-free."""

    def __init__(self, reservoir: int = 1028):
        self._samples = collections.deque(maxlen=reservoir)
        self.meter = Meter()
        self._sum = collections.deque()
        self._sum_v = 0.0
        self._lock = threading.Lock()

    def update(self, seconds: float) -> None:
        self._samples.append(seconds)
        self._sum.append(seconds)
        if len(self._sum) > 4096:
            self._fold_sum()
        self.meter.mark()

    def _fold_sum(self) -> float:
        with self._lock:
            q = self._sum
            s = 0.0
            for _ in range(len(q)):
                s += q.popleft()
            self._sum_v += s
            return self._sum_v

    def time(self):
        t = self

        class _Ctx:
            def __enter__(self):
                self.t0 = time.perf_counter()
                return self

            def __exit__(self, *exc):
                t.update(time.perf_counter() - self.t0)
        return _Ctx()

    @property
    def count(self) -> int:
        return self.meter.count

    def percentile(self, p: float) -> float:
        s = sorted(list(self._samples))
        if not s:
            return 0.0
        return s[min(len(s) - 1, int(p * len(s)))]

    def mean(self) -> float:
        total = self._fold_sum()
        c = self.count
        return total / c if c else 0.0

    def value(self):
        return self.mean()


class Gauge:
    def __init__(self, fn):
        self.fn = fn

    def value(self):
        try:
            return self.fn()
        except Exception:  # noqa: BLE001
            return float("nan")


class Histogram(Timer):
    pass


_TAG_SEP = "."


def metric_name(instance: str, name: str, tags: dict | None = None) -> str:
    """``Worker.BytesReadAlluxio`` or ``Worker.BytesReadAlluxio.User:alice`` (tags sorted)."""
    base = name if name.startswith(instance + ".") or not instance else f"{instance}.{name}"
    if tags:
        base += _TAG_SEP + _TAG_SEP.join(f"{k}:{v}" for k, v in sorted(tags.items()))
    return base


class MetricsRegistry:
    def __init__(self):
        self._lock = threading.RLock()
        self._m: dict[str, object] = {}

    def _get(self, name, factory):
        m = self._m.get(name)          # lock-free hit (dict reads are atomic)
        if m is not None:
            return m
        with self._lock:
            m = self._m.get(name)
            if m is None:
                m = self._m[name] = factory()
            return m

    def counter(self, name: str) -> Counter:
        return self._get(name, Counter)

    def meter(self, name: str) -> Meter:
        return self._get(name, Meter)

    def timer(self, name: str) -> Timer:
        return self._get(name, Timer)

    def histogram(self, name: str) -> Histogram:
        return self._get(name, Histogram)

    def gauge(self, name: str, fn) -> Gauge:
        with self._lock:
            g = Gauge(fn)
            self._m[name] = g
            return g

    def remove(self, name: str) -> None:
        with self._lock:
            self._m.pop(name, None)

    def clear(self) -> None:
        with self._lock:
            self._m.clear()

    def items(self):
        with self._lock:
            return list(self._m.items())

    def snapshot(self) -> dict[str, float]:
        return {k: v.value() for k, v in self.items()}

    def typed(self, name: str):
        with self._lock:
            return self._m.get(name)


class MetricsSystem:
    """Process-wide registry with instance prefixing and master-report helpers."""

    def __init__(self, instance: str = "Client"):
        self.instance = instance
        self.registry = MetricsRegistry()
        self._sinks = []
        self._last_reported: dict[str, float] = {}
        self._lock = threading.Lock()

    def counter(self, name, tags=None) -> Counter:
        return self.registry.counter(metric_name(self.instance, name, tags))

    def meter(self, name, tags=None) -> Meter:
        return self.registry.meter(metric_name(self.instance, name, tags))

    def timer(self, name, tags=None) -> Timer:
        return self.registry.timer(metric_name(self.instance, name, tags))

    def gauge(self, name, fn, tags=None) -> Gauge:
        return self.registry.gauge(metric_name(self.instance, name, tags), fn)

    # ---- reporting to the master (delta counters, like MetricsSystem.reportMetrics) ----------
    def report_metrics(self):
        """Return ``[(full_name, type, value)]`` with counter values as deltas since last report."""
        out = []
        with self._lock:
            for name, m in self.registry.items():
                if isinstance(m, Counter):
                    v = float(m.count)
                    prev = self._last_reported.get(name, 0.0)
                    if v != prev:
                        out.append((name, "COUNTER", v - prev))
                        self._last_reported[name] = v
                elif isinstance(m, Gauge):
                    v = m.value()
                    if isinstance(v, (int, float)) and not math.isnan(v):
                        out.append((name, "GAUGE", float(v)))
                elif isinstance(m, Timer):
                    out.append((name, "TIMER", float(m.count)))
                elif isinstance(m, Meter):
                    out.append((name, "METER", m.one_minute_rate()))
        return out

    # ---- sinks --------------------------------------------------------------------------------
    def to_json(self) -> str:
        gauges, counters, meters, timers = {}, {}, {}, {}
        for name, m in self.registry.items():
            if isinstance(m, Counter):
                counters[name] = {"count": m.count}
            elif isinstance(m, Timer):
                timers[name] = {"count": m.count, "mean": m.mean(), "p99": m.percentile(0.99)}
            elif isinstance(m, Meter):
                meters[name] = {"count": m.count, "m1_rate": m.one_minute_rate(), "mean_rate": m.mean_rate()}
            elif isinstance(m, Gauge):
                gauges[name] = {"value": m.value()}
        return json.dumps({"version": "4.0.0", "gauges": gauges, "counters": counters, "meters": meters,
                           "timers": timers}, default=str, sort_keys=True)

    def to_prometheus(self) -> str:
        return prometheus_text(self.registry.items())

    def add_sink(self, sink) -> None:
        self._sinks.append(sink)

    def start_sinks(self) -> None:
        for s in self._sinks:
            s.start(self)

    def stop_sinks(self) -> None:
        for s in self._sinks:
            s.stop()


_PROM_BAD = re.compile(r"[^a-zA-Z0-9_:]")


def prometheus_text(items) -> str:
    lines = []
    for name, m in items:
        base, _, tagstr = name.partition(_TAG_SEP) if False else (name, "", "")
        parts = name.split(".")
        labels = {}
        keep = []
        for p in parts:
            if ":" in p:
                k, v = p.split(":", 1)
                labels[_PROM_BAD.sub("_", k)] = v
            else:
                keep.append(p)
        pname = _PROM_BAD.sub("_", "_".join(keep))
        lab = ("{" + ",".join(f'{k}="{v}"' for k, v in sorted(labels.items())) + "}") if labels else ""
        if isinstance(m, Counter):
            lines.append(f"# TYPE {pname}_total counter")
            lines.append(f"{pname}_total{lab} {m.count}")
        elif isinstance(m, Timer):
            lines.append(f"# TYPE {pname} summary")
            lines.append(f"{pname}_count{lab} {m.count}")
            lines.append(f"{pname}_sum{lab} {m.mean() * m.count}")
        elif isinstance(m, Meter):
            lines.append(f"# TYPE {pname}_total counter")
            lines.append(f"{pname}_total{lab} {m.count}")
        elif isinstance(m, Gauge):
            v = m.value()
            if isinstance(v, (int, float)):
                lines.append(f"# TYPE {pname} gauge")
                lines.append(f"{pname}{lab} {v}")
    return "\n".join(lines) + "\n"


class _PeriodicSink:
    def __init__(self, period_s: float = 10.0):
        self.period = period_s
        self._stop = threading.Event()
        self._t = None

    def start(self, system: MetricsSystem):
        self._system = system
        self._t = threading.Thread(target=self._run, daemon=True, name=type(self).__name__)
        self._t.start()

    def _run(self):
        while not self._stop.wait(self.period):
            self.report(self._system)

    def stop(self):
        self._stop.set()

    def report(self, system):  # pragma: no cover
        raise NotImplementedError


class ConsoleSink(_PeriodicSink):
    def report(self, system):
        for k, v in sorted(system.registry.snapshot().items()):
            print(f"{k} = {v}")


class CsvSink(_PeriodicSink):
    def __init__(self, directory: str, period_s: float = 10.0):
        super().__init__(period_s)
        self.dir = directory
        os.makedirs(directory, exist_ok=True)

    def report(self, system):
        now = time.time()
        for k, v in system.registry.snapshot().items():
            p = os.path.join(self.dir, k + ".csv")
            new = not os.path.exists(p)
            with open(p, "a", newline="") as f:
                w = csv.writer(f)
                if new:
                    w.writerow(["t", "value"])
                w.writerow([f"{now:.3f}", v])


class GraphiteSink(_PeriodicSink):
    """Plaintext Graphite protocol over TCP: ``<prefix.name> <value> <epoch>\n`` (GraphiteSink.java)."""

    def __init__(self, host: str, port: int, period_s: float = 10.0, prefix: str = ""):
        super().__init__(period_s)
        self.host, self.port, self.prefix = host, int(port), prefix

    def report(self, system):
        import socket
        now = int(time.time())
        lines = []
        for k, v in sorted(system.registry.snapshot().items()):
            if isinstance(v, (int, float)) and not math.isnan(v):
                name = (self.prefix + "." if self.prefix else "") + re.sub(r"[\s]", "_", k)
                lines.append(f"{name} {v} {now}\n")
        if lines:
            with socket.create_connection((self.host, self.port), timeout=5) as so:
                so.sendall("".join(lines).encode())


class LoggingSink(_PeriodicSink):
    """Slf4jSink: metrics to the ``alluxio_amd.metrics`` logger, optionally regex-filtered."""

    def __init__(self, period_s: float = 10.0, filter_regex: str | None = None):
        super().__init__(period_s)
        self.filter = re.compile(filter_regex) if filter_regex else None
        self.log = logging.getLogger("alluxio_amd.metrics")

    def report(self, system):
        for k, v in sorted(system.registry.snapshot().items()):
            if self.filter is None or self.filter.search(k):
                self.log.info("type=METRIC name=%s value=%s", k, v)


_UNITS = {"milliseconds": 0.001, "seconds": 1.0, "minutes": 60.0, "hours": 3600.0}


def sinks_from_properties(props: dict) -> list:
    """``sink.<name>.class`` / ``.period`` / ``.unit`` / sink options (conf/metrics.properties)."""
    groups: dict[str, dict] = {}
    for k, v in props.items():
        if k.startswith("sink.") and k.count(".") >= 2:
            _, name, opt = k.split(".", 2)
            groups.setdefault(name, {})[opt] = v
    out = []
    for name, o in sorted(groups.items()):
        cls = o.get("class", "").rsplit(".", 1)[-1]
        period = float(o.get("period", 10)) * _UNITS.get(o.get("unit", "seconds").lower(), 1.0)
        if cls == "ConsoleSink":
            out.append(ConsoleSink(period))
        elif cls == "CsvSink":
            out.append(CsvSink(o.get("directory", "/tmp"), period))
        elif cls == "GraphiteSink":
            out.append(GraphiteSink(o["host"], int(o["port"]), period, o.get("prefix", "")))
        elif cls == "Slf4jSink":
            out.append(LoggingSink(period, o.get("filter-regex")))
        # MetricsServlet / PrometheusMetricsServlet are the web endpoints; JmxSink has no analogue
    return out


def load_sinks(conf, system: "MetricsSystem") -> list:
    """Attach the sinks configured in ``alluxio.metrics.conf.file`` to ``system`` and start them."""
    try:
        path = conf.get("alluxio.metrics.conf.file") if conf is not None else None
    except Exception:  # noqa: BLE001  (unresolvable ${alluxio.conf.dir})
        return []
    if not path or not os.path.isfile(path):
        return []
    from ..conf import load_properties_file
    sinks = sinks_from_properties(load_properties_file(path))
    for s in sinks:
        system.add_sink(s)
        s.start(system)
    return sinks


_SYSTEMS: dict[str, MetricsSystem] = {}
_SYS_LOCK = threading.Lock()


def metrics(instance: str = "Client") -> MetricsSystem:
    """Process-wide metrics system per instance type (Master / Worker / Client / JobWorker ...)."""
    with _SYS_LOCK:
        s = _SYSTEMS.get(instance)
        if s is None:
            s = _SYSTEMS[instance] = MetricsSystem(instance)
        return s


def reset_all() -> None:
    with _SYS_LOCK:
        for s in _SYSTEMS.values():
            s.registry.clear()
        _SYSTEMS.clear()


__all__ = ["Counter", "Meter", "Timer", "Gauge", "MetricsRegistry", "MetricsSystem", "metrics",
           "prometheus_text", "ConsoleSink", "CsvSink", "GraphiteSink", "LoggingSink", "sinks_from_properties",
           "load_sinks", "metric_name", "reset_all", "bisect"]
