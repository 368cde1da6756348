"""Opt-in phase timing of master operations (where one CreateFile's time goes under load).

Enabled by ``ALLUXIO_MASTER_OP_TIMING=<file>`` in the master's environment: the native RPC
dispatcher records each call's queue-to-handler, handler and journal-flush wait times, the
namespace records path-lock and tree-write-lock waits, and at exit (or ``dump()``) the per-phase
count / mean / p50 / p99 in microseconds go to ``<file>`` as JSON.  Off by default: then ``add``
is a no-op behind one module-global check.
"""
from __future__ import annotations

import atexit
import json
import os
import random
import threading

PATH = os.environ.get("ALLUXIO_MASTER_OP_TIMING", "")
ENABLED = bool(PATH)
_LOCK = threading.Lock()
_SAMPLES: dict[str, list[float]] = {}
_COUNTS: dict[str, int] = {}
_SUMS: dict[str, float] = {}
_KEEP = 20000


def add(key: str, seconds: float) -> None:
    if not ENABLED:
        return
    with _LOCK:
        n = _COUNTS.get(key, 0) + 1
        _COUNTS[key] = n
        _SUMS[key] = _SUMS.get(key, 0.0) + seconds
        s = _SAMPLES.setdefault(key, [])
        if len(s) < _KEEP:
            s.append(seconds)
        else:                      # reservoir: percentiles stay unbiased over a long run
            j = random.randrange(n)
            if j < _KEEP:
                s[j] = seconds


_REPORTERS: dict = {}


def add_reporter(name: str, fn) -> None:
    """``fn()`` -> dict, included in the report under ``name`` (e.g. native journal commit stats)."""
    _REPORTERS[name] = fn


def report() -> dict:
    with _LOCK:
        out = {}
        for name, fn in list(_REPORTERS.items()):
            try:
                out[name] = fn()
            except Exception as e:  # noqa: BLE001
                out[name] = {"error": str(e)}
        for k, s in _SAMPLES.items():
            v = sorted(s)
            out[k] = {"count": _COUNTS[k], "mean_us": round(_SUMS[k] / _COUNTS[k] * 1e6, 1),
                      "p50_us": round(v[len(v) // 2] * 1e6, 1), "p99_us": round(v[min(len(v) - 1, int(len(v) * 0.99))] * 1e6, 1)}
        return out


def dump(path: str | None = None) -> None:
    p = path or PATH
    if p:
        with open(p, "w") as f:
            json.dump(report(), f, indent=1, sort_keys=True)


if ENABLED:
    atexit.register(dump)
