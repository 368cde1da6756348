"""Wall-clock stack sampler for server processes (slow-path profiling).

The reference relies on JVM profilers and its own ``alluxio.util.logging.SamplingLogger`` /
slow-RPC timing logs; a Python process has no JFR, and ``cProfile`` only sees the thread that
enabled it.  This sampler walks ``sys._current_frames()`` of every thread at a fixed interval and
counts leaf functions and whole call stacks, so a master under a multi-threaded RPC load shows
where its handler threads actually spend their time (including time spent waiting on locks).

A sample is taken only when the sampler thread holds the GIL, which it mostly gets when other
threads block, so a GIL-bound process over-reports its parked frames: read it for where requests
wait (locks, journal flushes, native calls), and use cProfile on the handler thread for CPU.

Enable it for a server process with ``ALLUXIO_PYSAMPLE=<out-file>`` (optionally
``ALLUXIO_PYSAMPLE_INTERVAL_MS``); the report is written at exit and on SIGTERM.
"""
from __future__ import annotations

import collections
import os
import signal
import sys
import threading
import time


# leaf frames of parked threads (idle pools, selectors): not work, so not counted
_IDLE = {"threading.py:wait", "threading.py:_wait_for_tstate_lock", "selectors.py:select",
         "queue.py:get", "socket.py:accept", "_base.py:wait", "thread.py:_worker"}


class StackSampler:
    def __init__(self, interval_s: float = 0.002, depth: int = 14):
        self.interval_s, self.depth = interval_s, depth
        self.leaf = collections.Counter()
        self.stacks = collections.Counter()
        self.own = collections.Counter()       # function appears anywhere in the stack (inclusive)
        self.samples = 0
        self.idle_lines = set(filter(None, os.environ.get("ALLUXIO_PYSAMPLE_IDLE", "").split(",")))
        self._stop = threading.Event()
        self._thread = None

    def start(self) -> "StackSampler":
        self._thread = threading.Thread(target=self._run, name="stack-sampler", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None and self._thread is not threading.current_thread():
            self._thread.join(1.0)

    def _run(self) -> None:
        me = threading.get_ident()
        while not self._stop.wait(self.interval_s):
            for tid, frame in sys._current_frames().items():
                if tid == me:
                    continue
                names = []
                f = frame
                while f is not None and len(names) < self.depth:
                    co = f.f_code
                    names.append(f"{os.path.basename(co.co_filename)}:{co.co_name}")
                    if len(names) == 1:     # the leaf keeps its line: tells a parked call from work
                        names[0] += f":{f.f_lineno}"
                    f = f.f_back
                if not names or names[0].rsplit(":", 1)[0] in _IDLE or names[0] in self.idle_lines:
                    continue
                self.samples += 1
                self.leaf[names[0]] += 1
                for n in set(names):
                    self.own[n] += 1
                self.stacks[" <- ".join(names[:8])] += 1

    def report(self, top: int = 40) -> str:
        n = max(1, self.samples)
        out = [f"samples: {self.samples} (interval {self.interval_s * 1e3:.1f} ms, all threads)", "", "leaf:"]
        out += [f"  {100 * c / n:6.2f}%  {k}" for k, c in self.leaf.most_common(top)]
        out += ["", "inclusive:"]
        out += [f"  {100 * c / n:6.2f}%  {k}" for k, c in self.own.most_common(top)]
        out += ["", "stacks:"]
        out += [f"  {100 * c / n:6.2f}%  {k}" for k, c in self.stacks.most_common(top)]
        return "\n".join(out) + "\n"


def maybe_start_from_env() -> StackSampler | None:
    """Start a sampler when ``ALLUXIO_PYSAMPLE`` names an output file; dump on exit / SIGTERM."""
    path = os.environ.get("ALLUXIO_PYSAMPLE")
    if not path:
        return None
    s = StackSampler(float(os.environ.get("ALLUXIO_PYSAMPLE_INTERVAL_MS", "2")) / 1e3).start()
    done = threading.Event()

    def dump(*_):
        if done.is_set():
            return
        done.set()
        s.stop()
        with open(path, "w") as f:
            f.write(s.report())

    import atexit
    atexit.register(dump)
    prev = signal.getsignal(signal.SIGTERM)

    def on_term(signum, frame):
        dump()
        if callable(prev):
            prev(signum, frame)
        else:
            os._exit(0)

    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, on_term)
    return s
