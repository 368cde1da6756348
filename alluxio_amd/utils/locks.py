"""Reader/writer locks and lock-resource helpers.

Python counterpart of the reference's ``ClientRWLock`` / ``LockResource`` /
``InodeLockManager`` building blocks (core/server/worker/src/main/java/alluxio/worker/block/
ClientRWLock.java, core/common/src/main/java/alluxio/resource/LockResource.java).  The worker's
hot-path block locks live in the native store (``csrc/block_store.cpp``); these are used by the
master inode tree and the control plane.
"""
from __future__ import annotations

import collections
import contextlib
import threading
import time
from collections import defaultdict


class RWLock:
    """Writer-preferring RW lock, reentrant for readers, with timeouts.

    Readers take a lock-free fast path: one GIL-atomic ``deque.append`` plus a check of the writer
    gate (Dekker-style: a writer raises the gate, then waits for the reader deque to drain; a
    reader appends, then backs out if the gate is up).  Uncontended read-mostly namespaces (every
    getStatus / listStatus) therefore never serialise on a mutex the way a Condition-based lock
    does under the GIL.  Writers, and readers that meet a writer, use the condition variable.
    """

    def __init__(self):
        self._cond = threading.Condition(threading.Lock())
        self._readers = collections.deque()   # one token per held read (all threads)
        self._writer: int | None = None
        self._writer_depth = 0
        self._waiting_writers = 0
        self._gate = False                    # a writer holds or waits for the lock
        self._tls = threading.local()         # this thread's read depth

    def _depth(self) -> int:
        return getattr(self._tls, "d", 0)

    def acquire_read(self, timeout: float | None = None) -> bool:
        d = self._depth()
        if d or self._writer == threading.get_ident():
            # nested read, or the write holder reading: never blocks
            self._readers.append(1)
            self._tls.d = d + 1
            return True
        self._readers.append(1)
        if not self._gate:
            self._tls.d = 1
            return True
        self._readers.pop()                   # a writer is in: back out and wait for it
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cond:
            self._cond.notify_all()
            while self._gate:
                if not self._wait(deadline):
                    return False
            self._readers.append(1)
        self._tls.d = 1
        return True

    def release_read(self) -> None:
        self._readers.pop()
        self._tls.d = self._depth() - 1
        if self._gate:
            with self._cond:
                self._cond.notify_all()

    def acquire_write(self, timeout: float | None = None) -> bool:
        me = threading.get_ident()
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cond:
            if self._writer == me:
                self._writer_depth += 1
                return True
            self._waiting_writers += 1
            self._gate = True
            ok = True
            contended = self._writer is not None or bool(self._readers)
            t_wait = time.perf_counter() if contended else 0.0
            try:
                while self._writer is not None or self._readers:
                    if not self._wait(deadline):
                        ok = False
                        break
            finally:
                self._waiting_writers -= 1
            if contended:
                from . import optiming
                if optiming.ENABLED:
                    optiming.add("tree_write_wait", time.perf_counter() - t_wait)
            if not ok:                        # timed out: reopen the gate unless others need it
                self._gate = self._writer is not None or self._waiting_writers > 0
                self._cond.notify_all()
                return False
            self._writer = me
            self._writer_depth = 1
            self._gate = True
            return True

    def release_write(self) -> None:
        with self._cond:
            self._writer_depth -= 1
            if self._writer_depth == 0:
                self._writer = None
                self._gate = self._waiting_writers > 0
                self._cond.notify_all()

    def _wait(self, deadline) -> bool:
        if deadline is None:
            self._cond.wait()
            return True
        remaining = deadline - time.monotonic()
        if remaining <= 0:
            return False
        self._cond.wait(remaining)
        return True

    @contextlib.contextmanager
    def read(self):
        self.acquire_read()
        try:
            yield
        finally:
            self.release_read()

    @contextlib.contextmanager
    def write(self):
        self.acquire_write()
        try:
            yield
        finally:
            self.release_write()

    @property
    def is_write_locked(self) -> bool:
        return self._writer is not None

    @property
    def reader_count(self) -> int:
        return len(self._readers)


class LockPool:
    """Lazily created, reference-counted keyed RW locks (reference ``LockPool``)."""

    def __init__(self):
        self._locks: dict = {}
        self._refs: dict = defaultdict(int)
        self._mu = threading.Lock()

    def _get(self, key) -> RWLock:
        with self._mu:
            lk = self._locks.get(key)
            if lk is None:
                lk = self._locks[key] = RWLock()
            self._refs[key] += 1
            return lk

    def _put(self, key) -> None:
        with self._mu:
            self._refs[key] -= 1
            if self._refs[key] <= 0:
                self._refs.pop(key, None)
                lk = self._locks.get(key)
                if lk is not None and lk.reader_count == 0 and not lk.is_write_locked:
                    self._locks.pop(key, None)

    @contextlib.contextmanager
    def locked(self, key, write: bool):
        lk = self._get(key)
        try:
            if write:
                lk.acquire_write()
            else:
                lk.acquire_read()
            try:
                yield
            finally:
                if write:
                    lk.release_write()
                else:
                    lk.release_read()
        finally:
            self._put(key)

    def size(self) -> int:
        with self._mu:
            return len(self._locks)
