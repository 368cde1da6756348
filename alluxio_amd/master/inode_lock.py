"""Path-scoped namespace locks held across UFS I/O.

Parity: core/server/master/src/main/java/alluxio/master/file/meta/InodeLockManager.java,
LockedInodePath.java and the lock patterns of InodeTree.java:99-111 (READ / WRITE_INODE /
WRITE_EDGE) with ``lockInodePath`` :375-436.  The reference locks every inode and edge on the
path in order; a mutation write-locks the edge (or inode) it changes and read-locks the rest, so a
slow UFS call made by one mutation only stalls operations on the *same* subtree.

Here the in-memory tree is guarded by one short-held reader/writer lock (``InodeTree.lock``:
pure dictionary work, microseconds), and the long part of a mutation — UFS ``mkdirs`` / ``delete`` /
``rename`` / ``listStatus`` / fingerprints — runs holding only a lock *list* from this manager:

* ``W`` on the path the mutation changes (the subtree rooted there: the first missing component
  for a create, the victim of a delete, both ends of a rename), ``IW`` (intention) on each
  ancestor;
* ``R`` on a path whose subtree must not change underneath, ``IR`` on its ancestors.

Standard multi-granularity compatibility: ``IR``~{IR, IW, R}, ``IW``~{IR, IW}, ``R``~{IR, R},
``W``~{}.  So a 2 s UFS delete of ``/a/b`` blocks a create under ``/a/b`` (IW vs W) and a delete of
``/a`` (W vs IW), but not a create of ``/a/c`` (IW/IW on ``/a``) nor any reader: reads take no path
locks, they see the namespace as of the last applied journal entry, which is linearisable because
a mutation applies its entries only at the end (resolve -> UFS I/O -> apply).

A lock list is acquired all-or-nothing under one mutex (no lock-order deadlocks between lists),
and is reentrant per thread: holds of the calling thread never conflict with its new requests, so
a mutation may call another one on its own subtree.
"""
from __future__ import annotations

import threading
import time

from ..utils import optiming
from ..utils.exceptions import DeadlineExceededException
from ..utils.uri import normalize_path

IR, IW, R, W = "IR", "IW", "R", "W"

_LANE = threading.local()


class WouldBlock(Exception):
    """Raised on a non-blocking RPC lane where the handler would wait on a path lock or start UFS
    I/O.  Nothing has been applied at that point; the RPC front end re-runs the request on its
    blocking pool, so the fast lanes never sit behind a slow UFS."""


class nonblocking_lane:
    """Marks the current thread as a fast RPC lane for the duration of one request."""

    def __enter__(self):
        self._prev = getattr(_LANE, "nb", False)
        _LANE.nb = True
        return self

    def __exit__(self, *exc):
        _LANE.nb = self._prev
        return False


def check_may_block(what: str) -> None:
    """Call before anything slow (UFS I/O) at a point where nothing has been applied yet."""
    if getattr(_LANE, "nb", False):
        raise WouldBlock(what)


_COMPAT = {
    IR: frozenset((IR, IW, R)),
    IW: frozenset((IR, IW)),
    R: frozenset((IR, R)),
    W: frozenset(),
}
_INTENT = {R: IR, W: IW, IR: IR, IW: IW}


def _ancestors(path: str) -> list[str]:
    """``/a/b/c`` -> ``["/", "/a", "/a/b"]``."""
    if path == "/":
        return []
    out = ["/"]
    i = path.find("/", 1)
    while i != -1:
        out.append(path[:i])
        i = path.find("/", i + 1)
    return out


class LockList:
    """The locks one operation holds (``LockedInodePath``); release with ``close`` / ``with``."""

    __slots__ = ("_mgr", "_holds", "_owner", "paths")

    def __init__(self, mgr: "PathLockManager", holds: list, owner: int, paths: list):
        self._mgr = mgr
        self._holds = holds
        self._owner = owner
        self.paths = paths

    def close(self) -> None:
        if self._holds:
            holds, self._holds = self._holds, []
            self._mgr._release(holds, self._owner)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class PathLockManager:
    """Multi-granularity path locks (the inode lock manager of the master)."""

    def __init__(self, timeout_s: float = 600.0):
        self._cond = threading.Condition(threading.Lock())
        # path -> {(mode, owner thread): count}
        self._held: dict[str, dict[tuple[str, int], int]] = {}
        self.timeout_s = timeout_s
        self.waits = 0            # acquisitions that had to wait (metrics / tests)

    @staticmethod
    def expand(requests) -> list[tuple[str, str]]:
        """[(path, R|W)] -> the (node, mode) holds: the mode on the path, intentions above."""
        holds = []
        for path, mode in requests:
            p = normalize_path(path)
            intent = _INTENT[mode]
            holds.extend((a, intent) for a in _ancestors(p))
            holds.append((p, mode))
        return holds

    def _conflicts(self, holds, me: int) -> bool:
        held = self._held
        for node, mode in holds:
            h = held.get(node)
            if not h:
                continue
            ok = _COMPAT[mode]
            for (m, owner) in h:
                if owner != me and m not in ok:
                    return True
        return False

    def lock(self, requests, timeout_s: float | None = None) -> LockList:
        """Acquire every request of ``[(path, "R"|"W")]`` atomically (blocks while any conflicts)."""
        holds = self.expand(requests)
        me = threading.get_ident()
        limit = self.timeout_s if timeout_s is None else timeout_s
        with self._cond:
            if self._conflicts(holds, me):
                if getattr(_LANE, "nb", False):
                    raise WouldBlock(f"namespace locks on {[p for p, _ in requests]} are held")
                self.waits += 1
                t_wait = time.monotonic()
                deadline = t_wait + limit
                while self._conflicts(holds, me):
                    rem = deadline - time.monotonic()
                    if rem <= 0:
                        raise DeadlineExceededException(
                            f"timed out after {limit:.0f}s waiting for namespace locks on "
                            f"{[p for p, _ in requests]}")
                    self._cond.wait(min(rem, 1.0))
                if optiming.ENABLED:
                    optiming.add("path_lock_wait", time.monotonic() - t_wait)
            held = self._held
            for node, mode in holds:
                h = held.get(node)
                if h is None:
                    h = held[node] = {}
                k = (mode, me)
                h[k] = h.get(k, 0) + 1
        return LockList(self, holds, me, [p for p, _ in requests])

    def _release(self, holds, owner: int) -> None:
        with self._cond:
            held = self._held
            for node, mode in holds:
                h = held.get(node)
                k = (mode, owner)
                c = h[k] - 1
                if c:
                    h[k] = c
                else:
                    del h[k]
                    if not h:
                        del held[node]
            self._cond.notify_all()

    def held_paths(self) -> dict:
        """Snapshot {path: [modes]} (diagnostics and tests)."""
        with self._cond:
            return {p: sorted(m for (m, _o) in h) for p, h in self._held.items()}
