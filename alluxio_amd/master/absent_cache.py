"""UFS absent-path cache.

Parity: core/server/master/src/main/java/alluxio/master/file/meta/AsyncUfsAbsentPathCache.java and
UfsAbsentPathCache.java -- a path that is in neither Alluxio nor the UFS is remembered, so repeated
lookups of missing paths (``getStatus`` with LoadMetadataType ONCE, the "ListStatus on a
non-existent file" case of docs/en/operation/Scalability-Tuning.md:148) answer "does not exist"
without a UFS round trip.  An entry also covers every path below it (a missing directory has no
children).  Entries are keyed by the mount id the path resolved to, so a remount under the same
Alluxio path invalidates them; creating or loading a path drops it and its ancestors; a metadata
sync drops everything under the synced path.  ``process_async`` records a miss on the
``alluxio.master.ufs.path.cache.threads`` pool, walking from the mount point down to the first
missing component, as the reference does; the capacity is an LRU bound
(``alluxio.master.ufs.path.cache.capacity``).
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import logging
import threading

LOG = logging.getLogger(__name__)


def _ancestors(path: str):
    """``path`` and its ancestors, deepest first (``/a/b`` -> ``/a/b``, ``/a``, ``/``)."""
    p = path.rstrip("/") or "/"
    while True:
        yield p
        if p == "/":
            return
        p = p.rsplit("/", 1)[0] or "/"


class AsyncUfsAbsentPathCache:
    def __init__(self, mount_table, capacity: int = 100_000, threads: int = 8):
        self.mount_table = mount_table
        self.capacity = max(1, capacity)
        self._entries: collections.OrderedDict = collections.OrderedDict()   # path -> mount id
        self._lock = threading.Lock()
        self._threads = max(1, threads)
        self._pool: cf.ThreadPoolExecutor | None = None
        self._pending: set = set()
        self.hits = 0
        self.misses = 0

    def _mount_id(self, path: str):
        try:
            return self.mount_table.resolve(path).mount_id
        except Exception:  # noqa: BLE001 - not under any mount
            return None

    # ---- queries ---------------------------------------------------------------------------
    def is_absent(self, path: str, exists=None) -> bool:
        """``exists(p)``: whether ``p`` is now in the Alluxio namespace -- an entry for a path
        that exists (a create or load raced with the miss that recorded it) is stale and dropped."""
        with self._lock:
            if not self._entries:
                self.misses += 1
                return False
            for p in _ancestors(path):
                mid = self._entries.get(p)
                if mid is None:
                    continue
                if mid != self._mount_id(p) or (exists is not None and exists(p)):
                    del self._entries[p]          # remounted since, or created since: stale
                    continue
                self._entries.move_to_end(p)
                self.hits += 1
                return True
            self.misses += 1
            return False

    def size(self) -> int:
        with self._lock:
            return len(self._entries)

    # ---- updates ---------------------------------------------------------------------------
    def add_single_path(self, path: str, mount_id=None) -> None:
        """Record ``path`` as absent under ``mount_id`` (the mount its UFS check resolved to;
        default: the current one) -- a check that raced with a remount records a stale id."""
        mid = self._mount_id(path) if mount_id is None else mount_id
        if mid is None:
            return
        with self._lock:
            self._entries[path.rstrip("/") or "/"] = mid
            self._entries.move_to_end(path.rstrip("/") or "/")
            while len(self._entries) > self.capacity:
                self._entries.popitem(last=False)

    def process_async(self, path: str) -> bool:
        """Record the shallowest missing component of ``path`` in the background; False when a
        check of this path is already queued."""
        with self._lock:
            if path in self._pending:
                return False
            self._pending.add(path)
            if self._pool is None:
                self._pool = cf.ThreadPoolExecutor(self._threads, thread_name_prefix="ufs-absent-path")
        self._pool.submit(self._process, path)
        return True

    def process_now(self, path: str) -> None:
        self._pending.add(path)
        self._process(path)

    def _process(self, path: str) -> None:
        try:
            chain = list(reversed(list(_ancestors(path))))      # shallowest first
            for p in chain:
                try:
                    res = self.mount_table.resolve(p)
                except Exception:  # noqa: BLE001
                    continue
                if self.mount_table.is_mount_point(p):
                    continue                                      # mount points always exist
                if res.ufs.get_status(res.uri) is None:
                    self.add_single_path(p, res.mount_id)
                    return
        except Exception:  # noqa: BLE001 - a failed check just leaves the path uncached
            LOG.debug("absent-path check of %s failed", path, exc_info=True)
        finally:
            with self._lock:
                self._pending.discard(path)

    def process_existence(self, path: str) -> None:
        """``path`` exists now: it and its ancestors are not absent."""
        with self._lock:
            if not self._entries:
                return
            for p in _ancestors(path):
                self._entries.pop(p, None)

    def invalidate_prefix(self, path: str) -> None:
        """Drop every entry at or below ``path`` (a metadata sync re-reads that subtree)."""
        root = path.rstrip("/") or "/"
        pre = root if root == "/" else root + "/"
        with self._lock:
            for p in [p for p in self._entries if p == root or p.startswith(pre)]:
                del self._entries[p]

    def clear(self) -> None:
        with self._lock:
            self._entries.clear()

    def close(self) -> None:
        if self._pool is not None:
            self._pool.shutdown(wait=False)
            self._pool = None
