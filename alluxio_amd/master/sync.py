"""Parallel metadata sync: :class:`UfsStatusCache` and :class:`InodeSyncStream`.

Parity:
- core/server/master/src/main/java/alluxio/master/file/meta/UfsStatusCache.java -- per-sync cache
  of UFS statuses and directory listings; ``prefetchChildren`` submits listings to the prefetch
  pool (``alluxio.master.metadata.sync.ufs.prefetch.pool.size``) ahead of the sync that needs them,
  ``fetchChildrenIfAbsent`` joins an in-flight prefetch instead of listing twice, and a child's
  status comes out of its parent's listing instead of a per-path ``getStatus``.
- core/server/master/src/main/java/alluxio/master/file/InodeSyncStream.java -- a sync of a path
  processes pending paths breadth-first with up to ``alluxio.master.metadata.sync.concurrency.level``
  paths in flight on the sync executor (``alluxio.master.metadata.sync.executor.pool.size``),
  prefetching the listings of the next paths while the current ones reconcile; each path
  reconciles the Alluxio inode against its UFS status (load / delete / reload on fingerprint
  change) and a directory queues its sub-directories.

UFS round trips (list, status) run on pool threads with the namespace lock released, so a sync of a
wide tree on an object store overlaps its listing latency; inode mutations still take the tree
write lock once per directory batch (one journal context per batch).
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import logging
import threading

LOG = logging.getLogger(__name__)


def _join(parent: str, name: str) -> str:
    return parent.rstrip("/") + "/" + name


class UfsStatusCache:
    """Statuses and listings fetched during one sync; ``fetch_list(path)`` / ``fetch_status(path)``
    do the UFS calls for an Alluxio path."""

    def __init__(self, fetch_list, fetch_status, pool: cf.Executor | None = None):
        self._fetch_list = fetch_list
        self._fetch_status = fetch_status
        self._pool = pool
        self._lock = threading.Lock()
        self._status: dict = {}            # alluxio path -> UfsStatus | None
        self._children: dict = {}          # alluxio path -> list[UfsStatus] | None (None: not a dir)
        self._pending: dict = {}           # alluxio path -> Future of the listing
        self.ufs_list_calls = 0
        self.ufs_status_calls = 0

    # ---- statuses ----------------------------------------------------------------------------
    def add_status(self, path: str, st) -> None:
        with self._lock:
            self._status[path] = st

    def get_status(self, path: str):
        """The status from a parent's listing when one was fetched, else one UFS call."""
        with self._lock:
            if path in self._status:
                return self._status[path]
        self.ufs_status_calls += 1
        st = self._fetch_status(path)
        with self._lock:
            self._status.setdefault(path, st)
        return st

    def has_status(self, path: str) -> bool:
        with self._lock:
            return path in self._status

    # ---- listings ----------------------------------------------------------------------------
    def _list(self, path: str):
        self.ufs_list_calls += 1
        try:
            return self._fetch_list(path)
        except Exception:  # noqa: BLE001 - a vanished/unreadable directory syncs as absent
            LOG.debug("listing %s failed", path, exc_info=True)
            return None

    def prefetch_children(self, path: str) -> None:
        if self._pool is None:
            return
        with self._lock:
            if path in self._children or path in self._pending:
                return
            self._pending[path] = self._pool.submit(self._list, path)

    def fetch_children(self, path: str):
        """Listing of ``path`` (joining an in-flight prefetch); child statuses enter the cache."""
        with self._lock:
            if path in self._children:
                return self._children[path]
            fut = self._pending.get(path)
        listing = fut.result() if fut is not None else self._list(path)
        with self._lock:
            self._pending.pop(path, None)
            self._children[path] = listing
            for st in listing or ():
                if st.name and "/" not in st.name:
                    self._status.setdefault(_join(path, st.name), st)
        return listing

    def remove(self, path: str) -> None:
        with self._lock:
            self._status.pop(path, None)
            self._children.pop(path, None)

    def cancel(self) -> None:
        with self._lock:
            for f in self._pending.values():
                f.cancel()
            self._pending.clear()


class InodeSyncStream:
    """One metadata sync of ``root`` (recursively when asked) against the UFS."""

    def __init__(self, fsm, root: str, recursive: bool, executor: cf.Executor | None,
                 prefetch_pool: cf.Executor | None, concurrency: int = 6):
        self.fsm = fsm
        self.root = root
        self.recursive = recursive
        self.executor = executor
        self.concurrency = max(1, concurrency)
        self.cache = UfsStatusCache(self._ufs_list, self._ufs_status, prefetch_pool)
        self.stats = {"added": 0, "removed": 0, "updated": 0, "synced_paths": 0}
        self._stats_lock = threading.Lock()

    # ---- UFS access for an Alluxio path --------------------------------------------------------
    def _ufs_list(self, path: str):
        res = self.fsm._resolve_ufs(path)
        return res.ufs.list_status(res.uri)

    def _ufs_status(self, path: str):
        res = self.fsm._resolve_ufs(path)
        return res.ufs.get_status(res.uri)

    def _bump(self, key: str, n: int = 1) -> None:
        with self._stats_lock:
            self.stats[key] += n

    # ---- driver ------------------------------------------------------------------------------
    def run(self) -> dict:
        from ..utils.exceptions import InvalidPathException
        try:
            self.fsm._resolve_ufs(self.root)
        except InvalidPathException:
            return self._result()
        pending = collections.deque([self.root])
        try:
            while pending:
                wave = [pending.popleft() for _ in range(min(self.concurrency, len(pending)))]
                # listings of this wave and the next one go out together; the reconcile of a path
                # then finds its listing fetched (or joins the in-flight fetch)
                for p in wave + list(pending)[: self.concurrency]:
                    self.cache.prefetch_children(p)
                if self.executor is None or len(wave) == 1:
                    results = [self._sync_path(p) for p in wave]
                else:
                    results = [f.result() for f in [self.executor.submit(self._sync_path, p) for p in wave]]
                for subdirs in results:
                    pending.extend(subdirs)
        finally:
            self.cache.cancel()
        return self._result()

    def _result(self) -> dict:
        out = dict(self.stats)
        out["ufs_list_calls"] = self.cache.ufs_list_calls
        out["ufs_status_calls"] = self.cache.ufs_status_calls
        return out

    # ---- one path ----------------------------------------------------------------------------
    def _sync_path(self, path: str) -> list[str]:
        """Reconcile ``path``; returns the sub-directories to sync next."""
        from ..underfs.base import Fingerprint
        fsm, tree = self.fsm, self.fsm.tree
        self._bump("synced_paths")
        st = self.cache.get_status(path)
        with tree.lock.read():
            inode = tree.get_or_none(path)
        if st is None:
            if inode is not None and inode.is_persisted and path != "/":
                fsm.delete(path, recursive=True, alluxio_only=True)
                self._bump("removed")
            return []
        if inode is None:
            fsm.load_metadata(path, recursive=False, create_ancestors=True, quiet=True, cache=self.cache)
            self._bump("added")
            return self._subdirs(path) if st.is_directory and self.recursive else []
        if inode.is_file:
            if self._changed(inode, st, path, Fingerprint):
                fsm.delete(path, alluxio_only=True)
                fsm.load_metadata(path, quiet=True, cache=self.cache)
                self._bump("updated")
            return []
        listing = self.cache.fetch_children(path)
        if listing is None:
            return []
        by_name = {s.name: s for s in listing if s.name and "/" not in s.name}
        with tree.lock.read():
            kids = {c.name: c for c in tree.list_children(inode)}
        for name, c in kids.items():
            cp = _join(path, name)
            s = by_name.get(name)
            if s is None:
                if c.is_persisted and not fsm.mount_table.is_mount_point(cp):
                    fsm.delete(cp, recursive=True, alluxio_only=True)
                    self._bump("removed")
            elif c.is_file and c.is_persisted and self._changed(c, s, cp, Fingerprint):
                fsm.delete(cp, alluxio_only=True)
                fsm.load_metadata(cp, quiet=True, cache=self.cache)
                self._bump("updated")
            elif c.is_directory != s.is_directory and c.is_persisted:
                fsm.delete(cp, recursive=True, alluxio_only=True)
                fsm.load_metadata(cp, quiet=True, cache=self.cache)
                self._bump("updated")
        new = [s for n, s in by_name.items() if n not in kids]
        if new:
            fsm.load_listed_children(path, new)
            self._bump("added", len(new))
        if not self.recursive:
            return []
        return [_join(path, n) for n, s in by_name.items() if s.is_directory]

    def _subdirs(self, path: str) -> list[str]:
        listing = self.cache.fetch_children(path) or []
        return [_join(path, s.name) for s in listing if s.is_directory and s.name and "/" not in s.name]

    def _changed(self, inode, st, path: str, Fingerprint) -> bool:
        if not inode.is_persisted:
            return False
        if st.is_file and not getattr(st, "content_hash", "") and self.cache.has_status(path):
            # a listing entry without a content hash (some object stores): ask for the full status
            self.cache.remove(path)
            st = self.cache.get_status(path)
            if st is None:
                return True
        res = self.fsm._resolve_ufs(path)
        fp = Fingerprint.create(res.ufs.ufs_type, st)
        old = Fingerprint.parse(inode.ufs_fingerprint)
        return old is None or not fp.matches_content(old)
