"""Inode metastores: HEAP (all inodes as objects) and ROCKS (disk-backed with an object cache).

Parity: core/server/master/src/main/java/alluxio/master/metastore/InodeStore.java:51-180 (the
SPI the inode tree uses), heap/HeapInodeStore.java, rocks/RocksInodeStore.java (inodes serialised
into an embedded KV store so the namespace can exceed the heap) and caching/CachingInodeStore.java
(write-back object cache with high/low water marks).  RocksDB is not available in this image, so
the ROCKS store is built on the stdlib's embedded SQLite (WAL, ``synchronous=OFF``: durability comes
from the journal, exactly like the reference's RocksDB metastore which is rebuilt from the journal).

Consistency model: every namespace mutation goes through ``InodeTree.apply(entry)``; the tree opens
a tracking scope around it and the store writes back every inode touched in that scope when it
closes (write-through per journal entry).  The object cache is therefore never the only copy of a
mutation, so evicting an entry is always safe; outside apply, objects are read-only views.
Directory edges (parent -> name -> child) stay in memory (small next to the inodes).
"""
from __future__ import annotations

import collections
import os
import sqlite3
import threading
from collections.abc import MutableMapping

from ..proto import pb


def _serialize(inode) -> tuple[int, bytes]:
    e = inode.to_entry()
    kind = 1 if inode.is_directory else 0
    inner = e.inode_directory if kind else e.inode_file
    return kind, inner.SerializeToString()


def _deserialize(kind: int, data: bytes):
    from .inode import InodeDirectory, InodeFile
    if kind:
        return InodeDirectory.from_entry(pb.journal.InodeDirectoryEntry.FromString(data))
    return InodeFile.from_entry(pb.journal.InodeFileEntry.FromString(data))


class HeapInodeStore(dict):
    """The default: a plain dict (tracking scopes are no-ops)."""

    kind = "HEAP"

    def begin(self) -> None:
        pass

    def end(self) -> None:
        pass

    def flush(self) -> None:
        pass

    def close(self) -> None:
        pass


class CachingSqliteInodeStore(MutableMapping):
    kind = "ROCKS"

    def __init__(self, path: str, cache_size: int = 100_000):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        self.path = path
        self.cache_size = max(16, cache_size)
        self._db = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._db.execute("PRAGMA synchronous=OFF")
        self._db.execute("CREATE TABLE IF NOT EXISTS inodes (id INTEGER PRIMARY KEY, kind INTEGER, data BLOB)")
        self._cache: collections.OrderedDict = collections.OrderedDict()
        self._lock = threading.RLock()
        self._tracking = 0
        self._touched: dict[int, object] = {}
        self.loads = 0
        self.writes = 0

    # ---- tracking scope (one journal entry) ----------------------------------------------------
    def begin(self) -> None:
        with self._lock:
            self._tracking += 1

    def end(self) -> None:
        with self._lock:
            self._tracking -= 1
            if self._tracking:
                return
            touched, self._touched = self._touched, {}
            rows = [(i, *_serialize(o)) for i, o in touched.items() if i in self._cache]
            if rows:
                self._db.executemany("INSERT OR REPLACE INTO inodes (id, kind, data) VALUES (?, ?, ?)", rows)
                self.writes += len(rows)
            self._evict()

    def _track(self, key, obj) -> None:
        if self._tracking:
            self._touched[key] = obj

    def _evict(self) -> None:
        while len(self._cache) > self.cache_size:
            k, _ = self._cache.popitem(last=False)
            self._touched.pop(k, None)

    # ---- mapping ------------------------------------------------------------------------------
    def _load(self, key):
        row = self._db.execute("SELECT kind, data FROM inodes WHERE id = ?", (key,)).fetchone()
        if row is None:
            return None
        self.loads += 1
        obj = _deserialize(row[0], row[1])
        self._cache[key] = obj
        if not self._tracking:
            self._evict()
        return obj

    def __getitem__(self, key):
        with self._lock:
            obj = self._cache.get(key)
            if obj is not None:
                self._cache.move_to_end(key)
            else:
                obj = self._load(key)
                if obj is None:
                    raise KeyError(key)
            self._track(key, obj)
            return obj

    def get(self, key, default=None):
        try:
            return self[key]
        except KeyError:
            return default

    def __setitem__(self, key, obj) -> None:
        with self._lock:
            self._cache[key] = obj
            self._cache.move_to_end(key)
            if self._tracking:
                self._touched[key] = obj
            else:
                self._db.execute("INSERT OR REPLACE INTO inodes (id, kind, data) VALUES (?, ?, ?)",
                                 (key, *_serialize(obj)))
                self.writes += 1
                self._evict()

    def __delitem__(self, key) -> None:
        with self._lock:
            self._cache.pop(key, None)
            self._touched.pop(key, None)
            self._db.execute("DELETE FROM inodes WHERE id = ?", (key,))

    def pop(self, key, *default):
        with self._lock:
            obj = self.get(key)
            if obj is None:
                if default:
                    return default[0]
                raise KeyError(key)
            del self[key]
            return obj

    def __contains__(self, key) -> bool:
        with self._lock:
            if key in self._cache:
                return True
            return self._db.execute("SELECT 1 FROM inodes WHERE id = ?", (key,)).fetchone() is not None

    def __len__(self) -> int:
        with self._lock:
            self.flush()
            return self._db.execute("SELECT COUNT(*) FROM inodes").fetchone()[0]

    def __iter__(self):
        with self._lock:
            self.flush()
            ids = [r[0] for r in self._db.execute("SELECT id FROM inodes ORDER BY id")]
        return iter(ids)

    def values(self):
        for k in list(iter(self)):
            v = self.get(k)
            if v is not None:
                yield v

    def items(self):
        for k in list(iter(self)):
            v = self.get(k)
            if v is not None:
                yield k, v

    def clear(self) -> None:
        with self._lock:
            self._cache.clear()
            self._touched.clear()
            self._db.execute("DELETE FROM inodes")

    def flush(self) -> None:
        """Write every cached object (objects are write-through already; this covers callers
        that mutated outside a tracking scope)."""
        with self._lock:
            rows = [(i, *_serialize(o)) for i, o in self._cache.items()]
            if rows:
                self._db.executemany("INSERT OR REPLACE INTO inodes (id, kind, data) VALUES (?, ?, ?)", rows)

    def close(self) -> None:
        with self._lock:
            self.flush()
            self._db.close()


def create_inode_store(conf):
    kind = (conf.get("alluxio.master.metastore", "HEAP") if conf is not None else "HEAP").upper()
    if kind == "ROCKS":
        d = conf.get("alluxio.master.metastore.dir")
        cache = conf.get_int("alluxio.master.metastore.inode.cache.max.size")
        return CachingSqliteInodeStore(os.path.join(d, "inodes.sqlite"), min(cache, 1_000_000))
    return HeapInodeStore()
