"""Small concurrent collections used by the masters.

``IndexedSet`` is the multi-index set the reference's BlockMaster keeps its worker sets in
(core/base/src/main/java/alluxio/collections/IndexedSet.java): objects are retrievable by any
of several declared field indexes (unique or non-unique).
"""
from __future__ import annotations

import threading
from collections import defaultdict


class IndexedSet:
    def __init__(self, **indexes):
        """``IndexedSet(id=(lambda w: w.id, True), address=(lambda w: w.address, True))``."""
        self._lock = threading.RLock()
        self._items: set[int] = set()
        self._objs: dict[int, object] = {}
        self._idx = {}
        for name, (fn, unique) in indexes.items():
            self._idx[name] = (fn, unique, {} if unique else defaultdict(set))

    def add(self, obj) -> bool:
        with self._lock:
            key = id(obj)
            if key in self._items:
                return False
            for name, (fn, unique, table) in self._idx.items():
                v = fn(obj)
                if unique and v in table:
                    return False
            self._items.add(key)
            self._objs[key] = obj
            for name, (fn, unique, table) in self._idx.items():
                v = fn(obj)
                if unique:
                    table[v] = obj
                else:
                    table[v].add(key)
            return True

    def remove(self, obj) -> bool:
        with self._lock:
            key = id(obj)
            if key not in self._items:
                return False
            self._items.discard(key)
            self._objs.pop(key, None)
            for name, (fn, unique, table) in self._idx.items():
                v = fn(obj)
                if unique:
                    if table.get(v) is obj:
                        table.pop(v, None)
                else:
                    s = table.get(v)
                    if s is not None:
                        s.discard(key)
                        if not s:
                            table.pop(v, None)
            return True

    def get_first_by_field(self, index: str, value):
        with self._lock:
            fn, unique, table = self._idx[index]
            if unique:
                return table.get(value)
            keys = table.get(value)
            if not keys:
                return None
            return self._objs[next(iter(keys))]

    def get_by_field(self, index: str, value) -> list:
        with self._lock:
            fn, unique, table = self._idx[index]
            if unique:
                o = table.get(value)
                return [o] if o is not None else []
            return [self._objs[k] for k in table.get(value, ())]

    def contains_field(self, index: str, value) -> bool:
        with self._lock:
            return value in self._idx[index][2]

    def remove_by_field(self, index: str, value) -> int:
        n = 0
        for o in self.get_by_field(index, value):
            n += self.remove(o)
        return n

    def __iter__(self):
        with self._lock:
            return iter(list(self._objs.values()))

    def __len__(self) -> int:
        with self._lock:
            return len(self._items)

    def clear(self) -> None:
        with self._lock:
            self._items.clear()
            self._objs.clear()
            for name, (fn, unique, table) in self._idx.items():
                table.clear()


class ConcurrentHashSet:
    def __init__(self, it=()):
        self._s = set(it)
        self._lock = threading.Lock()

    def add(self, x):
        with self._lock:
            self._s.add(x)

    def discard(self, x):
        with self._lock:
            self._s.discard(x)

    def __contains__(self, x):
        with self._lock:
            return x in self._s

    def snapshot(self) -> set:
        with self._lock:
            return set(self._s)

    def __len__(self):
        with self._lock:
            return len(self._s)
