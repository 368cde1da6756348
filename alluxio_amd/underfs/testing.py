"""Fault-injection UFS wrappers for tests.

Parity: tests/src/test/java/alluxio/testutils/underfs/delegating/DelegatingUnderFileSystem.java
(delegate everything, override selectively), sleeping/SleepingUnderFileSystem.java (inject
latency per op) and the flaky UFS used by FlakyUfsIntegrationTest.java:51-80 (fail a fraction of
deletes).  Register them under their own scheme with :func:`install`.
"""
from __future__ import annotations

import random
import time

from .base import UnderFileSystem
from .registry import UnderFileSystemFactory, register_factory, unregister_factory


class DelegatingUnderFileSystem(UnderFileSystem):
    def __init__(self, delegate: UnderFileSystem):
        super().__init__(delegate.root_uri, delegate.conf, delegate.properties)
        self.delegate = delegate
        self.scheme = delegate.scheme
        self.ufs_type = delegate.ufs_type

    def __getattr__(self, item):
        return getattr(self.delegate, item)

    def create(self, path, options=None):
        return self.delegate.create(path, options)

    def open(self, path, options=None):
        return self.delegate.open(path, options)

    def delete_file(self, path):
        return self.delegate.delete_file(path)

    def delete_directory(self, path, options=None):
        return self.delegate.delete_directory(path, options)

    def get_status(self, path):
        return self.delegate.get_status(path)

    def list_status(self, path, options=None):
        return self.delegate.list_status(path, options)

    def mkdirs(self, path, options=None):
        return self.delegate.mkdirs(path, options)

    def rename_file(self, src, dst):
        return self.delegate.rename_file(src, dst)

    def rename_directory(self, src, dst):
        return self.delegate.rename_directory(src, dst)


class SleepingUnderFileSystem(DelegatingUnderFileSystem):
    """Adds ``sleep_ms[op]`` before each named operation."""

    def __init__(self, delegate, sleep_ms: dict[str, float]):
        super().__init__(delegate)
        self.sleep_ms = sleep_ms

    def _nap(self, op):
        ms = self.sleep_ms.get(op, 0)
        if ms:
            time.sleep(ms / 1000.0)

    def create(self, path, options=None):
        self._nap("create")
        return super().create(path, options)

    def open(self, path, options=None):
        self._nap("open")
        return super().open(path, options)

    def get_status(self, path):
        self._nap("get_status")
        return super().get_status(path)

    def list_status(self, path, options=None):
        self._nap("list_status")
        return super().list_status(path, options)

    def delete_file(self, path):
        self._nap("delete_file")
        return super().delete_file(path)

    def mkdirs(self, path, options=None):
        self._nap("mkdirs")
        return super().mkdirs(path, options)

    def delete_directory(self, path, options=None):
        self._nap("delete_directory")
        return super().delete_directory(path, options)

    def rename_file(self, src, dst):
        self._nap("rename_file")
        return super().rename_file(src, dst)

    def rename_directory(self, src, dst):
        self._nap("rename_directory")
        return super().rename_directory(src, dst)

    def exists(self, path):
        self._nap("exists")
        return self.delegate.exists(path)

    def get_fingerprint(self, path):
        self._nap("get_fingerprint")
        return self.delegate.get_fingerprint(path)

    def set_owner(self, path, owner, group):
        self._nap("set_owner")
        return self.delegate.set_owner(path, owner, group)

    def set_mode(self, path, mode):
        self._nap("set_mode")
        return self.delegate.set_mode(path, mode)


SLEEP_OPS = ("create", "open", "get_status", "list_status", "delete_file", "delete_directory", "mkdirs",
             "rename_file", "rename_directory", "exists", "get_fingerprint", "set_owner", "set_mode")


class SleepingUfsFactory(UnderFileSystemFactory):
    """``sleepfs:///<local path>``: a local UFS behind :class:`SleepingUnderFileSystem`, so a
    master in another process can be given a slow UFS by configuration alone (reference
    SleepingUnderFileSystemFactory).  Latency per op: mount property or configuration key
    ``alluxio.underfs.sleep.<op>.ms``, default ``alluxio.underfs.sleep.ms`` (0)."""

    scheme = "sleepfs"

    def create(self, uri, conf=None, properties=None):
        from .local import LocalUnderFileSystem
        props = dict(properties or {})

        def get(key, default="0"):
            if key in props:
                return props[key]
            if conf is not None and conf.get_raw(key) is not None:
                return conf.get_raw(key)
            return default
        base = float(get("alluxio.underfs.sleep.ms"))
        sleep = {op: float(get(f"alluxio.underfs.sleep.{op}.ms", str(base))) for op in SLEEP_OPS}
        local = "/" + uri.split("://", 1)[1].lstrip("/")
        ufs = SleepingUnderFileSystem(LocalUnderFileSystem(local, conf, properties), sleep)
        ufs.root_uri = uri
        return ufs


class FlakyUnderFileSystem(DelegatingUnderFileSystem):
    """Fails ``rate`` of the listed operations with an IOError (seeded, reproducible)."""

    def __init__(self, delegate, ops=("delete_file",), rate: float = 0.5, seed: int = 0):
        super().__init__(delegate)
        self.ops = set(ops)
        self.rate = rate
        self.rng = random.Random(seed)

    def _maybe_fail(self, op):
        if op in self.ops and self.rng.random() < self.rate:
            raise OSError(f"injected failure in {op}")

    def delete_file(self, path):
        self._maybe_fail("delete_file")
        return super().delete_file(path)

    def create(self, path, options=None):
        self._maybe_fail("create")
        return super().create(path, options)

    def open(self, path, options=None):
        self._maybe_fail("open")
        return super().open(path, options)

    def rename_file(self, src, dst):
        self._maybe_fail("rename_file")
        return super().rename_file(src, dst)


class _WrapFactory(UnderFileSystemFactory):
    def __init__(self, scheme, inner_scheme_factory, wrapper):
        self.scheme = scheme
        self._inner = inner_scheme_factory
        self._wrap = wrapper

    def create(self, uri, conf=None, properties=None):
        from . import registry
        inner_uri = uri.replace(self.scheme + "://", self._inner + "://", 1)
        if self._inner == "file":
            inner_uri = uri.split("://", 1)[1]
            inner_uri = "/" + inner_uri.lstrip("/")
        return self._wrap(registry.create(inner_uri, conf, properties))


def install(scheme: str, inner: str, wrapper):
    """Register ``scheme://`` URIs as ``wrapper(<inner-scheme UFS>)``; returns an uninstaller."""
    f = _WrapFactory(scheme, inner, wrapper)
    register_factory(f, first=True)
    return lambda: unregister_factory(f)
