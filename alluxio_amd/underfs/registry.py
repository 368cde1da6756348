"""UFS factory registry (reference UnderFileSystemFactoryRegistry.java:24,63-115 + ServiceLoader).

Factories register per scheme; third-party UFS plug in via ``register_factory`` or the
``alluxio_amd.underfs`` entry-point group.  ``create(uri)`` picks the first factory that
``supports`` the URI and configuration, like the reference's ``find`` over eligible factories.
"""
from __future__ import annotations

import threading

from .base import UnderFileSystem, UnderFileSystemWithLogging

_LOCK = threading.Lock()
_FACTORIES: list[tuple[str, object]] = []
_LOADED = False


class UnderFileSystemFactory:
    scheme = ""

    def supports(self, uri: str, conf=None) -> bool:
        return uri.startswith(self.scheme + "://") or (self.scheme == "file" and uri.startswith("/"))

    def create(self, uri: str, conf=None, properties=None) -> UnderFileSystem:  # pragma: no cover
        raise NotImplementedError


class _ClassFactory(UnderFileSystemFactory):
    def __init__(self, scheme: str, cls):
        self.scheme = scheme
        self.cls = cls

    def create(self, uri, conf=None, properties=None):
        return self.cls(uri, conf, properties)


def register_factory(factory: UnderFileSystemFactory, first: bool = False) -> None:
    with _LOCK:
        entry = (factory.scheme, factory)
        if first:
            _FACTORIES.insert(0, entry)
        else:
            _FACTORIES.append(entry)


def unregister_factory(factory: UnderFileSystemFactory) -> None:
    with _LOCK:
        _FACTORIES[:] = [e for e in _FACTORIES if e[1] is not factory]


def _load_builtin() -> None:
    global _LOADED
    if _LOADED:
        return
    _LOADED = True
    from .local import LocalUnderFileSystem
    from .memory import MemoryUnderFileSystem
    register_factory(_ClassFactory("file", LocalUnderFileSystem))
    register_factory(_ClassFactory("mem", MemoryUnderFileSystem))
    from . import s3, web, hdfs, swift, wasb, webhdfs, ozone  # noqa: F401  (self-registering)
    from .testing import SleepingUfsFactory
    register_factory(SleepingUfsFactory())
    from . import synthetic  # noqa: F401  (self-registering)
    try:
        from importlib.metadata import entry_points
        for ep in entry_points().select(group="alluxio_amd.underfs"):
            register_factory(ep.load()())
    except Exception:  # noqa: BLE001
        pass


def find(uri: str, conf=None) -> UnderFileSystemFactory | None:
    _load_builtin()
    with _LOCK:
        for _, f in _FACTORIES:
            if f.supports(uri, conf):
                return f
    return None


def create(uri: str, conf=None, properties=None, logging_wrapper: bool = False,
           metrics=None) -> UnderFileSystem:
    f = find(uri, conf)
    if f is None:
        raise ValueError(f"no under file system factory found for {uri!r}")
    ufs = f.create(uri, conf, properties)
    from .lz4frame import wrap
    ufs = wrap(ufs, properties, conf)
    return UnderFileSystemWithLogging(ufs, metrics) if logging_wrapper else ufs


def schemes() -> list[str]:
    _load_builtin()
    with _LOCK:
        return sorted({s for s, _ in _FACTORIES})
