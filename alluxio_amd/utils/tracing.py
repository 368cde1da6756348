"""roctx ranges from Python (SURVEY 5.1 tracing / profiling).

``trace_range("phase")`` pushes a roctx range on the calling thread (through the native extension,
which links the ROCm roctx library); under ``rocprofv3 --marker-trace --kernel-trace`` the range
brackets the kernels and copies issued inside it.  The native store adds its own ranges
(``BlockStore.ingest_files``, ``BlockStore.free_space``, ...: csrc/trace.h).  Without a profiler
attached a range costs well under a microsecond; ``ALLUXIO_AMD_ROCTX=0`` turns the Python ranges off.
"""
from __future__ import annotations

import contextlib
import functools
import os

_ENABLED = os.environ.get("ALLUXIO_AMD_ROCTX", "1") != "0"


def enabled() -> bool:
    return _ENABLED


@contextlib.contextmanager
def trace_range(name: str):
    if not _ENABLED:
        yield
        return
    from ..ops.native import lib
    C = lib()
    C.trace_push(name)
    try:
        yield
    finally:
        C.trace_pop()


def traced(name: str):
    """Decorator form of :func:`trace_range`."""
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **kw):
            with trace_range(name):
                return fn(*a, **kw)
        return wrapper
    return deco


def mark(name: str) -> None:
    if _ENABLED:
        from ..ops.native import lib
        lib().trace_mark(name)
