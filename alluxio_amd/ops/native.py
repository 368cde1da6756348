"""Loader for the native extension + error mapping + device helpers.

The extension is built in-tree (``alluxio_amd/_C*.so``); importing this module builds it if it is
missing or stale (hipcc cross-compiles for gfx950 without a GPU).  On a GPU box the HIP paths are
the ones that run: :func:`require_device` fails loudly instead of silently using a host fallback.
"""
from __future__ import annotations

import contextlib
import functools
import importlib
import os
import threading

from ..utils import exceptions as ex

_lock = threading.Lock()
_mod = None

ERR_NOT_FOUND = 1
ERR_ALREADY_EXISTS = 2
ERR_OUT_OF_SPACE = 3
ERR_INVALID_STATE = 4
ERR_HIP = 5
ERR_INVALID_ARGUMENT = 6
ERR_IO = 7
ERR_TIMEOUT = 8

_CODE_TO_EXC = {
    ERR_NOT_FOUND: ex.BlockDoesNotExistException,
    ERR_ALREADY_EXISTS: ex.BlockAlreadyExistsException,
    ERR_OUT_OF_SPACE: ex.WorkerOutOfSpaceException,
    ERR_INVALID_STATE: ex.InvalidWorkerStateException,
    ERR_HIP: ex.InternalException,
    ERR_INVALID_ARGUMENT: ex.InvalidArgumentException,
    ERR_IO: ex.UnavailableException,
    ERR_TIMEOUT: ex.DeadlineExceededException,
}


def lib():
    """The ``alluxio_amd._C`` module (built on first use)."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None:
            alt = os.environ.get("ALLUXIO_AMD_NATIVE_SO")   # e.g. a sanitizer build (tools/sanitize.sh)
            if os.environ.get("ALLUXIO_AMD_NO_BUILD") != "1" and not alt:
                from .build import build
                build()
            # One HIP runtime per process: load torch's libamdhip64 first so the extension binds
            # to the same runtime (same soname) instead of pulling a second copy from /opt/rocm.
            import torch  # noqa: F401
            if alt:
                import importlib.util as ilu
                import sys
                spec = ilu.spec_from_file_location("alluxio_amd._C", alt)
                _mod = ilu.module_from_spec(spec)
                sys.modules["alluxio_amd._C"] = _mod
                spec.loader.exec_module(_mod)
            else:
                _mod = importlib.import_module("alluxio_amd._C")
    return _mod


def translate(e: BaseException) -> BaseException:
    m = lib()
    if isinstance(e, m.StoreError) and len(e.args) >= 2:
        return _CODE_TO_EXC.get(e.args[0], ex.InternalException)(str(e.args[1]))
    return e


@contextlib.contextmanager
def native_errors():
    try:
        yield
    except Exception as e:  # noqa: BLE001
        m = lib()
        if isinstance(e, m.StoreError):
            raise translate(e) from None
        raise


def wrap_errors(fn):
    @functools.wraps(fn)
    def inner(*a, **kw):
        with native_errors():
            return fn(*a, **kw)
    return inner


_DEVICE_COUNT: int | None = None
_DEVICE_COUNT_LOCK = threading.Lock()


def device_count() -> int:
    """Number of visible HIP devices (0 on CPU-only hosts).  Computed once under a lock: the
    first query initialises the runtime (amdsmi), and threads racing into that first query could
    otherwise see a transient failure as "no GPU" (and, e.g., memcpy a device pointer on the host)."""
    global _DEVICE_COUNT
    n = _DEVICE_COUNT
    if n is not None:
        return n
    with _DEVICE_COUNT_LOCK:
        if _DEVICE_COUNT is None:
            count = 0
            try:
                import torch
                if torch.cuda.is_available():
                    count = torch.cuda.device_count()
            except Exception:  # noqa: BLE001
                count = 0
            _DEVICE_COUNT = count
        return _DEVICE_COUNT


def has_gpu() -> bool:
    return device_count() > 0


def require_device() -> None:
    if not has_gpu():
        raise RuntimeError("a HIP device is required for this operation (none visible)")


def current_stream_handle(device=None) -> int:
    import torch
    return int(torch.cuda.current_stream(device).cuda_stream)
