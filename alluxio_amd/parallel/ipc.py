"""HIP IPC short-circuit reads of HBM blocks held by a same-node worker process.

The reference short-circuit path (core/server/worker/.../grpc/ShortCircuitBlockReadHandler.java,
core/client/fs/.../block/stream/LocalFileDataReader.java:58-70) gives a local client the block
file path to mmap.  On MI355X the block lives in a worker's HBM arena, so the worker exports the
arena allocation once as a HIP IPC handle (``OpenDeviceBlock`` returns handle + arena offset +
the block's page list, with the block read-locked); the client maps the arena into its own
address space and gathers the pages into its destination with the batched copy kernel running
on *its* GPU — over xGMI when the worker owns a different GPU of the node.  No bytes cross the
host or the RPC channel.
"""
from __future__ import annotations

import threading

from ..ops.native import lib


# Allocations this process exported: handle bytes -> allocation base.  HIP refuses to open a
# process's own IPC handle ("invalid device context"), and a same-process client needs no mapping.
_LOCAL_EXPORTS: dict[bytes, int] = {}


def export_handle(tensor) -> tuple[bytes, int]:
    """(IPC handle bytes, offset of the tensor's data inside the exported allocation)."""
    handle, offset, _ = lib().ipc_export(tensor.data_ptr())
    _LOCAL_EXPORTS[bytes(handle)] = tensor.data_ptr() - int(offset)
    return bytes(handle), int(offset)


OPEN_TIMEOUT_MS = [30_000]     # alluxio.user.short.circuit.open.timeout (set_open_timeout)


def set_open_timeout(ms: int) -> None:
    OPEN_TIMEOUT_MS[0] = max(1, int(ms))


class IpcMappings:
    """Per-process cache of opened arena mappings keyed by (handle bytes, device)."""

    def __init__(self):
        self._lock = threading.Lock()
        self._maps: dict[tuple[bytes, int], int] = {}

    def open(self, handle: bytes, device: int) -> int:
        key = (bytes(handle), device)
        local = _LOCAL_EXPORTS.get(key[0])
        if local is not None:
            return local
        with self._lock:
            base = self._maps.get(key)
            if base is None:
                # bounded: an import that never returns (seen on some arena sizes, see
                # worker/store.py) makes this handle unavailable instead of hanging the reader;
                # callers fall back to the worker's gRPC data port
                try:
                    base = lib().ipc_open_bounded(key[0], device, OPEN_TIMEOUT_MS[0])
                except TimeoutError as e:
                    from ..utils.exceptions import UnavailableException
                    raise UnavailableException(f"HIP IPC import of the worker arena timed out: {e}") from e
                self._maps[key] = base
            return base

    def close_all(self) -> None:
        with self._lock:
            for base in self._maps.values():
                lib().ipc_close(base)
            self._maps.clear()


MAPPINGS = IpcMappings()


# Shared DRAM arenas of THIS process: (pid, fd) -> base address (no self-mapping needed).
_LOCAL_SHARED: dict[tuple[int, int], int] = {}


def register_local_shared(fd: int, base: int) -> None:
    import os
    _LOCAL_SHARED[(os.getpid(), fd)] = base


class ShmMappings:
    """Per-process cache of shared DRAM arenas of other local worker processes, mapped through
    ``/proc/<pid>/fd/<fd>`` and page-locked for the GPU when one is present."""

    def __init__(self):
        self._lock = threading.Lock()
        self._maps: dict[tuple[int, int], tuple[object, int, bool]] = {}

    def open(self, pid: int, fd: int, nbytes: int) -> int:
        local = _LOCAL_SHARED.get((pid, fd))
        if local is not None:
            return local
        import ctypes
        import mmap
        import os
        with self._lock:
            got = self._maps.get((pid, fd))
            if got is not None:
                return got[1]
            f = os.open(f"/proc/{pid}/fd/{fd}", os.O_RDWR)
            try:
                mm = mmap.mmap(f, nbytes, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
            finally:
                os.close(f)
            base = ctypes.addressof(ctypes.c_char.from_buffer(mm))
            registered = bool(lib().host_register(base, nbytes)) if nbytes else False
            self._maps[(pid, fd)] = (mm, base, registered)
            return base

    def close_all(self) -> None:
        with self._lock:
            for mm, base, registered in self._maps.values():
                if registered:
                    lib().host_unregister(base)
            # ctypes views pin the mmap objects; they are released with the process
            self._maps.clear()


SHM = ShmMappings()


def map_handle(h, device: int) -> int:
    """Address, in this process, of the first byte of the arena a ``DeviceBlockHandle`` describes
    (page ``p`` of the block starts at ``base + p * page_size``).  HBM arenas are opened through
    HIP IPC on ``device`` (peer HBM is then read over xGMI by kernels on ``device``); shared DRAM
    arenas are mmap'ed.  Raises ``RuntimeError`` when the handle carries neither."""
    if getattr(h, "arena_kind", "") == "dram":
        if h.host_fd < 0:
            raise RuntimeError(f"block {h.block_id}: DRAM arena not shared")
        return SHM.open(h.pid, h.host_fd, h.arena_bytes) + h.arena_offset
    if not h.arena_ipc_handle:
        raise RuntimeError(f"block {h.block_id}: worker did not export an IPC handle")
    return MAPPINGS.open(h.arena_ipc_handle, device) + h.arena_offset


def page_segments(src_base: int, pages, page_size: int, offset: int, length: int, dst_ptr: int):
    """Copy segments (src, dst, bytes) for bytes [offset, offset+length) of a paged block,
    merging physically adjacent pages into one segment."""
    segs = []
    pos, end, dst = offset, offset + length, dst_ptr
    while pos < end:
        pi, po = divmod(pos, page_size)
        take = min(page_size - po, end - pos)
        src = src_base + pages[pi] * page_size + po
        if segs and segs[-1][0] + segs[-1][2] == src and segs[-1][1] + segs[-1][2] == dst:
            s = segs[-1]
            segs[-1] = (s[0], s[1], s[2] + take)
        else:
            segs.append((src, dst, take))
        pos += take
        dst += take
    return segs


def gather_block(handle_msg, offset: int, length: int, dst_ptr: int, device: int, stream: int = 0) -> int:
    """Copy part of a device block described by a ``DeviceBlockHandle`` into ``dst_ptr`` (device
    memory of ``device``) with one batched-copy launch; returns bytes copied."""
    if offset < 0 or offset + length > handle_msg.length:
        raise ValueError(f"range [{offset}, {offset + length}) outside block of {handle_msg.length} bytes")
    base = map_handle(handle_msg, device)
    segs = page_segments(base, list(handle_msg.pages), handle_msg.page_size, offset, length, dst_ptr)
    lib().batched_copy(segs, stream, True)
    return length


def verify_handle_crc(h, device: int) -> None:
    """Check a mapped block against the per-page CRC32Cs its worker computed at commit (the
    ``crc32c`` of a ``DeviceBlockHandle``): the CRC kernel runs on ``device`` over the mapped pages
    (peer HBM read over xGMI), a shared DRAM arena is checked on the host.  Raises
    ``DataLossException`` on a mismatch."""
    from ..ops.native import has_gpu, lib
    from ..utils.exceptions import DataLossException
    crcs = list(h.crc32c)
    if not crcs:
        return
    base = map_handle(h, device)
    ps, n = h.page_size, h.length
    C = lib()
    got = []
    for i, p in enumerate(h.pages):
        ln = min(ps, n - i * ps)
        if ln <= 0:
            break
        addr = base + int(p) * ps
        if h.arena_kind == "dram" or not has_gpu():
            got.append(C.crc32c_ptr(addr, ln, 0))
        else:
            import torch
            with torch.cuda.device(device):
                got.extend(C.crc32c_device(addr, ln, 0, 0))
    if got != crcs[:len(got)] or len(got) != len(crcs):
        raise DataLossException(f"block {h.block_id}: CRC32C mismatch on the shared pages")
