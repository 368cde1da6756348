"""Tiered-store construction: configuration -> native page arenas.

Parity: worker tier layout keys ``alluxio.worker.tieredstore.level{N}.{alias,dirs.path,
dirs.quota,dirs.mediumtype}`` (core/common/.../PropertyKey.java:2933-2985, levels :3079),
BlockMetadataManager's tier/dir scan (core/server/worker/.../BlockMetadataManager.java:84-104).

Dir path grammar (comma separated, one quota per dir):
  ``hbm`` / ``hbm:<device>``   device arena on the worker's MI355X (medium HBM)
  ``dram``                     pinned host arena (medium DRAM; plain host memory without a GPU)
  ``auto``                     ``hbm`` when a HIP device is visible, else ``dram``
  ``/some/dir``                file-backed dir (SSD/HDD)
HBM arenas are one native ``hipMalloc`` each, DRAM arenas a shared-memory file; both are handed to
the native store as raw pointers and wrapped in zero-copy tensors that give page views for RCCL
transfers and HIP IPC export.
"""
from __future__ import annotations

import logging
import os
import weakref

from ..conf import Configuration, Templates
from ..ops.native import has_gpu, lib, wrap_errors

LOG = logging.getLogger(__name__)

ANNOTATORS = {"LRU": 0, "LRFU": 1}
ALLOCATORS = {"MAXFREE": 0, "GREEDY": 1, "ROUNDROBIN": 2}


class Arena:
    """A contiguous allocation backing one storage dir.

    ``hbm`` arenas are one device allocation, exported to same-node processes as a HIP IPC handle.
    ``dram`` arenas are an anonymous shared-memory file (``memfd``) mapped into the worker and
    page-locked for the GPU when one is present: a same-node client or peer worker maps the same
    pages through ``/proc/<worker pid>/fd/<fd>`` — the DRAM-tier analogue of the reference's
    short-circuit mmap of block files (LocalFileDataReader.java:58-70), with no bytes on the RPC
    channel.
    """

    def __init__(self, kind: str, nbytes: int, device: int = 0, alloc_bytes: int | None = None):
        import torch
        self.kind = kind
        self.nbytes = nbytes
        self.device = device
        self.fd = -1
        self._mmap = None
        self._registered = False
        if kind == "hbm":
            # One plain hipMalloc (csrc/ipc.cpp device_arena_alloc) of `alloc_bytes` (see
            # ipc_safe_size) whose first `nbytes` are the tier; the native store takes ownership
            # (DirSpec.owns_base) and frees it when it is destroyed, so no page it hands out
            # outlives the memory.
            self.alloc_bytes = max(alloc_bytes or nbytes, nbytes, 1)
            if os.environ.get("ALLUXIO_HBM_ARENA_TORCH") == "1":
                # A/B knob: the arena as a caching-allocator tensor (round-4 layout), kept alive
                # by this object instead of owned by the store
                self._dptr = None
                self._owner = torch.empty(self.alloc_bytes, dtype=torch.uint8,
                                          device=torch.device("cuda", device))
                self.tensor = self._owner[:nbytes]
            else:
                self._dptr = lib().device_arena_alloc(self.alloc_bytes, device)
                self.tensor = _device_tensor(self._dptr, nbytes, device)
        elif kind == "dram":
            self.tensor = self._shared_host(nbytes)
        else:
            raise ValueError(kind)
        self.base = self.tensor.data_ptr()

    def _shared_host(self, nbytes: int):
        import mmap

        import numpy as np
        import torch
        try:
            fd = os.memfd_create("alluxio-amd-dram", getattr(os, "MFD_CLOEXEC", 1))
            os.ftruncate(fd, max(nbytes, 1))
            mm = mmap.mmap(fd, max(nbytes, 1), mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        except (AttributeError, OSError):
            LOG.debug("memfd unavailable: private DRAM arena", exc_info=True)
            return torch.empty(nbytes, dtype=torch.uint8, pin_memory=has_gpu())
        self.fd, self._mmap = fd, mm
        t = torch.from_numpy(np.frombuffer(mm, dtype=np.uint8, count=nbytes))
        from ..parallel.ipc import register_local_shared
        register_local_shared(fd, t.data_ptr())
        if has_gpu() and nbytes:
            self._registered = bool(lib().host_register(t.data_ptr(), nbytes))
        # the memfd pins the memory until closed: release it with the arena even without close()
        self._finalizer = weakref.finalize(self, _release_shared, fd, t.data_ptr() if self._registered else 0)
        return t

    def prefault(self) -> None:
        """Populate the arena's pages in the background (MADV_POPULATE_WRITE, 64 MiB at a time,
        GIL released): the first write into a page of a shared-memory arena otherwise takes a
        fault that allocates and zeroes it, which caps the first fill of the tier at ~0.6 GB/s
        per stream on a VM.  A GPU host pins (hipHostRegister) -- and so populates -- the arena
        already."""
        if self._registered or self._mmap is None or not self.nbytes:
            return
        import ctypes
        import threading
        base, n = self.base, self.nbytes

        def run():
            libc = ctypes.CDLL(None, use_errno=True)
            step = 64 << 20
            for off in range(0, n, step):
                if self.fd < 0:
                    return                              # closed meanwhile
                if libc.madvise(ctypes.c_void_p(base + off), ctypes.c_size_t(min(step, n - off)), 23) != 0:
                    return                              # MADV_POPULATE_WRITE needs Linux 5.14+
        threading.Thread(target=run, name="dram-prefault", daemon=True).start()

    def share_handle(self) -> tuple[int, int] | None:
        """(pid, fd) through which another local process maps a shared DRAM arena, else None."""
        return (os.getpid(), self.fd) if self.fd >= 0 else None

    def close(self) -> None:
        fin = getattr(self, "_finalizer", None)
        if fin is not None:
            fin()
        self.fd = -1
        self._registered = False

    def view(self, offset: int, nbytes: int):
        return self.tensor[offset:offset + nbytes]

    def ipc_handle(self) -> tuple[bytes, int]:
        """(HIP IPC handle of the arena's allocation, arena offset inside it) — exported once
        and cached (short-circuit export to same-node processes)."""
        if self.kind != "hbm":
            raise ValueError("only device arenas can be exported over HIP IPC")
        if getattr(self, "_ipc", None) is None:
            from ..parallel.ipc import export_handle
            self._ipc = export_handle(self.tensor)
        return self._ipc


IPC_SIZE_BIT = 1 << 31


def ipc_safe_size(nbytes: int) -> int:
    """Allocation size for an HBM arena that other processes import through HIP IPC.

    Measured on MI355X (ROCm 7.2, dmabuf IPC): ``hipIpcOpenMemHandle`` in an importing process
    never returns when bit 31 of the allocation size is set (size mod 4 GiB >= 2 GiB) -- 3 / 6 /
    7 GiB allocations hang, 256 MiB / 5 / 8 / 9 GiB open at once -- for native hipMalloc arenas as
    for caching-allocator segments (profiles/r5_ipc_arena_sizes.md,
    tests/test_ipc_gpu.py::test_unpadded_arena_import_times_out).  The pattern fits a 32-bit
    signed size somewhere in the import path.  Such sizes are padded up to the next multiple of
    4 GiB; the padding is never handed out."""
    if nbytes & IPC_SIZE_BIT:
        return (nbytes + (4 << 30) - 1) // (4 << 30) * (4 << 30)
    return nbytes


class _DeviceBuffer:
    """__cuda_array_interface__ of a raw device allocation (a zero-copy torch view of it)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 2, "strides": None}


def _device_tensor(ptr: int, nbytes: int, device: int):
    import torch
    return torch.as_tensor(_DeviceBuffer(ptr, nbytes), device=torch.device("cuda", device))


def _release_shared(fd: int, registered_ptr: int) -> None:
    if registered_ptr:
        try:
            lib().host_unregister(registered_ptr)
        except Exception:  # noqa: BLE001
            pass
    try:
        os.close(fd)
    except OSError:
        pass


class DirConfig:
    def __init__(self, tier: int, alias: str, path: str, quota: int, medium: str):
        self.tier, self.alias, self.path, self.quota, self.medium = tier, alias, path, quota, medium


def _resolve_kind(path: str) -> tuple[str, int | None]:
    p = path.strip()
    if p == "auto":
        return ("hbm", None) if has_gpu() else ("dram", None)
    if p.startswith("hbm"):
        dev = p.split(":", 1)[1] if ":" in p else ""
        return "hbm", int(dev) if dev.isdigit() else None
    if p in ("dram", "mem", "ram"):
        return "dram", None
    return "file", None


def parse_tiers(conf: Configuration) -> list[DirConfig]:
    from ..utils.format import parse_space_size
    out = []
    for level in range(conf.get_int("alluxio.worker.tieredstore.levels")):
        alias = conf.get(Templates.WORKER_TIERED_STORE_LEVEL_ALIAS.format(level))
        paths = conf.get_list(Templates.WORKER_TIERED_STORE_LEVEL_DIRS_PATH.format(level))
        quotas = conf.get_list(Templates.WORKER_TIERED_STORE_LEVEL_DIRS_QUOTA.format(level))
        mediums = conf.get_list(Templates.WORKER_TIERED_STORE_LEVEL_DIRS_MEDIUMTYPE.format(level))
        for i, p in enumerate(paths):
            q = quotas[min(i, len(quotas) - 1)] if quotas else "1GB"
            kind, _ = _resolve_kind(p)
            medium = mediums[min(i, len(mediums) - 1)] if mediums else ""
            if kind == "hbm":
                medium = "HBM"
            elif kind == "dram":
                medium = "DRAM" if medium in ("", "HBM") else medium
            out.append(DirConfig(level, alias, p, parse_space_size(q), medium or "SSD"))
    return out


class TieredStore:
    """Owns the arenas and the native :class:`BlockStore` of one worker."""

    def __init__(self, conf: Configuration, device: int | None = None, work_dir: str | None = None):
        C = lib()
        self.conf = conf
        self.device = device if device is not None else _default_device(conf)
        page = conf.get_bytes("alluxio.worker.hbm.page.size")
        frac = conf.get_float("alluxio.worker.hbm.arena.fraction")
        self.dirs = parse_tiers(conf)
        self.arenas: list[Arena | None] = []
        specs = []
        self.tier_aliases: list[str] = []
        for d in self.dirs:
            kind, dev = _resolve_kind(d.path)
            spec = C.DirSpec()
            spec.tier = d.tier
            spec.tier_alias = d.alias
            spec.medium = d.medium
            spec.page_size = page
            spec.device = self.device if dev is None else dev
            quota = d.quota
            if kind == "hbm":
                if not has_gpu():
                    raise RuntimeError(f"tier {d.alias} dir {d.path!r} needs a HIP device but none is visible")
                if frac > 0:
                    import torch
                    free, _ = torch.cuda.mem_get_info(spec.device)
                    quota = int(free * frac)
                    if quota & IPC_SIZE_BIT:
                        # a share of free memory has no room for IPC padding: round the tier
                        # down to the largest importable size instead (< 2 GiB less)
                        quota = (quota & ~((4 << 30) - 1)) + IPC_SIZE_BIT - page
                quota -= quota % page
                alloc = ipc_safe_size(quota)
                if alloc != quota:
                    LOG.warning("HBM tier %s: %d bytes allocated for a %d-byte arena (%d padding bytes, "
                                "never used: HIP IPC cannot import sizes with bit 31 set)",
                                d.alias, alloc, quota, alloc - quota)
                arena = Arena("hbm", quota, spec.device, alloc)
                spec.kind = C.DirKind.DEVICE
                spec.base = arena.base
                spec.owns_base = arena._dptr is not None
            elif kind == "dram":
                quota -= quota % page
                arena = Arena("dram", quota)
                if conf.get_bool("alluxio.worker.tieredstore.dram.prefault", "false"):
                    arena.prefault()
                spec.kind = C.DirKind.HOST
                spec.base = arena.base
            else:
                arena = None
                path = d.path
                if work_dir and not os.path.isabs(path):
                    path = os.path.join(work_dir, path)
                os.makedirs(path, exist_ok=True)
                spec.kind = C.DirKind.FILE
                spec.path = path
            spec.capacity = quota
            specs.append(spec)
            self.arenas.append(arena)
            if d.alias not in self.tier_aliases:
                self.tier_aliases.append(d.alias)
        # multi-tier stores keep align.reserved.bytes (at most a quarter) of every dir free for
        # tier-management swaps (the reference's reserved space, AllocateOptions.useReservedSpace)
        if len({d.tier for d in self.dirs}) > 1 and (
                conf.get_bool("alluxio.worker.management.tier.align.enabled")
                or conf.get_bool("alluxio.worker.management.tier.promote.enabled")
                or conf.get_bool("alluxio.worker.management.tier.swap.restore.enabled")):
            want = conf.get_bytes("alluxio.worker.management.tier.align.reserved.bytes")
            for spec in specs:
                r = min(want, spec.capacity // 4)
                spec.reserved = r - r % page if spec.kind != C.DirKind.FILE else r
        annot = conf.get("alluxio.worker.block.annotator.class").rsplit(".", 1)[-1].replace("Annotator", "").upper()
        alloc = conf.get("alluxio.worker.allocator.class").rsplit(".", 1)[-1].replace("Allocator", "").upper()
        self.native = C.BlockStore(specs, ANNOTATORS.get(annot, 0), ALLOCATORS.get(alloc, 0),
                                   conf.get_float("alluxio.worker.block.annotator.lrfu.step.factor"),
                                   conf.get_float("alluxio.worker.block.annotator.lrfu.attenuation.factor"),
                                   self.device)
        self.has_device_tier = any(a is not None and a.kind == "hbm" for a in self.arenas)
        self.native.set_use_device_evict(conf.get_bool("alluxio.worker.eviction.device.enabled", "true"))
        self.native.set_demote_on_evict(conf.get_bool("alluxio.worker.tieredstore.eviction.demote", "true"))
        # TieredBlockStore.allocateSpace frees size + free.ahead.bytes when it has to evict.  With an
        # HBM tier one eviction round frees at least alluxio.worker.hbm.evict.batch.bytes (capped at
        # 1/32 of the smallest HBM dir): the device radix select then runs once per batch of
        # creates instead of once per create (16 writers, 64 MiB blocks: CACHE_THROUGH 21.2 ->
        # 24.1 GB/s, profiles/r6_free_ahead.md)
        ahead = conf.get_bytes("alluxio.worker.tieredstore.free.ahead.bytes", "0")
        hbm_caps = [sp.capacity for sp, a in zip(specs, self.arenas) if a is not None and a.kind == "hbm"]
        if hbm_caps:
            batch = conf.get_bytes("alluxio.worker.hbm.evict.batch.bytes", "1GB")
            ahead = max(ahead, min(batch, min(hbm_caps) // 32))
        self.native.set_free_ahead(ahead)
        self.native.set_use_device_alloc(conf.get_bool("alluxio.worker.hbm.device.alloc.enabled", "true"),
                                         conf.get_int("alluxio.worker.hbm.device.alloc.min.pages", "1024"))
        LOG.info("tiered store: %s", self.native.stats())

    def arena_for_dir(self, d: int) -> Arena | None:
        return self.arenas[d]

    def dir_medium(self, d: int) -> str:
        return self.dirs[d].medium

    def tier_of_alias(self, alias: str) -> int:
        for d in self.dirs:
            if d.alias == alias:
                return d.tier
        return -1

    def capacity_by_tier(self) -> dict[str, int]:
        out: dict[str, int] = {}
        for i, d in enumerate(self.dirs):
            out[d.alias] = out.get(d.alias, 0) + self.native.dir_capacity(i)
        return out

    def used_by_tier(self) -> dict[str, int]:
        out: dict[str, int] = {}
        for i, d in enumerate(self.dirs):
            used = self.native.dir_capacity(i) - self.native.dir_available(i)
            out[d.alias] = out.get(d.alias, 0) + used
        return out

    @wrap_errors
    def block_view(self, block_id: int):
        """Device/host tensor views of the block's page runs (for RCCL send / zero-copy reads)."""
        pages, d, ps, base = self.native.block_pages(block_id)
        info = self.native.block_info(block_id)
        arena = self.arenas[d]
        if arena is None:
            raise ValueError("block lives in a file tier; no memory view")
        views = []
        i = 0
        remaining = info.length
        while i < len(pages) and remaining > 0:
            j = i + 1
            while j < len(pages) and pages[j] == pages[j - 1] + 1:
                j += 1
            n = min((j - i) * ps, remaining)
            views.append(arena.view(pages[i] * ps, n))
            remaining -= n
            i = j
        return views


def _default_device(conf: Configuration) -> int:
    d = conf.get_int("alluxio.worker.gpu.device")
    if d >= 0:
        return d
    lr = os.environ.get("LOCAL_RANK")
    if lr is not None and has_gpu():
        import torch
        return int(lr) % max(1, torch.cuda.device_count())
    return 0
