"""Client-side local page cache.

Parity: core/client/fs/src/main/java/alluxio/client/file/cache/ — LocalCacheManager.java:75-360
(page-granular cache: get/put/delete, two-phase evict-then-put under striped page locks,
restore of a LOCAL store's pages on restart, async put), PageStore.java + store/LocalPageStore.java
(``<dir>/<page size>/<bucket>/<file id>/<page index>`` files), store/RocksPageStore.java,
MetaStore.java / DefaultMetaStore.java (page index + bytes), evictor/{LRU,LFU}CacheEvictor.java,
LocalCacheFileInStream.java (read through the cache: hit -> copy, miss -> read the whole page
from the external stream, put, copy) and LocalCacheFileSystem.java (wraps openFile).

Store types: ``LOCAL`` (files, survives restarts), ``MEM`` (host memory) and the MI355X ``HBM``
store — a fixed-page device arena; a cache hit for a device destination is a D2D copy and a
multi-page read into a GPU tensor is gathered by one batched-copy launch.
"""
from __future__ import annotations

import collections
import io
import logging
import math
import os
import threading
import zlib

from .. import metrics as msys

LOG = logging.getLogger(__name__)


class PageId(tuple):
    __slots__ = ()

    def __new__(cls, file_id: str, page_index: int):
        return super().__new__(cls, (str(file_id), int(page_index)))

    @property
    def file_id(self):
        return self[0]

    @property
    def page_index(self):
        return self[1]


# ---- evictors ---------------------------------------------------------------------------------
class LRUCacheEvictor:
    def __init__(self, conf=None):
        self._d: collections.OrderedDict = collections.OrderedDict()

    def update_on_get(self, pid):
        if pid in self._d:
            self._d.move_to_end(pid)

    def update_on_put(self, pid):
        self._d[pid] = True
        self._d.move_to_end(pid)

    def update_on_delete(self, pid):
        self._d.pop(pid, None)

    def evict(self):
        return next(iter(self._d), None)


class LFUCacheEvictor:
    """Buckets by floor(log_base(count)) (LFUCacheEvictor.java); LRU within a bucket."""

    def __init__(self, conf=None):
        self.base = float(conf.get("alluxio.user.client.cache.evictor.lfu.logbase")) if conf else 2.0
        self._count: dict = {}
        self._buckets: dict[int, collections.OrderedDict] = collections.defaultdict(collections.OrderedDict)

    def _bucket(self, n):
        return int(math.log(n, self.base)) if n > 0 else 0

    def _touch(self, pid, delta):
        old = self._count.get(pid)
        if old is not None:
            self._buckets[self._bucket(old)].pop(pid, None)
        n = (old or 0) + delta
        self._count[pid] = n
        self._buckets[self._bucket(n)][pid] = True

    def update_on_get(self, pid):
        if pid in self._count:
            self._touch(pid, 1)

    def update_on_put(self, pid):
        self._touch(pid, 1)

    def update_on_delete(self, pid):
        n = self._count.pop(pid, None)
        if n is not None:
            self._buckets[self._bucket(n)].pop(pid, None)

    def evict(self):
        for b in sorted(self._buckets):
            if self._buckets[b]:
                return next(iter(self._buckets[b]))
        return None


# ---- page stores ------------------------------------------------------------------------------
class LocalPageStore:
    """One file per page: ``<root>/<page_size>/<bucket>/<file_id>/<page_index>``."""

    OPTIONS_FILE = "options.pb"

    def __init__(self, root: str, page_size: int, buckets: int = 1000, cache_size: int = 0):
        self.root = os.path.join(root, str(page_size))
        self.buckets = buckets
        os.makedirs(self.root, exist_ok=True)
        self._check_options(page_size, cache_size)

    def _check_options(self, page_size: int, cache_size: int) -> None:
        """Store-wide options (proto/client/cache.proto PPageStoreCommonOptions): a store written
        with a different page size or by another version is discarded instead of restored."""
        from .. import __version__
        from ..proto import pb
        want = pb.client_cache.PPageStoreCommonOptions(pageSize=page_size, cacheSize=cache_size,
                                                      alluxioVersion=__version__)
        path = os.path.join(self.root, self.OPTIONS_FILE)
        if os.path.exists(path):
            with open(path, "rb") as f:
                have = pb.client_cache.PPageStoreCommonOptions.FromString(f.read())
            if have.pageSize == want.pageSize and have.alluxioVersion == want.alluxioVersion:
                return
            import shutil
            for n in os.listdir(self.root):
                q = os.path.join(self.root, n)
                shutil.rmtree(q) if os.path.isdir(q) else os.remove(q)
        with open(path, "wb") as f:
            f.write(want.SerializeToString())

    def _path(self, pid):
        b = zlib.crc32(pid.file_id.encode()) % self.buckets  # stable across processes (restore)
        return os.path.join(self.root, str(b), pid.file_id, str(pid.page_index))

    def put(self, pid, data: bytes) -> None:
        p = self._path(pid)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        tmp = p + ".tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, p)

    def get(self, pid, offset: int, length: int) -> bytes | None:
        try:
            with open(self._path(pid), "rb") as f:
                f.seek(offset)
                return f.read(length)
        except FileNotFoundError:
            return None

    def delete(self, pid) -> None:
        try:
            os.remove(self._path(pid))
        except FileNotFoundError:
            pass

    def restore(self):
        """[(PageId, bytes)] of pages already on disk (LocalCacheManager restore)."""
        out = []
        for b in os.listdir(self.root):
            bdir = os.path.join(self.root, b)
            if not os.path.isdir(bdir):
                continue
            for fid in os.listdir(bdir):
                for name in os.listdir(os.path.join(bdir, fid)):
                    if name.endswith(".tmp"):
                        continue
                    p = os.path.join(bdir, fid, name)
                    out.append((PageId(fid, int(name)), os.path.getsize(p)))
        return out


class MemPageStore:
    def __init__(self):
        self._d: dict = {}

    def put(self, pid, data: bytes) -> None:
        self._d[pid] = bytes(data)

    def get(self, pid, offset, length):
        d = self._d.get(pid)
        return None if d is None else d[offset:offset + length]

    def delete(self, pid) -> None:
        self._d.pop(pid, None)

    def restore(self):
        return []


class HbmPageStore:
    """Fixed page slots in one HBM arena, indexed by the native device hash table (K9).

    Backed by ``_C.PageCache`` (csrc/page_cache.{h,cpp}): page ``(file_id, index)`` has the key
    ``(interned file id << 24) | index``.  The open-addressing table keeps an authoritative host
    mirror plus a device copy probed by ``page_lookup_gather_kernel`` (csrc/kernels.hip), so a batch
    of pages whose keys are computed ON the GPU (a device-side sampler) is resolved and copied by
    one launch (:meth:`gather`) with no host round trip.  Pages shorter than the page size can use
    up the slots before the manager's byte budget does: the native store then evicts its least
    recently used pages (host gets and device gathers both count as uses) and reports them through
    ``on_evict`` so the manager's metastore stays exact.  Without a HIP device the same table and
    arena live in host memory (CPU builds and tests).
    """

    INDEX_BITS = 24

    def __init__(self, capacity: int, page_size: int, device=None, use_device: bool | None = None):
        from ..ops.native import has_gpu, lib
        self.page_size = page_size
        self.use_device = has_gpu() if use_device is None else bool(use_device)
        self.device = None
        dev = 0
        if self.use_device:
            import torch
            self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
            dev = self.device.index
        self.cache = lib().PageCache(dev, max(1, capacity // page_size) * page_size, page_size, self.use_device)
        self.slots = self.cache.slots
        self._fid: dict = {}
        self._fname: list = []
        self._lock = threading.Lock()
        self.on_evict = None

    def file_key(self, file_id) -> int:
        file_id = str(file_id)
        k = self._fid.get(file_id)
        if k is None:
            with self._lock:
                k = self._fid.get(file_id)
                if k is None:
                    k = len(self._fname)
                    self._fname.append(file_id)
                    self._fid[file_id] = k
        return k

    def key(self, pid) -> int:
        if not 0 <= pid.page_index < (1 << self.INDEX_BITS):
            raise ValueError(f"page index {pid.page_index} does not fit an HBM page key")
        return (self.file_key(pid.file_id) << self.INDEX_BITS) | pid.page_index

    def pid_of(self, key: int):
        return PageId(self._fname[key >> self.INDEX_BITS], key & ((1 << self.INDEX_BITS) - 1))

    def _stream(self) -> int:
        if not self.use_device:
            return 0
        import torch
        return int(torch.cuda.current_stream(self.device).cuda_stream)

    def put(self, pid, data) -> None:
        k = self.key(pid)
        if hasattr(data, "data_ptr"):
            import torch
            t = data.contiguous().view(-1).view(torch.uint8)
            if t.is_cuda and self.use_device:
                evicted = self.cache.put(k, t.data_ptr(), t.numel(), 1, self._stream(), True)
            else:
                evicted = self.cache.put_bytes(k, t.cpu().numpy(), True)
        else:
            evicted = self.cache.put_bytes(k, data, True)
        if self.on_evict is not None:
            for e in evicted:
                self.on_evict(self.pid_of(e))

    def ptr(self, pid, offset):
        slot, _ = self.cache.lookup(self.key(pid))
        return None if slot < 0 else self.cache.slot_ptr(slot) + offset

    def read_segments(self, pids, offsets, lengths, dsts, on_device: bool = True):
        """Copy ``lengths[i]`` bytes at ``offsets[i]`` of page ``pids[i]`` to address ``dsts[i]``
        (device memory when ``on_device``, else host), one batched launch on the current stream.
        Returns the indices that missed; their destinations are untouched."""
        keys = [self.key(p) for p in pids]
        kind = 1 if (on_device and self.use_device) else 0
        return list(self.cache.read_segments(keys, list(offsets), list(lengths), list(dsts), kind,
                                             self._stream()))

    def get(self, pid, offset, length):
        k = self.key(pid)
        slot, n = self.cache.lookup(k)
        if slot < 0:
            return None
        if offset >= n:
            return b""
        return self.cache.get_bytes(k, offset, min(length, n - offset))

    def delete(self, pid) -> None:
        self.cache.erase(self.key(pid))

    def restore(self):
        return []

    def gather(self, file_id, page_indices, out):
        """Fused lookup + copy of whole pages ``page_indices`` (integer tensor; on the GPU for a
        device store) of ``file_id`` into the rows of ``out`` (uint8 ``[n, >= page_size]``, where
        the store lives).  One kernel launch, no host sync.  Returns int32 tensors ``(slots,
        lens)``; slot -1 / len 0 marks a miss (that row is left untouched)."""
        import torch
        keys = (page_indices.reshape(-1).to(torch.int64) | (self.file_key(file_id) << self.INDEX_BITS)).contiguous()
        n = keys.numel()
        if out.dim() != 2 or out.dtype != torch.uint8 or out.stride(1) != 1 or out.shape[0] < n \
                or out.shape[1] < self.page_size:
            raise ValueError("out must be a uint8 [n, >= page_size] tensor with contiguous rows")
        if keys.is_cuda != self.use_device or out.is_cuda != self.use_device:
            raise ValueError("page indices and out must live where the page store does")
        slots = torch.empty(n, dtype=torch.int32, device=keys.device)
        lens = torch.empty_like(slots)
        if n:
            self.cache.gather(keys.data_ptr(), n, out.data_ptr(), out.stride(0), slots.data_ptr(),
                              lens.data_ptr(), self._stream())
        return slots, lens


# ---- manager ----------------------------------------------------------------------------------
class LocalCacheManager:
    LOCKS = 1024

    def __init__(self, conf, store=None):
        from ..utils.format import parse_space_size
        self.conf = conf
        self.page_size = parse_space_size(conf.get("alluxio.user.client.cache.page.size"))
        self.capacity = parse_space_size(conf.get("alluxio.user.client.cache.size"))
        ev = conf.get("alluxio.user.client.cache.evictor.class").rsplit(".", 1)[-1]
        self.evictor = LFUCacheEvictor(conf) if ev.startswith("LFU") else LRUCacheEvictor(conf)
        stype = conf.get("alluxio.user.client.cache.store.type").upper()
        if store is not None:
            self.store = store
        elif stype == "HBM":
            self.store = HbmPageStore(self.capacity, self.page_size)
        elif stype == "MEM":
            self.store = MemPageStore()
        else:
            self.store = LocalPageStore(conf.get("alluxio.user.client.cache.dir"), self.page_size,
                                        conf.get_int("alluxio.user.client.cache.local.store.file.buckets"),
                                        self.capacity)
        self.meta: dict = {}   # PageId -> bytes
        self.bytes = 0
        self._meta_lock = threading.RLock()
        self._page_locks = [threading.RLock() for _ in range(self.LOCKS)]
        self.metrics = msys.metrics("Client")
        if hasattr(self.store, "on_evict"):
            self.store.on_evict = self._on_store_evict
        for pid, n in self.store.restore():
            if self.bytes + n > self.capacity:
                self.store.delete(pid)
                continue
            self.meta[pid] = n
            self.bytes += n
            self.evictor.update_on_put(pid)

    def _lock(self, pid):
        return self._page_locks[hash(pid) % self.LOCKS]

    def put(self, pid, data) -> bool:
        n = len(data)
        if n > self.page_size:
            return False
        with self._lock(pid):
            with self._meta_lock:
                if pid in self.meta:
                    return True
                # phase 1: evict until the page fits
                while self.bytes + n > self.capacity:
                    victim = self.evictor.evict()
                    if victim is None:
                        return False
                    self._delete_locked(victim)
                    self.metrics.counter("ClientCachePagesEvicted").inc()
            # phase 2: store + index
            try:
                self.store.put(pid, data)
            except Exception:  # noqa: BLE001
                LOG.debug("page store put failed", exc_info=True)
                return False
            with self._meta_lock:
                self.meta[pid] = n
                self.bytes += n
                self.evictor.update_on_put(pid)
            self.metrics.counter("ClientCacheBytesWrittenCache").inc(n)
            return True

    def get(self, pid, offset: int, length: int) -> bytes | None:
        with self._lock(pid):
            with self._meta_lock:
                if pid not in self.meta:
                    self.metrics.counter("ClientCacheBytesRequestedExternal").inc(length)
                    return None
                self.evictor.update_on_get(pid)
            out = self.store.get(pid, offset, length)
        if out is not None:
            self.metrics.counter("ClientCacheBytesReadCache").inc(len(out))
        return out

    def _delete_locked(self, pid) -> None:
        n = self.meta.pop(pid, None)
        if n is None:
            return
        self.bytes -= n
        self.evictor.update_on_delete(pid)
        self.store.delete(pid)

    def delete(self, pid) -> bool:
        with self._lock(pid), self._meta_lock:
            had = pid in self.meta
            self._delete_locked(pid)
            return had

    def _on_store_evict(self, pid) -> None:
        """The store dropped ``pid`` by itself (HBM slot pressure): forget it here too."""
        with self._meta_lock:
            n = self.meta.pop(pid, None)
            if n is None:
                return
            self.bytes -= n
            self.evictor.update_on_delete(pid)
        self.metrics.counter("ClientCachePagesEvicted").inc()

    def gather(self, file_id, page_indices, out):
        """Batched page read from the HBM store: one fused hash-lookup + copy launch for pages
        whose indices may be computed on the GPU (see :meth:`HbmPageStore.gather`)."""
        if not hasattr(self.store, "gather"):
            raise ValueError("batched page gather needs the HBM page store")
        return self.store.gather(file_id, page_indices, out)

    def has(self, pid) -> bool:
        with self._meta_lock:
            return pid in self.meta


class LocalCacheFileInStream(io.RawIOBase):
    """Positioned/sequential reads served page-wise from the local cache, filling misses from
    the external (Alluxio) stream a whole page at a time.  Same read API as FileInStream."""

    def __init__(self, status, open_external, cache: LocalCacheManager):
        super().__init__()
        self.status = status
        self.length = status.length
        self.cache = cache
        self._open_external = open_external
        self._ext = None
        self.pos = 0
        self.file_id = f"{status.fileId}-{status.lastModificationTimeMs}"

    def _external(self):
        if self._ext is None:
            self._ext = self._open_external()
        return self._ext

    def _page(self, idx: int, off: int, n: int) -> bytes:
        pid = PageId(self.file_id, idx)
        got = self.cache.get(pid, off, n)
        if got is not None:
            return got
        ps = self.cache.page_size
        start = idx * ps
        ext = self._external()
        ext.seek(start)
        page = ext.read(min(ps, self.length - start))
        self.cache.put(pid, page)
        return page[off:off + n]

    def pread_bytes(self, position: int, size: int) -> bytes:
        size = max(0, min(size, self.length - position))
        ps = self.cache.page_size
        out = []
        done = 0
        while done < size:
            p = position + done
            idx, off = divmod(p, ps)
            take = min(size - done, ps - off)
            out.append(self._page(idx, off, take))
            done += take
        return b"".join(out)

    def readable(self):
        return True

    def seekable(self):
        return True

    def read(self, size: int = -1) -> bytes:
        if size is None or size < 0:
            size = self.length - self.pos
        data = self.pread_bytes(self.pos, size)
        self.pos += len(data)
        return data

    def readall(self):
        return self.read(-1)

    def readinto(self, b) -> int:
        mv = memoryview(b).cast("B")
        data = self.read(len(mv))
        mv[:len(data)] = data
        return len(data)

    def pread(self, position: int, buf, nbytes: int | None = None) -> int:
        mv = memoryview(buf).cast("B") if not hasattr(buf, "data_ptr") else None
        if mv is None:
            import numpy as np
            import torch
            n = buf.numel() * buf.element_size() if nbytes is None else nbytes
            data = self.pread_bytes(position, n)
            buf.view(torch.uint8)[:len(data)].copy_(torch.from_numpy(np.frombuffer(data, dtype=np.uint8)))
            return len(data)
        data = self.pread_bytes(position, len(mv) if nbytes is None else nbytes)
        mv[:len(data)] = data
        return len(data)

    def read_into(self, tensor) -> int:
        """Fill a (device) tensor from the current position.  Cached HBM pages are copied by the
        native store in one batched launch per group of pages: slots are resolved and the copy
        queued under the store lock, so no concurrent put can recycle a slot before its bytes were
        read.  Missing pages are fetched and cached first, a group at a time (a group is capped at
        a quarter of the cache, so a read longer than the cache still works); a page evicted
        between fill and copy is served through the byte path."""
        import numpy as np
        import torch
        n = min(tensor.numel() * tensor.element_size(), self.length - self.pos)
        store = self.cache.store
        flat = tensor.view(-1).view(torch.uint8) if tensor.is_contiguous() else None
        if flat is None or not (tensor.is_cuda and isinstance(store, HbmPageStore)):
            data = self.read(n)
            tensor.view(torch.uint8).view(-1)[:len(data)].copy_(torch.from_numpy(np.frombuffer(data, dtype=np.uint8)))
            return len(data)
        ps = self.cache.page_size
        group = max(1, store.slots // 4)
        dst = flat.data_ptr()
        done = 0
        while done < n:
            pieces = []                      # (page index, offset in page, bytes, dst offset)
            while done < n and len(pieces) < group:
                p = self.pos + done
                idx, off = divmod(p, ps)
                take = min(n - done, ps - off)
                pieces.append((idx, off, take, done))
                done += take
            for idx, _, _, _ in pieces:
                pid = PageId(self.file_id, idx)
                if not self.cache.has(pid):
                    self._page(idx, 0, 0)   # fetch + put
            missed = store.read_segments([PageId(self.file_id, i) for i, _, _, _ in pieces],
                                         [o for _, o, _, _ in pieces], [t for _, _, t, _ in pieces],
                                         [dst + d for _, _, _, d in pieces])
            hit = set(range(len(pieces))) - set(missed)
            for j in hit:
                self.cache.evictor.update_on_get(PageId(self.file_id, pieces[j][0]))
            for j in missed:                 # evicted meanwhile: byte path for this page
                idx, off, take, d = pieces[j]
                chunk = self._page(idx, off, take)
                flat[d:d + len(chunk)].copy_(torch.from_numpy(np.frombuffer(chunk, dtype=np.uint8)))
        self.pos += n
        return n

    def read_pages(self, page_indices, out, fill_misses: bool = True):
        """Read whole pages ``page_indices`` (integer tensor, e.g. drawn by a sampler on the GPU)
        into the rows of ``out`` with one fused hash-lookup + gather launch on the HBM page store.
        With ``fill_misses`` (one host sync) pages that missed are read through the external
        stream, cached and gathered again; without it the call never waits and misses keep
        length 0.  Returns the valid bytes of every row (int32 tensor)."""
        import torch
        slots, lens = self.cache.gather(self.file_id, page_indices, out)
        if not fill_misses:
            return lens
        miss = (slots < 0).nonzero().flatten()
        if miss.numel() == 0:
            return lens
        idx = page_indices.reshape(-1).to(torch.int64)[miss]
        ps = self.cache.page_size
        for p in sorted(set(idx.cpu().tolist())):
            if 0 <= p and p * ps < self.length:
                self._page(p, 0, 0)
        tmp = torch.zeros((idx.numel(), ps), dtype=torch.uint8, device=out.device)
        _, got = self.cache.gather(self.file_id, idx, tmp)
        out[miss, :ps] = tmp
        lens[miss] = got
        return lens

    def seek(self, pos: int, whence: int = 0) -> int:
        self.pos = {0: pos, 1: self.pos + pos, 2: self.length + pos}[whence]
        return self.pos

    def tell(self) -> int:
        return self.pos

    def close(self) -> None:
        if not self.closed and self._ext is not None:
            self._ext.close()
        super().close()
