"""Training-input integration: HBM-cached datasets gathered straight into GPU batches.

The reference serves ML input pipelines through its POSIX (FUSE) and Hadoop clients — a trainer
opens files and issues small reads, one syscall / RPC per record.  On MI355X the dataset's blocks
sit in the worker's HBM arena, so a whole batch of records (random indices, spanning block
boundaries) is planned on the host and moved by ONE page-gather kernel launch into a
``[batch, record_bytes]`` device tensor, on a side stream, double-buffered so the next batch is in
flight while the model consumes the current one:

* worker in this process  -> ``BlockStore.read_batch`` (native planner + gather kernel);
* worker in another process on this node -> HIP IPC mapping of its arena (held for the loader's
  lifetime) + the batched copy kernel on this GPU (over xGMI when the worker owns another GPU);
* anything else -> the regular client stream per record (host path).

``FixedRecordDataset`` is the map-style view (``torch.utils.data.Dataset``) for code that wants
per-sample access; ``DeviceBatchLoader`` is the fast path.
"""
from __future__ import annotations

import numpy as np

from ..utils import ids
from ..utils.tracing import traced


class _FileLayout:
    """Path, length and block layout of one file; the BlockInfo list is materialised on first use
    (a 1 M-file listing must not pay for 1 M sub-message wrappers it may never touch)."""

    __slots__ = ("info", "path", "length", "block_size", "_blocks")

    def __init__(self, status):
        i = status.info
        self.info = i
        self.path = i.path
        self.length = i.length
        self.block_size = i.blockSizeBytes
        self._blocks = None

    @property
    def blocks(self):
        if self._blocks is None:
            self._blocks = [fbi.blockInfo for fbi in self.info.fileBlockInfos]
        return self._blocks

    @property
    def block_ids(self):
        return self.info.blockIds


class _LazyLayouts:
    """``files`` of a columnar listing: the _FileLayout of entry i is parsed on first access."""

    def __init__(self, cols, keep):
        self._cols, self._keep = cols, keep
        self._cache: dict = {}

    def __len__(self) -> int:
        return len(self._keep)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        lay = self._cache.get(i)
        if lay is None:
            lay = self._cache[i] = _FileLayout(self._cols.status(int(self._keep[i])))
        return lay

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


class FixedRecordDataset:
    """Records of ``record_bytes`` laid end to end across one or more files."""

    def __init__(self, fs, paths, record_bytes: int, dtype="uint8", shape=None, device=None):
        import torch
        self.fs = fs
        self.record_bytes = record_bytes
        self.dtype = getattr(torch, str(dtype)) if isinstance(dtype, str) else dtype
        self.shape = tuple(shape) if shape else None
        self.device = device
        self.files = [_FileLayout(fs.get_status(p)) for p in ([paths] if isinstance(paths, str) else paths)]
        self.counts = [f.length // record_bytes for f in self.files]
        self.starts = np.cumsum([0] + self.counts)

    def __len__(self):
        return int(self.starts[-1])

    def locate(self, idx: int) -> tuple[int, int]:
        """(file index, byte offset) of record ``idx``."""
        if idx < 0:
            idx += len(self)
        if not 0 <= idx < len(self):
            raise IndexError(idx)
        f = int(np.searchsorted(self.starts, idx, side="right") - 1)
        return f, (idx - int(self.starts[f])) * self.record_bytes

    def _view(self, raw):
        t = raw.view(self.dtype)
        return t.view(self.shape) if self.shape else t

    def __getitem__(self, idx):
        import torch
        f, off = self.locate(idx)
        out = torch.empty(self.record_bytes, dtype=torch.uint8, device=self.device)
        with self.fs.open_file(self.files[f].path) as s:
            s.pread(off, out)
        return self._view(out)


class FileListDataset(FixedRecordDataset):
    """One record per file of a directory (BASELINE config 4: ImageNet-shaped 128 KB files), with
    the metadata of every file from ONE ``listStatus`` (batched metadata: no per-file getStatus;
    the FileInfos carry their block ids and locations).  Files longer than ``record_bytes`` are
    truncated, shorter ones zero-padded (``lengths`` keeps the true sizes)."""

    def __init__(self, fs, directory: str, record_bytes: int | None = None, dtype="uint8", shape=None,
                 device=None):
        import torch
        self.fs = fs
        self.dtype = getattr(torch, str(dtype)) if isinstance(dtype, str) else dtype
        self.shape = tuple(shape) if shape else None
        self.device = device
        cols = fs.list_status_columns(directory) if hasattr(fs, "list_status_columns") else None
        if cols is None:
            sts = sorted((s for s in fs.list_status(directory) if not s.is_folder), key=lambda s: s.path)
            self.paths = [s.path for s in sts]
            self.lengths = np.array([s.length for s in sts], dtype=np.uint64)
            self.files = [_FileLayout(s) for s in sts]
            nblocks = np.array([len(f.block_ids) for f in self.files], dtype=np.int64)
            bsizes = np.array([f.block_size for f in self.files], dtype=np.int64)
            self.block_ids = np.array([f.block_ids[0] if len(f.block_ids) else -1 for f in self.files], dtype=np.int64)
        else:
            # columnar listing: no per-file Python objects until a file's layout is needed
            keep = np.nonzero(cols.folder == 0)[0]
            paths = [cols.paths[i] for i in keep]
            if any(paths[k] > paths[k + 1] for k in range(len(paths) - 1)):
                order = sorted(range(len(paths)), key=paths.__getitem__)
                keep, paths = keep[order], [paths[k] for k in order]
            self.paths = paths
            self.lengths = cols.lengths[keep].astype(np.uint64)
            self.files = _LazyLayouts(cols, keep)
            nblocks, bsizes = cols.nblocks[keep], cols.block_sizes[keep]
            self.block_ids = cols.first_blocks[keep].astype(np.int64)
        n = len(self.paths)
        self.record_bytes = int(record_bytes or (self.lengths.max() if n else 0))
        self.counts = [1] * n
        self.starts = np.arange(n + 1)
        # single-block records: the gather plan is a vector op over these arrays
        self.single_block = bool(np.all(nblocks == 1)) and bool(np.all(bsizes >= self.record_bytes))
        self.read_lengths = np.minimum(self.lengths, np.uint64(self.record_bytes))

    def locate(self, idx: int) -> tuple[int, int]:
        if idx < 0:
            idx += len(self)
        if not 0 <= idx < len(self):
            raise IndexError(idx)
        return idx, 0


class DeviceBatchLoader:
    """Iterates ``[batch, *shape]`` device tensors of records gathered by one kernel per batch."""

    def __init__(self, dataset: FixedRecordDataset, batch_size: int, shuffle: bool = False, seed: int = 0,
                 drop_last: bool = False, device=None, prefetch: int = 2):
        import torch
        self.ds = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.prefetch = max(1, prefetch)
        self.epoch = 0
        self._sources = None
        self.session = ids.create_session_id()
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None

    # ---- sources ------------------------------------------------------------------------------
    def _open_sources(self):
        """Per block: ('local', worker) | ('ipc', DeviceBlockHandle, base) | ('stream', None)."""
        if self._sources is not None:
            return self._sources
        ctx = self.ds.fs.ctx
        src = {}
        self._locks = []
        for f in self.ds.files:
            for b in f.blocks:
                chosen = ("stream", None)
                for loc in b.locations:
                    w = ctx.in_process_worker(loc.workerAddress)
                    if w is not None:
                        self._locks.append((w, w.lock_block(self.session, b.blockId)))
                        chosen = ("local", w)
                        break
                # same-node holder: map its arena (HBM via HIP IPC, DRAM via shared memory) and
                # gather with the copy kernel (host memcpy without a GPU)
                from ..ops.native import has_gpu
                if chosen[0] == "stream" and (self.device.type == "cuda" or not has_gpu()):
                    for loc in b.locations:
                        if not ctx.is_local(loc.workerAddress):
                            continue
                        try:
                            from ..client.context import worker_address_str
                            from ..parallel.ipc import map_handle
                            from ..proto import pb
                            stub = ctx.worker_stub(worker_address_str(loc.workerAddress))
                            h = stub.OpenDeviceBlock(pb.block.OpenDeviceBlockRequest(block_id=b.blockId,
                                                                                     session_id=self.session))
                            try:
                                base = map_handle(h, self.device.index or 0)
                            except Exception:
                                stub.UnlockDeviceBlock(pb.block.UnlockDeviceBlockRequest(
                                    block_id=b.blockId, lock_id=h.lock_id, session_id=self.session))
                                raise
                            self._locks.append((stub, h))
                            chosen = ("ipc", (h, base))
                            break
                        except Exception:  # noqa: BLE001 - fall back to the stream path
                            continue
                src[b.blockId] = chosen
        self._sources = src
        return src

    def close(self):
        from ..proto import pb
        for holder, lk in getattr(self, "_locks", []):
            try:
                if isinstance(lk, int):
                    holder.unlock(lk)
                else:
                    holder.UnlockDeviceBlock(pb.block.UnlockDeviceBlockRequest(
                        block_id=lk.block_id, lock_id=lk.lock_id, session_id=self.session))
            except Exception:  # noqa: BLE001
                pass
        self._locks = []
        self._sources = None
        self._one_worker = False

    # ---- planning -----------------------------------------------------------------------------
    def _pieces(self, rec_idx: int):
        """[(block info, offset in block, length, offset in record)] for one record."""
        f, off = self.ds.locate(rec_idx)
        lay = self.ds.files[f]
        out, done, n = [], 0, self.ds.record_bytes
        while done < n:
            bi = (off + done) // lay.block_size
            boff = (off + done) - bi * lay.block_size
            take = min(n - done, lay.block_size - boff)
            out.append((lay.blocks[bi], boff, take, done))
            done += take
        return out

    def _single_worker(self):
        """The in-process worker holding every block of a single-block-record dataset (then the
        batch plan is pure array arithmetic + one ``read_batch_arrays``), else None."""
        if not getattr(self.ds, "single_block", False):
            return None
        if getattr(self, "_one_worker", False) is not False:
            return self._one_worker
        srcs = self._open_sources()
        ws = {id(o): o for how, o in srcs.values() if how == "local"}
        self._one_worker = next(iter(ws.values())) if len(ws) == 1 and \
            all(how == "local" for how, _ in srcs.values()) else None
        return self._one_worker

    @traced("DeviceBatchLoader.fill")
    def _fill(self, out, indices):
        """Gather records ``indices`` into rows of ``out`` (uint8 [B, record_bytes])."""
        w = self._single_worker()
        if w is not None:
            ix = np.asarray(indices, dtype=np.int64)
            lens = self.ds.read_lengths[ix]
            if (lens < self.ds.record_bytes).any():
                out.zero_()                # pad short files
            dsts = np.uint64(out.data_ptr()) + np.arange(len(ix), dtype=np.uint64) * np.uint64(self.ds.record_bytes)
            stream = int(self.stream.cuda_stream) if self.stream is not None else 0
            w.native.read_batch_arrays(self.ds.block_ids[ix], np.zeros(len(ix), dtype=np.uint64), lens, dsts,
                                       1 if out.is_cuda else 0, stream, not out.is_cuda)
            w._count_read(int(lens.sum()), 1 if out.is_cuda else 0)
            return
        srcs = self._open_sources()
        kind = 1 if out.is_cuda else 0
        row = self.ds.record_bytes
        by_worker: dict[int, tuple] = {}
        ipc_segs = []
        slow = []
        base_ptr = out.data_ptr()
        for r, idx in enumerate(indices):
            for bi, boff, n, roff in self._pieces(int(idx)):
                how, obj = srcs[bi.blockId]
                dst = base_ptr + r * row + roff
                if how == "local":
                    by_worker.setdefault(id(obj), (obj, []))[1].append((bi.blockId, boff, n, dst, kind))
                elif how == "ipc":
                    h, base = obj
                    from ..parallel.ipc import page_segments
                    ipc_segs.extend(page_segments(base, list(h.pages), h.page_size, boff, n, dst))
                else:
                    slow.append((r, int(idx)))
        stream = int(self.stream.cuda_stream) if self.stream is not None else 0
        for w, reqs in by_worker.values():
            w.read_batch(reqs, stream, sync=not out.is_cuda)
        if ipc_segs:
            from ..ops.native import lib
            lib().batched_copy(ipc_segs, stream, True)
        for r, idx in sorted(set(slow)):
            f, off = self.ds.locate(idx)
            with self.ds.fs.open_file(self.ds.files[f].path) as s:
                s.pread(off, out[r])

    # ---- iteration ----------------------------------------------------------------------------
    def __len__(self):
        n = len(self.ds)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        import torch
        n = len(self.ds)
        order = np.random.default_rng(self.seed + self.epoch).permutation(n) if self.shuffle else np.arange(n)
        self.epoch += 1
        batches = [order[i:i + self.batch_size] for i in range(0, n, self.batch_size)]
        if self.drop_last and batches and len(batches[-1]) < self.batch_size:
            batches.pop()
        pending = []

        def launch(ix):
            buf = torch.empty((len(ix), self.ds.record_bytes), dtype=torch.uint8, device=self.device)
            if self.stream is not None:
                with torch.cuda.stream(self.stream):
                    self._fill(buf, ix)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
            else:
                self._fill(buf, ix)
                ev = None
            return buf, ev

        it = iter(batches)
        for ix in it:
            pending.append(launch(ix))
            if len(pending) >= self.prefetch:
                break
        while pending:
            buf, ev = pending.pop(0)
            nxt = next(it, None)
            if nxt is not None:
                pending.append(launch(nxt))
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
                buf.record_stream(torch.cuda.current_stream(self.device))
            t = buf.view(self.ds.dtype)
            yield t.view((buf.shape[0],) + self.ds.shape) if self.ds.shape else t

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
