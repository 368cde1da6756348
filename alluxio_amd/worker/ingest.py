"""K3: UFS -> HBM ingest with the H2D copy overlapped with the next UFS read.

Reference: UnderFileSystemBlockReader.java:205-243 reads a chunk from the UFS stream and appends
it to the local block writer before returning it, one chunk at a time; AsyncCacheRequestManager
(:88-150) caches whole blocks the same way in the background.  On MI355X the append is a
host->HBM DMA, so a serial loop leaves the UFS idle while the DMA runs and the DMA engine idle
while the UFS is read.  :class:`IngestPipeline` keeps ``depth`` pinned staging buffers and a
dedicated HIP side stream: chunk *i* is read from the UFS into buffer ``i % depth`` (GIL released
in the file/socket read), its H2D copy into the block's pages is queued on the side stream without
waiting, and an event per buffer gates its reuse ``depth`` chunks later.  Reads of chunk *i+1*
therefore overlap the DMA of chunk *i*; the only host wait is the final stream sync before commit.

Blocks on a host tier (DRAM) take the same path: the store's write is then a host memcpy.
"""
from __future__ import annotations

import threading
import time

from ..ops.native import native_errors

HOST = 0


class IngestPipeline:
    def __init__(self, worker, chunk: int, depth: int = 3):
        import torch

        from ..ops.native import has_gpu
        self.w = worker
        self.chunk = chunk
        self.depth = max(1, depth)
        self.gpu = has_gpu() and worker.store.has_device_tier
        dev = worker.store.device if self.gpu else None
        self.bufs = [torch.empty(chunk, dtype=torch.uint8, pin_memory=has_gpu()) for _ in range(self.depth)]
        self.stream = torch.cuda.Stream(device=dev) if self.gpu else None
        self.events = [None] * self.depth
        self.stats = {"chunks": 0, "bytes": 0, "read_s": 0.0, "wait_s": 0.0}

    def _wait_slot(self, k: int) -> None:
        ev = self.events[k]
        if ev is not None:
            t = time.perf_counter()
            ev.synchronize()            # the DMA out of this buffer (depth chunks ago) is done
            self.stats["wait_s"] += time.perf_counter() - t
            self.events[k] = None

    def run(self, session_id: int, block_id: int, reader, length: int, on_chunk=None) -> int:
        """Copy ``length`` bytes from ``reader`` (``readinto``/``read``) into the temp block at
        offset 0; ``on_chunk(memoryview)`` sees each chunk before its buffer is reused (the
        read-through stream hands it to the client).  Returns the bytes ingested."""
        import torch
        pos, k = 0, 0
        sh = self.stream.cuda_stream if self.stream is not None else 0
        try:
            while pos < length:
                slot = k % self.depth
                self._wait_slot(slot)
                buf = self.bufs[slot]
                n = min(self.chunk, length - pos)
                mv = memoryview(buf.numpy())[:n]
                t = time.perf_counter()
                got = _read_into(reader, mv)
                self.stats["read_s"] += time.perf_counter() - t
                if not got:
                    break
                with native_errors():
                    self.w.native.write(session_id, block_id, pos, buf.data_ptr(), got, HOST, sh, False)
                if self.stream is not None:
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                    self.events[slot] = ev
                if on_chunk is not None:
                    on_chunk(mv[:got])
                pos += got
                k += 1
                self.stats["chunks"] += 1
                self.stats["bytes"] += got
        finally:
            if self.stream is not None:
                self.stream.synchronize()
            self.events = [None] * self.depth
        return pos


def _read_into(reader, mv) -> int:
    if hasattr(reader, "readinto"):
        got = reader.readinto(mv)
        return got or 0
    data = reader.read(len(mv))
    n = len(data)
    mv[:n] = data
    return n


class IngestPool:
    """Pipelines (pinned buffer sets + side streams) shared by concurrent caching threads."""

    def __init__(self, worker, chunk: int, depth: int, size: int):
        self.w, self.chunk, self.depth, self.size = worker, chunk, depth, max(1, size)
        self._free: list[IngestPipeline] = []
        self._made = 0
        self._cond = threading.Condition()

    def acquire(self) -> IngestPipeline:
        with self._cond:
            while not self._free and self._made >= self.size:
                self._cond.wait()
            if self._free:
                return self._free.pop()
            self._made += 1
        return IngestPipeline(self.w, self.chunk, self.depth)

    def release(self, p: IngestPipeline) -> None:
        with self._cond:
            self._free.append(p)
            self._cond.notify()
