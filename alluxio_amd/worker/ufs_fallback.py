"""UFS fallback block writes (the "UFS tier" of ASYNC_THROUGH writes).

Parity: core/server/worker/src/main/java/alluxio/worker/grpc/UfsFallbackBlockWriteHandler.java
(writes go to a local temp block; when the worker runs out of space the bytes written so far are
copied into a *UFS block file* and the rest of the stream continues there; the block is then
committed to the master as "in UFS" with ``commitBlockInUfs``), BlockUtils.getUfsBlockPath
(``<mount UFS root>/.alluxio_ufs_blocks.alluxio.0x1D91AC0E01AB0165.tmp/<blockId>``),
DefaultBlockWorker.openUfsBlock (:515-529: a read with ``block_in_ufs_tier`` and no UFS path is
served from that file) and DefaultFileSystemMaster's persist cleanup (:3985-3996: the staging UFS
block files are deleted once the file is persisted).

The same writer serves the gRPC ``WriteBlock`` handler (request type UFS_FALLBACK_BLOCK) and the
in-process client's local block writer.
"""
from __future__ import annotations

import logging

from ..ops.native import native_errors
from ..proto import pb
from ..utils.exceptions import WorkerOutOfSpaceException

LOG = logging.getLogger(__name__)

MAGIC_NUMBER = 0x1D91AC0E01AB0165
UFS_BLOCKS_DIR = ".alluxio_ufs_blocks" + ".alluxio.0x%016X.tmp" % MAGIC_NUMBER   # PathUtils.temporaryFileName
HOST = 0


def ufs_block_path(mount_uri: str, block_id: int) -> str:
    return mount_uri.rstrip("/") + "/" + UFS_BLOCKS_DIR + "/" + str(block_id)


class UfsFallbackBlockWriter:
    """Write one block locally, spilling to a UFS block file when the worker is out of space."""

    def __init__(self, worker, session: int, block_id: int, mount_id: int, tier: int = 0, medium: str = "",
                 reserve: int = 1 << 20, local: bool = True, pin: bool = False):
        self.w = worker
        self.session, self.block_id, self.mount_id = session, block_id, mount_id
        self.pos = 0
        self.pin = pin
        self.local = local
        self._out = self._ufs = self._path = None
        if local:
            try:
                worker.create_block(session, block_id, tier, medium, reserve, pin)
            except WorkerOutOfSpaceException:
                self.local = False
        if not self.local:
            self._open_ufs(0)

    @property
    def in_ufs(self) -> bool:
        return not self.local

    def _open_ufs(self, carry: int) -> None:
        from ..underfs.base import CreateOptions
        self._ufs, self._path = self.w.ufs_block_target(self.mount_id, self.block_id)
        self._out = self._ufs.create(self._path, CreateOptions(create_parent=True, ensure_atomic=True))
        if carry:
            # the bytes already in the temp block move to the UFS block file
            # (UfsFallbackBlockWriteHandler.transferToUfsBlock)
            step = 8 << 20
            for off in range(0, carry, step):
                n = min(step, carry - off)
                with native_errors():
                    data = self.w.native.read_frame(self.block_id, off, n, b"")
                self._out.write(data)
        if self.w.native.has_temp_block(self.block_id):
            try:
                self.w.abort_block(self.session, self.block_id)
            except Exception:  # noqa: BLE001
                pass
        self.w.metrics.counter("UfsFallbackBlocks").inc()

    def write(self, data) -> None:
        mv = memoryview(data)
        if self.local:
            try:
                self.w.write_bytes(self.session, self.block_id, self.pos, mv)
                self.pos += len(mv)
                return
            except WorkerOutOfSpaceException:
                LOG.warning("not enough space to write block %d locally, falling back to the UFS after %d bytes",
                            self.block_id, self.pos)
                self.local = False
                self._open_ufs(self.pos)
        self._out.write(mv)
        self.pos += len(mv)
        self.w.metrics.counter("BytesWrittenUfs").inc(len(mv))

    def write_ptr(self, offset: int, ptr: int, length: int, kind: int) -> None:
        if self.local:
            try:
                self.w.write_ptr(self.session, self.block_id, offset, ptr, length, kind)
                self.pos = max(self.pos, offset + length)
                return
            except WorkerOutOfSpaceException:
                self.local = False
                self._open_ufs(self.pos)
        import ctypes
        if kind == HOST:
            data = ctypes.string_at(ptr, length)
        else:
            import torch

            from ..ops.native import lib
            tmp = torch.empty(length, dtype=torch.uint8, device="cuda")
            lib().batched_copy([(ptr, tmp.data_ptr(), length)], 0)
            data = tmp.cpu().numpy().tobytes()
        self._out.write(data)
        self.pos = max(self.pos, offset + length)
        self.w.metrics.counter("BytesWrittenUfs").inc(length)

    def commit(self) -> None:
        if self.local:
            self.w.commit_block(self.session, self.block_id, self.pin)
            return
        self._out.close()
        self._out = None
        self.w.commit_block_in_ufs(self.block_id, self.pos)

    def cancel(self) -> None:
        if self.local:
            try:
                self.w.abort_block(self.session, self.block_id)
            except Exception:  # noqa: BLE001
                pass
            return
        try:
            if self._out is not None:
                self._out.close()
            self._ufs.delete_file(self._path)
        except Exception:  # noqa: BLE001
            LOG.debug("cleanup of UFS block %s failed", self._path, exc_info=True)


def resolve_ufs_block_opts(worker, block_id: int, opts):
    """A read of a UFS-tier block (``block_in_ufs_tier`` without a UFS path) is served from the
    block's UFS block file (DefaultBlockWorker.openUfsBlock)."""
    if opts is not None and opts.block_in_ufs_tier and not opts.ufs_path:
        o = pb.dataserver.OpenUfsBlockOptions()
        o.CopyFrom(opts)
        ufs, path = worker.ufs_block_target(opts.mountId, block_id)
        o.ufs_path = path
        o.offset_in_file = 0
        return o
    return opts
