"""Persist a cached file to its UFS (reference job/server/.../plan/persist/PersistDefinition.java:
read through the Alluxio client, write a temporary UFS file, rename into place, report the
fingerprint; master side: DefaultFileSystemMaster PersistenceScheduler/PersistenceChecker)."""
from __future__ import annotations

import logging
import os
import uuid

from ..proto import pb
from ..underfs import registry
from ..underfs.base import CreateOptions

LOG = logging.getLogger(__name__)


def _persist_from_worker(fs, info) -> int | None:
    """Persist a fully cached file without moving its bytes through this process: open the file's
    UFS stream (a native UFS_FILE WriteBlock) on the worker that holds every block and send one
    ``AppendBlock`` per block -- the worker copies each block out of its store (pipelined D2H from
    HBM) into a temp file it renames into place at commit, the same path as the CACHE_THROUGH tee.
    Object-store files take the same path: the worker's S3 stream fills its multipart parts from
    the store.  None when that shape does not apply (blocks spread over workers, no native
    writer); the caller then copies through the client."""
    from ..client.context import worker_address_str
    from ..client.streams import UfsWriter
    if not info.fileBlockInfos:
        return None
    common = None
    for fbi in info.fileBlockInfos:
        here = {worker_address_str(l.workerAddress): l.workerAddress for l in fbi.blockInfo.locations}
        common = here if common is None else {k: v for k, v in common.items() if k in here}
    if not common:
        return None
    addr = sorted(common)[0]
    w = UfsWriter(fs.ctx, info, addr, None, common[addr])
    if w._sink is None:                      # no native writer to that worker
        w.cancel()
        return None
    try:
        for fbi in info.fileBlockInfos:
            w.append_block(fbi.blockInfo.blockId, fbi.blockInfo.length)
        w.close()
    except BaseException:
        w.cancel()
        raise
    return w.length


def _mount_properties(fs, ufs_path: str) -> dict:
    """The options of the mount holding ``ufs_path`` (endpoint, credentials, part sizes: the
    reference resolves the UFS through the mount's UfsManager entry): the mount-table entry with
    the longest UFS URI prefix."""
    try:
        table = fs.get_mount_table()
    except Exception:  # noqa: BLE001 - an older master: client configuration only
        LOG.debug("no mount table", exc_info=True)
        return {}
    best, props = -1, {}
    for mp in table.values():
        root = mp.ufsUri.rstrip("/")
        if (ufs_path == root or ufs_path.startswith(root + "/")) and len(root) > best:
            best, props = len(root), dict(mp.properties)
    return props


def persist_file(fs, path: str, conf=None, chunk: int = 8 << 20) -> int:
    """Copy ``path`` from Alluxio to its UFS location; returns bytes written."""
    st = fs.get_status(path)
    info = st.info
    if (conf or fs.ctx.conf).get_bool("alluxio.job.persist.worker.append.enabled", "true"):
        try:
            n = _persist_from_worker(fs, info)
        except Exception:  # noqa: BLE001 - e.g. a block evicted meanwhile: copy through the client
            LOG.warning("worker-side persist of %s failed; copying through the client", path, exc_info=True)
            n = None
        if n is not None:
            return n
    ufs = registry.create(info.ufsPath, conf or fs.ctx.conf, _mount_properties(fs, info.ufsPath) or None)
    parent = os.path.dirname(info.ufsPath.rstrip("/"))
    if parent and not ufs.exists(parent):
        ufs.mkdirs(parent)
    tmp = f"{info.ufsPath}.alluxio.persist.{uuid.uuid4().hex[:8]}"
    n = 0
    with fs.open_file(path, read_type="NO_CACHE") as src, ufs.create(tmp, CreateOptions(mode=info.mode or 0o644)) as out:
        while True:
            data = src.read(chunk)
            if not data:
                break
            out.write(data)
            n += len(data)
    if ufs.exists(info.ufsPath):
        ufs.delete_file(info.ufsPath)
    if not ufs.rename_file(tmp, info.ufsPath):
        raise IOError(f"failed to rename {tmp} -> {info.ufsPath}")
    return n


def inline_persist_handler(fs_master, fs):
    """A persist handler that runs the copy synchronously in the master process (used when no
    job service is attached); the job service submits PersistDefinition jobs instead."""
    def handler(file_id: int, path: str):
        ok = False
        try:
            persist_file(fs, path)
            ok = True
        except Exception:  # noqa: BLE001
            LOG.exception("persist of %s failed", path)
        fs_master.persist_done(file_id, ok)
        return -1
    return handler


__all__ = ["persist_file", "inline_persist_handler", "pb"]
