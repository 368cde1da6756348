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


def persist_file(fs, path: str, conf=None, chunk: int = 8 << 20) -> int:
    """Copy ``path`` from Alluxio to its UFS location; returns bytes written."""
    st = fs.get_status(path)
    info = st.info
    ufs = registry.create(info.ufsPath, conf or fs.ctx.conf)
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
