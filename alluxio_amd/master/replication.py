"""Replication checker: enforce per-file min/max block replication through the job service.

Parity: core/server/master/src/main/java/alluxio/master/file/replication/ReplicationChecker.java:57-341
(heartbeat :127 — for every file with replication limits, compare each block's live replica
count with replicationMin/Max; under-replicated blocks get a ``replicate`` job for the missing
copies, over-replicated ones an ``evict`` job for the excess; at most one outstanding job per
block; pinned files are never evicted below their minimum).  On an MI355X node the replicate
task is an xGMI pull by the target worker (parallel/transfer.py).
"""
from __future__ import annotations

import logging

LOG = logging.getLogger(__name__)


class ReplicationChecker:
    def __init__(self, fs_master, job_master, max_jobs: int = 1000):
        self.fsm = fs_master
        self.jm = job_master
        self.max_jobs = max_jobs
        self.inflight: dict[int, int] = {}   # block id -> job id

    def _busy(self, bid: int) -> bool:
        jid = self.inflight.get(bid)
        if jid is None:
            return False
        try:
            st = self.jm.status(jid).status
        except Exception:  # noqa: BLE001 - purged
            st = "COMPLETED"
        if st in ("COMPLETED", "FAILED", "CANCELED"):
            del self.inflight[bid]
            return False
        return True

    def heartbeat(self) -> int:
        from ..job import EvictConfig, ReplicateConfig
        live_workers = len(self.fsm.block_master.worker_info_list())
        submitted = 0
        for path, bid, have, rmin, rmax, pinned in self.fsm.replication_targets():
            if submitted >= self.max_jobs or self._busy(bid):
                continue
            if have < rmin and have > 0:
                want = min(rmin, live_workers) - have
                if want > 0:
                    self.inflight[bid] = self.jm.run(ReplicateConfig(block_id=bid, replicas=want, path=path))
                    submitted += 1
            elif rmax >= 0 and have > rmax:
                excess = have - max(rmax, rmin if pinned else rmax)
                if excess > 0:
                    self.inflight[bid] = self.jm.run(EvictConfig(block_id=bid, replicas=excess))
                    submitted += 1
        return submitted
