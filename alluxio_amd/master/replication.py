"""Replication checker: enforce per-file replication limits and pinned media through the job service.

Parity: core/server/master/src/main/java/alluxio/master/file/replication/ReplicationChecker.java
(341 lines):

* ``heartbeat`` (:127-147) does nothing in safe mode, sleeps the quiet period, then runs three
  passes: REPLICATE over the pinned files (a file with ``replicationMin > 0`` is pinned), EVICT
  over the replication-limited files (``replicationMax`` set), and the mis-replication pass over
  the pinned files.
* ``check`` (:245-317): a block's target minimum is ``replicationMin``, raised to
  ``replicationDurable`` while the file is TO_BE_PERSISTED (ASYNC_THROUGH before its persist
  job finished); the same raise applies to the maximum.  A block below its minimum gets a
  ``replicate`` request for the missing copies -- also at 0 copies, where the job re-caches it from
  the UFS -- unless the file is not persisted and the block master counts the block as lost (no
  source left).  A block above its maximum gets an ``evict`` request for the excess.
* The job service pushing back (busy / resource exhausted) doubles the quiet period up to
  ``MAX_QUIET_PERIOD_SECONDS`` and ends the pass; every accepted request halves it.
* ``findMisplacedBlock`` (:162-202) / ``checkMisreplicated`` (:204-243): for a file pinned to
  media, if fewer than ``replicationMin`` copies sit on a pinned medium, the copies elsewhere are
  moved there (``migrate`` -> a ``move`` job on that worker: on MI355X, ``pin /ds HBM`` lands the
  blocks in the HBM tier by a DMA move).

The handler (reference job/client/.../DefaultReplicationHandler.java) submits the jobs; this
build's :class:`JobReplicationHandler` also keeps at most one outstanding job per block and kind.
"""
from __future__ import annotations

import logging
import time

from ..utils.exceptions import ResourceExhaustedException, UnavailableException

LOG = logging.getLogger(__name__)

MAX_QUIET_PERIOD_SECONDS = 64


class JobServiceBusy(ResourceExhaustedException):
    """The job service refused a request for now (reference JobDoesNotExist/ResourceExhausted)."""


class ReplicationHandler:
    """Reference job/client/src/main/java/alluxio/job/plan/replicate/ReplicationHandler.java."""

    def evict(self, path: str, block_id: int, num_replicas: int) -> int:
        raise NotImplementedError

    def replicate(self, path: str, block_id: int, num_replicas: int) -> int:
        raise NotImplementedError

    def migrate(self, path: str, block_id: int, worker_host: str, medium: str) -> int:
        raise NotImplementedError


class JobReplicationHandler(ReplicationHandler):
    """Submits evict / replicate / move jobs to the job master; a block with a job of the same kind
    still running is skipped (the heartbeat would otherwise pile up duplicates)."""

    def __init__(self, job_master, max_jobs: int = 1000):
        self.jm = job_master
        self.max_jobs = max_jobs
        self.inflight: dict[tuple[str, int], int] = {}

    def _running(self, key) -> bool:
        jid = self.inflight.get(key)
        if jid is None:
            return False
        try:
            st = self.jm.status(jid).status
        except Exception:  # noqa: BLE001 - purged
            st = "COMPLETED"
        if st in ("COMPLETED", "FAILED", "CANCELED"):
            del self.inflight[key]
            return False
        return True

    def _submit(self, kind: str, block_id: int, cfg) -> int:
        key = (kind, block_id)
        if self._running(key):
            return self.inflight[key]
        if len(self.inflight) >= self.max_jobs:
            for k in list(self.inflight):
                self._running(k)
            if len(self.inflight) >= self.max_jobs:
                raise JobServiceBusy(f"{len(self.inflight)} replication jobs outstanding")
        jid = self.jm.run(cfg)
        self.inflight[key] = jid
        return jid

    def evict(self, path, block_id, num_replicas):
        from ..job import EvictConfig
        return self._submit("evict", block_id, EvictConfig(block_id=block_id, replicas=num_replicas))

    def replicate(self, path, block_id, num_replicas):
        from ..job import ReplicateConfig
        return self._submit("replicate", block_id, ReplicateConfig(block_id=block_id, replicas=num_replicas,
                                                                   path=path))

    def migrate(self, path, block_id, worker_host, medium):
        from ..job import MoveConfig
        return self._submit("move", block_id, MoveConfig(block_id=block_id, worker_host=worker_host, medium=medium))


class ReplicationChecker:
    REPLICATE, EVICT = "REPLICATE", "EVICT"

    def __init__(self, fs_master, handler, safe_mode=None, max_jobs: int = 1000):
        self.fsm = fs_master
        # a job master (legacy call sites) gets the job-service handler
        self.handler = handler if isinstance(handler, ReplicationHandler) else JobReplicationHandler(handler, max_jobs)
        self.safe_mode = safe_mode
        self.quiet_period_s = 0
        self.sleep = time.sleep

    # ---- heartbeat ------------------------------------------------------------------------------
    def heartbeat(self) -> int:
        """One pass; returns the requests the handler accepted."""
        if self.safe_mode is not None and self.safe_mode.in_safe_mode():
            return 0   # skip while not all workers have re-registered
        if self.quiet_period_s:
            self.sleep(self.quiet_period_s)
        n = self.check(self.fsm.pinned_file_ids(), self.REPLICATE)
        n += self.check(self.fsm.replication_limited_file_ids(), self.EVICT)
        n += self.check_misreplicated(self.fsm.pinned_file_ids())
        return n

    def check(self, file_ids, mode: str) -> int:
        bm = self.fsm.block_master
        lost = bm.lost_blocks()
        requests: dict[int, tuple[str, int]] = {}
        for fid in file_ids:
            v = self.fsm.replication_view(fid)
            if v is None:
                continue
            for bid in v.block_ids:
                bi = bm.block_info_or_none(bid)
                have = len(bi.locations) if bi is not None else 0
                if mode == self.EVICT:
                    cap = v.replication_max
                    if v.persistence_state == "TO_BE_PERSISTED" and v.replication_durable > cap:
                        cap = v.replication_durable
                    if cap >= 0 and have > cap:
                        requests[bid] = (v.path, have - cap)
                else:
                    need = v.replication_min
                    if v.persistence_state == "TO_BE_PERSISTED" and v.replication_durable > need:
                        need = v.replication_durable
                    if have < need:
                        if not v.persisted and bid in lost:
                            continue      # no copy and no UFS source: nothing can restore it
                        requests[bid] = (v.path, need - have)
        accepted = 0
        for bid, (path, n) in requests.items():
            try:
                if mode == self.EVICT:
                    self.handler.evict(path, bid, n)
                else:
                    self.handler.replicate(path, bid, n)
                self.quiet_period_s //= 2
                accepted += 1
            except ResourceExhaustedException as e:
                LOG.warning("The job service is busy, will retry later. %s", e)
                self.quiet_period_s = 1 if self.quiet_period_s == 0 else \
                    min(MAX_QUIET_PERIOD_SECONDS, self.quiet_period_s * 2)
                return accepted
            except UnavailableException as e:
                LOG.warning("Unable to complete the replication check: %s, will retry later.", e)
                return accepted
            except Exception as e:  # noqa: BLE001
                LOG.warning("Unexpected exception starting a %s job (uri=%s, block ID=%d, num replicas=%d): %s",
                            mode, path, bid, n, e)
        return accepted

    @staticmethod
    def find_misplaced(medium_types, replication_min: int, locations) -> dict[str, str]:
        """worker host -> pinned medium for the copies to move so that at least
        ``replication_min`` copies sit on a pinned medium (ReplicationChecker.findMisplacedBlock)."""
        if not medium_types:
            return {}
        first = medium_types[0]
        correct, candidates = 0, []
        for loc in locations:
            if loc.mediumType in medium_types:
                correct += 1
            else:
                candidates.append(loc.workerAddress.host)
        if correct >= replication_min:
            return {}
        moves, to_move = {}, replication_min - correct
        for host in candidates:
            moves[host] = first
            to_move -= 1
            if to_move == 0:
                break
        return moves

    def check_misreplicated(self, file_ids) -> int:
        bm = self.fsm.block_master
        accepted = 0
        for fid in file_ids:
            v = self.fsm.replication_view(fid)
            if v is None or not v.medium_types:
                continue
            for bid in v.block_ids:
                bi = bm.block_info_or_none(bid)
                if bi is None:
                    continue      # not cached anywhere (possibly only in the UFS): nothing to move
                for host, medium in self.find_misplaced(v.medium_types, v.replication_min, bi.locations).items():
                    try:
                        self.handler.migrate(v.path, bid, host, medium)
                        accepted += 1
                    except Exception as e:  # noqa: BLE001
                        LOG.warning("Unexpected exception starting a migration job (uri=%s, block ID=%d, "
                                    "workerHost=%s): %s", v.path, bid, host, e)
        return accepted
