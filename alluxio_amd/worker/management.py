"""Background tier management: align / promote / swap-restore between adjacent tiers.

Parity: core/server/worker/src/main/java/alluxio/worker/block/management/
ManagementTaskCoordinator.java:39-190 (runs the provider's tasks when user I/O is idle, with
backoff), tier/TierManagementTaskProvider.java:40-174 (task selection), tier/AlignTask.java
(swap blocks so the upper tier holds the hotter ones, ``align.range`` per pass),
tier/PromoteTask.java (move hot lower-tier blocks up while the upper tier is under
``promote.quota.percent``), tier/SwapRestoreTask.java (move cold blocks down when a tier eats
into its reserved space) and DefaultStoreLoadTracker.java:34-64 (user-I/O load detection with a
cool-down window).

On MI355X the usual tiers are HBM (MEM) above pinned host DRAM / NVMe; a move is a page-gather
D2D/D2H/H2D copy inside the native store on its internal stream.  Hotness comes from the same
annotator order (LRU clock or LRFU CRF) the eviction kernel uses, read across both tiers.
"""
from __future__ import annotations

import logging
import time

from ..utils import ids
from ..utils.exceptions import AlluxioStatusException

LOG = logging.getLogger(__name__)


class TierManager:
    def __init__(self, worker, conf):
        self.w = worker
        self.conf = conf
        self.align_enabled = conf.get_bool("alluxio.worker.management.tier.align.enabled")
        self.promote_enabled = conf.get_bool("alluxio.worker.management.tier.promote.enabled")
        self.swap_enabled = conf.get_bool("alluxio.worker.management.tier.swap.restore.enabled")
        self.align_range = conf.get_int("alluxio.worker.management.tier.align.range")
        self.promote_range = conf.get_int("alluxio.worker.management.tier.promote.range")
        self.promote_quota = conf.get_int("alluxio.worker.management.tier.promote.quota.percent") / 100.0
        self.reserved = conf.get_bytes("alluxio.worker.management.tier.align.reserved.bytes")
        self.cool_down_s = conf.get_ms("alluxio.worker.management.load.detection.cool.down.time") / 1000.0
        self._last_io = 0.0
        self._last_bytes = 0
        self.session = ids.create_session_id()
        self.stats = {"promoted": 0, "aligned": 0, "restored": 0, "skipped_busy": 0}

    # ---- load detection -----------------------------------------------------------------------
    def user_io_active(self) -> bool:
        m = self.w.metrics
        n = m.counter("BytesReadAlluxio").count + m.counter("BytesWrittenAlluxio").count
        now = time.time()
        if n != self._last_bytes:
            self._last_bytes = n
            self._last_io = now
        return now - self._last_io < self.cool_down_s

    # ---- tier geometry ------------------------------------------------------------------------
    def tiers(self) -> list[int]:
        return sorted({d.tier for d in self.w.store.dirs})

    def _tier_space(self, tier: int) -> tuple[int, int]:
        cap = avail = 0
        for i, d in enumerate(self.w.store.dirs):
            if d.tier == tier:
                cap += self.w.native.dir_capacity(i)
                avail += self.w.native.dir_available(i)
        return cap, avail

    def _tier_blocks_hot_first(self, tier: int) -> list[int]:
        return list(reversed(self.w.native.eviction_order(tier, 0)))

    def _move(self, bid: int, tier: int, evict: bool) -> bool:
        try:
            self.w.native.move_block(self.session, bid, tier, "", evict)
            return True
        except Exception as e:  # noqa: BLE001 - locked / vanished / no space: skip this block
            LOG.debug("tier move of %d to %d skipped: %s", bid, tier, e)
            return False

    # ---- tasks --------------------------------------------------------------------------------
    def promote(self, upper: int, lower: int) -> int:
        cap, avail = self._tier_space(upper)
        moved = 0
        for bid in self._tier_blocks_hot_first(lower)[:self.promote_range]:
            info = self.w.native.block_info(bid)
            if cap - avail + info.length > self.promote_quota * cap:
                break
            if self._move(bid, upper, evict=False):
                moved += 1
                avail -= info.length
        self.stats["promoted"] += moved
        return moved

    def align(self, upper: int, lower: int) -> int:
        """Swap pairs (coldest upper, hottest lower) while the lower block is hotter."""
        rank = {b: i for i, b in enumerate(self.w.native.eviction_order(-1, 0))}  # higher = hotter
        cold_up = [b for b in self.w.native.eviction_order(upper, 0)][:self.align_range]
        hot_low = self._tier_blocks_hot_first(lower)[:self.align_range]
        swapped = 0
        for cu, hl in zip(cold_up, hot_low):
            if rank.get(hl, -1) <= rank.get(cu, -1):
                break
            if self._move(cu, lower, evict=True) and self._move(hl, upper, evict=True):
                swapped += 1
        self.stats["aligned"] += swapped
        return swapped

    def swap_restore(self, upper: int, lower: int) -> int:
        """Move the coldest upper-tier blocks down until ``reserved`` bytes are free again."""
        cap, avail = self._tier_space(upper)
        need = min(self.reserved, cap // 10) - avail
        moved = 0
        if need <= 0:
            return 0
        for bid in self.w.native.eviction_order(upper, need):
            if self._move(bid, lower, evict=True):
                moved += 1
        self.stats["restored"] += moved
        return moved

    def run_once(self, force: bool = False) -> dict:
        if not force and self.user_io_active():
            self.stats["skipped_busy"] += 1
            return dict(self.stats)
        ts = self.tiers()
        for upper, lower in zip(ts, ts[1:]):
            try:
                if self.swap_enabled:
                    self.swap_restore(upper, lower)
                if self.promote_enabled:
                    self.promote(upper, lower)
                if self.align_enabled:
                    self.align(upper, lower)
            except AlluxioStatusException:
                LOG.debug("tier management pass failed", exc_info=True)
        return dict(self.stats)
