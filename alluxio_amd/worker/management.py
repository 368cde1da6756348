"""Background tier management: align / promote / swap-restore between adjacent tiers (K8).

Parity: core/server/worker/src/main/java/alluxio/worker/block/management/
ManagementTaskCoordinator.java:39-190 (runs the provider's tasks when user I/O is idle, with
backoff), tier/TierManagementTaskProvider.java:40-174 (task selection), tier/AlignTask.java
(swap blocks so the upper tier holds the hotter ones, ``align.range`` per pass, using the dirs'
reserved space), tier/PromoteTask.java (move hot lower-tier blocks up while the upper tier is
under ``promote.quota.percent``), tier/SwapRestoreTask.java (move blocks out of a tier that eats
into its reserved space), BlockTransferPartitioner.java (split transfers into groups that touch
disjoint locations) + BlockTransferExecutor.java (run the groups concurrently) and
DefaultStoreLoadTracker.java:34-64 (user-I/O load detection with a cool-down window).

MI355X design:
* tier order: the k coldest blocks of the upper tier and the k hottest of the lower tier come from
  the device grid select over the HBM-resident annotations (``BlockStore.tier_order``, O(n) on the
  GPU, only the k winners are ordered on the host) -- the "device tier-order merge": the swap
  count is the length of the prefix where hottest-lower[i] is hotter than coldest-upper[i];
* transfers: partitioned by (source dir, destination tier); each partition is ONE batched native
  move (``BlockStore.move_blocks``: all HBM<->HBM pieces in one batched-copy launch, HBM<->DRAM as
  async DMA, one stream sync), partitions run concurrently on
  ``alluxio.worker.management.block.transfer.concurrency.limit`` threads;
* swaps use the dirs' reserved space (``alluxio.worker.management.tier.align.reserved.bytes``,
  kept free for user allocations), exactly like the reference's AllocateOptions.useReservedSpace.
"""
from __future__ import annotations

import logging
import threading
import time
from concurrent.futures import ThreadPoolExecutor

from ..utils import ids
from ..utils.exceptions import AlluxioStatusException

LOG = logging.getLogger(__name__)


class StoreLoadTracker:
    """User I/O seen within the cool-down window = load (DefaultStoreLoadTracker)."""

    def __init__(self, worker, cool_down_s: float):
        self.w = worker
        self.cool_down_s = cool_down_s
        self._last_io = 0.0
        self._last_bytes = 0

    def loaded(self) -> bool:
        m = self.w.metrics
        n = m.counter("BytesReadAlluxio").count + m.counter("BytesWrittenAlluxio").count
        now = time.time()
        if n != self._last_bytes:
            self._last_bytes = n
            self._last_io = now
        return now - self._last_io < self.cool_down_s


class BlockTransferPartitioner:
    """Group transfers so every group touches one (source dir, destination tier) pair: groups are
    independent batched moves (BlockTransferPartitioner.partitionTransfers)."""

    @staticmethod
    def partition(native, transfers: list[tuple[int, int]], max_partitions: int) -> list[list[tuple[int, int]]]:
        groups: dict = {}
        for bid, dst in transfers:
            try:
                src_dir = native.block_info(bid).dir
            except Exception:  # noqa: BLE001 - vanished
                continue
            groups.setdefault((src_dir, dst), []).append((bid, dst))
        parts = sorted(groups.values(), key=len, reverse=True)
        if len(parts) <= max_partitions:
            return parts
        # fold the smallest groups into the largest ones with the same destination
        out = parts[:max_partitions]
        for g in parts[max_partitions:]:
            tgt = next((o for o in out if o[0][1] == g[0][1]), out[-1])
            tgt.extend(g)
        return out


class BlockTransferExecutor:
    """Run transfer partitions concurrently, each as one batched native move."""

    def __init__(self, worker, concurrency: int, session: int):
        self.w = worker
        self.concurrency = max(1, concurrency)
        self.session = session
        self._pool = ThreadPoolExecutor(max_workers=self.concurrency, thread_name_prefix="tier-transfer")

    def execute(self, transfers: list[tuple[int, int]], use_reserved: bool = True, evict: bool = False) -> list[int]:
        parts = BlockTransferPartitioner.partition(self.w.native, transfers, self.concurrency)

        def run(part):
            dst = part[0][1]
            try:
                return self.w.native.move_blocks(self.session, [b for b, _ in part], dst, "", evict, use_reserved)
            except Exception as e:  # noqa: BLE001 - locked / no space: the rest of the pass goes on
                LOG.debug("batched tier move to %d failed: %s", dst, e)
                return []
        moved = []
        for r in self._pool.map(run, parts):
            moved.extend(r)
        return moved

    def close(self) -> None:
        self._pool.shutdown(wait=False)


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
        self.load = StoreLoadTracker(worker, conf.get_ms("alluxio.worker.management.load.detection.cool.down.time")
                                     / 1000.0)
        self.device_order = conf.get_bool("alluxio.worker.eviction.device.enabled", "true")
        self.session = ids.create_session_id()
        conc = conf.get_raw("alluxio.worker.management.block.transfer.concurrency.limit")
        self.executor = BlockTransferExecutor(worker, int(conc) if conc else 4, self.session)
        self.stats = {"promoted": 0, "aligned": 0, "restored": 0, "skipped_busy": 0, "passes": 0}
        self._thread = None
        self._stop = threading.Event()

    # ---- compatibility shims (tests / callers tune these directly) ----------------------------
    @property
    def cool_down_s(self) -> float:
        return self.load.cool_down_s

    @cool_down_s.setter
    def cool_down_s(self, v: float) -> None:
        self.load.cool_down_s = v

    def user_io_active(self) -> bool:
        return self.load.loaded()

    # ---- tier geometry ------------------------------------------------------------------------
    def tiers(self) -> list[int]:
        return sorted({d.tier for d in self.w.store.dirs})

    def _dirs(self, tier: int) -> list[int]:
        return [i for i, d in enumerate(self.w.store.dirs) if d.tier == tier]

    def _tier_space(self, tier: int) -> tuple[int, int]:
        cap = avail = 0
        for i in self._dirs(tier):
            cap += self.w.native.dir_capacity(i)
            avail += self.w.native.dir_available(i)
        return cap, avail

    def order(self, tier: int, k: int, hottest: bool) -> list[int]:
        """k blocks of ``tier`` in annotator order (device select + host order of the k)."""
        return self.w.native.tier_order(tier, k, hottest, self.device_order)

    def aligned(self, upper: int, lower: int) -> bool:
        """Every upper-tier block is at least as hot as every lower-tier block."""
        cold_up = self.order(upper, 1, False)
        hot_low = self.order(lower, 1, True)
        if not cold_up or not hot_low:
            return True
        return self._swap_count(cold_up, hot_low) == 0

    def _swap_count(self, cold_up: list[int], hot_low: list[int]) -> int:
        """Length of the prefix where hot_low[i] is hotter than cold_up[i]: the merge path of the
        two orders (both lists are monotone, so the predicate holds on a prefix).  Keys are the
        annotator keys of one common order (larger = hotter)."""
        n = min(len(cold_up), len(hot_low))
        if n == 0:
            return 0
        keys = self.w.native.annotator_keys(cold_up[:n] + hot_low[:n])
        ku, kl = keys[:n], keys[n:]
        lo, hi = 0, n            # binary search the first i with kl[i] <= ku[i]
        while lo < hi:
            mid = (lo + hi) // 2
            if kl[mid] > ku[mid] and kl[mid] != 0xFFFFFFFF:
                lo = mid + 1
            else:
                hi = mid
        return lo

    # ---- tasks --------------------------------------------------------------------------------
    def promote(self, upper: int, lower: int) -> int:
        cap, avail = self._tier_space(upper)
        used = cap - avail
        picks = []
        for bid in self.order(lower, self.promote_range, True):
            length = self.w.native.block_info(bid).length
            if used + length > self.promote_quota * cap:
                break
            picks.append((bid, upper))
            used += length
        moved = self.executor.execute(picks, use_reserved=False) if picks else []
        self.stats["promoted"] += len(moved)
        return len(moved)

    def align(self, upper: int, lower: int) -> int:
        """Swap the k coldest upper-tier blocks with the k hottest lower-tier blocks while the
        lower one is hotter; moves run through the reserved space, down first, then up."""
        cold_up = self.order(upper, self.align_range, False)
        hot_low = self.order(lower, self.align_range, True)
        k = self._swap_count(cold_up, hot_low)
        if k == 0:
            return 0
        down = self.executor.execute([(b, lower) for b in cold_up[:k]], use_reserved=True)
        # as many up as went down (the space they freed, plus the reserve for the in-flight pair)
        up = self.executor.execute([(b, upper) for b in hot_low[:len(down)]], use_reserved=True) if down else []
        swapped = min(len(down), len(up))
        self.stats["aligned"] += swapped
        return swapped

    def swap_restore(self, upper: int, lower: int) -> int:
        """A dir whose reserved space is in use (swaps or promotions filled it) gets its coldest
        blocks moved down until the reserve is free again (SwapRestoreTask)."""
        moved_total = 0
        for d in self._dirs(upper):
            reserve = self.w.native.dir_spec(d).reserved
            if reserve <= 0:
                continue
            in_reserve = reserve - self.w.native.dir_mgmt_available(d)
            if in_reserve <= 0:
                continue
            picks, got = [], 0
            for bid in self.order(upper, max(1, self.align_range), False):
                info = self.w.native.block_info(bid)
                if info.dir != d:
                    continue
                picks.append((bid, lower))
                got += info.length
                if got >= in_reserve:
                    break
            moved = self.executor.execute(picks, use_reserved=False, evict=True) if picks else []
            moved_total += len(moved)
        self.stats["restored"] += moved_total
        return moved_total

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
        self.stats["passes"] += 1
        return dict(self.stats)

    # ---- coordinator --------------------------------------------------------------------------
    def start(self, interval_s: float = 1.0) -> None:
        """ManagementTaskCoordinator: run passes while user I/O is idle, backing off otherwise."""
        if self._thread is not None:
            return
        self._stop.clear()

        def loop():
            backoff = interval_s
            while not self._stop.wait(backoff):
                busy = self.user_io_active()
                if not busy:
                    try:
                        self.run_once(force=True)
                    except Exception:  # noqa: BLE001
                        LOG.debug("tier management pass failed", exc_info=True)
                    backoff = interval_s
                else:
                    self.stats["skipped_busy"] += 1
                    backoff = min(backoff * 2, max(interval_s, self.cool_down_s))
        self._thread = threading.Thread(target=loop, daemon=True, name="tier-management")
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None
        self.executor.close()
