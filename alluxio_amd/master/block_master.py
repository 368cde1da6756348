"""Block master: worker registry, block locations, container ids, lost-worker detection.

Parity: core/server/master/src/main/java/alluxio/master/block/DefaultBlockMaster.java
(getNewContainerId :628 journaled BlockContainerIdGeneratorEntry; commitBlock :670-716 journaled
BlockInfoEntry + location; getWorkerId :844-866 reusing ids for known addresses; workerRegister
:869-913; workerHeartbeat :916-950 returning Nothing/Register/Free; generateBlockInfo
:1037-1072; LostWorkerDetectionHeartbeatExecutor :1087-1113), MasterWorkerInfo.java (per-worker
capacity/usage per tier, blocks, to-be-removed blocks), the worker sets kept in IndexedSets.
"""
from __future__ import annotations

import logging
import threading
import time

from ..journal.system import Journaled
from ..proto import pb
from ..utils import ids
from ..utils.collections import IndexedSet
from ..utils.exceptions import BlockDoesNotExistException, NotFoundException

LOG = logging.getLogger(__name__)

CONTAINER_BATCH = 1000  # container ids reserved per journal entry


def address_key(addr) -> tuple:
    return (addr.host, addr.rpcPort, addr.dataPort, addr.domainSocketPath)


class MasterWorkerInfo:
    def __init__(self, worker_id: int, address):
        self.id = worker_id
        self.address = address
        self.start_time_ms = int(time.time() * 1000)
        self.last_updated_ms = int(time.time() * 1000)
        self.registered = False
        self.storage_tiers: list[str] = []
        self.capacity: dict[str, int] = {}
        self.used: dict[str, int] = {}
        self.blocks: set[int] = set()
        self.to_remove: set[int] = set()
        self.lost_storage: dict[str, list[str]] = {}
        self.lock = threading.RLock()

    @property
    def key(self):
        return address_key(self.address)

    def capacity_bytes(self) -> int:
        return sum(self.capacity.values())

    def used_bytes(self) -> int:
        return sum(self.used.values())

    def to_proto(self, state: str):
        w = pb.block.WorkerInfo(id=self.id, address=self.address,
                                lastContactSec=int((time.time() * 1000 - self.last_updated_ms) / 1000),
                                state=state, capacityBytes=self.capacity_bytes(), usedBytes=self.used_bytes(),
                                startTimeMs=self.start_time_ms)
        for k, v in self.capacity.items():
            w.capacityBytesOnTiers[k] = v
        for k, v in self.used.items():
            w.usedBytesOnTiers[k] = v
        return w


class BlockMeta:
    __slots__ = ("length", "locations")

    def __init__(self, length: int):
        self.length = length
        self.locations: dict[int, tuple[str, str]] = {}  # worker id -> (tier alias, medium)


class BlockMaster(Journaled):
    journal_name = "BlockMaster"

    def __init__(self, conf=None, journal_system=None, metrics=None, worker_timeout_ms: int = 300_000,
                 global_tiers=("MEM", "SSD", "HDD")):
        self.conf = conf
        self.journal = journal_system
        self.metrics = metrics
        self.worker_timeout_ms = worker_timeout_ms
        self.global_tiers = list(global_tiers)
        self._lock = threading.RLock()
        self._blocks: dict[int, BlockMeta] = {}
        self._next_container = 0
        self._container_limit = 0
        self._registered = IndexedSet(id=(lambda w: w.id, True), addr=(lambda w: w.key, True))
        self._temp = IndexedSet(id=(lambda w: w.id, True), addr=(lambda w: w.key, True))
        self._lost = IndexedSet(id=(lambda w: w.id, True), addr=(lambda w: w.key, True))
        self._lost_blocks: set[int] = set()
        # bumped whenever a block's length/locations or the live-worker set change: versions the
        # FileSystemMaster's cached FileInfo replies (they embed block locations)
        self.location_epoch = 0
        self.epoch_listeners: list = []
        self.lost_worker_listeners = []
        self.worker_registered_listeners = []
        self.safe_mode = None
        self._bi_cache: tuple = (None, {})

    def _bump_epoch(self) -> None:
        self.location_epoch += 1
        for cb in self.epoch_listeners:
            cb()

    # ---- Journaled ----------------------------------------------------------------------------
    def reset_state(self) -> None:
        with self._lock:
            self._bump_epoch()
            self._blocks.clear()
            self._next_container = 0
            self._container_limit = 0

    def process_journal_entry(self, e) -> bool:
        with self._lock:
            self._bump_epoch()
            if e.HasField("block_container_id_generator"):
                self._container_limit = e.block_container_id_generator.next_container_id
                self._next_container = max(self._next_container, self._container_limit)
            elif e.HasField("block_info"):
                bi = e.block_info
                m = self._blocks.get(bi.block_id)
                if m is None:
                    self._blocks[bi.block_id] = BlockMeta(bi.length)
                else:
                    m.length = bi.length
            elif e.HasField("delete_block"):
                self._blocks.pop(e.delete_block.block_id, None)
            else:
                return False
            return True

    def journal_entries(self):
        with self._lock:
            yield pb.journal.JournalEntry(block_container_id_generator=pb.journal.BlockContainerIdGeneratorEntry(
                next_container_id=self._container_limit))
            for bid, m in sorted(self._blocks.items()):
                yield pb.journal.JournalEntry(block_info=pb.journal.BlockInfoEntry(block_id=bid, length=m.length))

    def _ctx(self):
        from ..journal.system import NoopJournalContext
        if self.journal is None:
            return NoopJournalContext()
        return self.journal.create_context(self.journal_name)

    # ---- container ids ------------------------------------------------------------------------
    def get_new_container_id(self) -> int:
        """Journaled in batches: one entry reserves CONTAINER_BATCH ids."""
        ctx = None
        with self._lock:
            cid = self._next_container
            self._next_container += 1
            if self._next_container > self._container_limit:
                limit = cid + CONTAINER_BATCH
                e = pb.journal.JournalEntry(block_container_id_generator=pb.journal.BlockContainerIdGeneratorEntry(
                    next_container_id=limit))
                self._container_limit = limit
                ctx = self._ctx()
                ctx.append(e)
        if ctx is not None:
            ctx.close()
        return cid

    def get_new_container_ids(self, n: int) -> list[int]:
        """``n`` consecutive container ids with at most one journal entry (a bulk metadata load)."""
        if n <= 0:
            return []
        ctx = None
        with self._lock:
            cid = self._next_container
            self._next_container += n
            if self._next_container > self._container_limit:
                limit = cid + n + CONTAINER_BATCH
                e = pb.journal.JournalEntry(block_container_id_generator=pb.journal.BlockContainerIdGeneratorEntry(
                    next_container_id=limit))
                self._container_limit = limit
                ctx = self._ctx()
                ctx.append(e)
        if ctx is not None:
            ctx.close()
        return list(range(cid, cid + n))

    def block_info_bytes(self, block_id: int) -> tuple[bytes, int, bool]:
        """(serialized BlockInfo, length, has a MEM location) of a block that has locations, or
        (b"", length, False) for one stored only in the UFS / unknown (the FileInfo encoder
        synthesises those).  Serialized infos are cached per location epoch."""
        m = self._blocks.get(block_id)
        if m is None or not m.locations:
            return b"", (m.length if m is not None else 0), False
        cache = self._bi_cache
        if cache[0] != self.location_epoch:
            cache = self._bi_cache = (self.location_epoch, {})
        hit = cache[1].get(block_id)
        if hit is None:
            bi = self.block_info_or_none(block_id)
            if bi is None or not bi.locations:
                return b"", m.length, False
            hit = (bi.SerializeToString(), bi.length, any(l.tierAlias == "MEM" for l in bi.locations))
            if cache[0] == self.location_epoch:
                cache[1][block_id] = hit
        return hit

    def commit_blocks_in_ufs_bulk(self, block_ids, lengths, fresh: bool = False) -> int:
        """Bulk form of :meth:`commit_blocks_in_ufs`: in-memory records for the new blocks and ONE
        natively encoded batched journal entry (csrc/meta_codec.cpp) instead of an entry object
        per block; returns how many were new.  ``fresh``: the ids belong to containers allocated
        for this call (they cannot exist yet), skip the existence check."""
        from ..journal.format import RawEntryBatch
        from ..ops.native import lib
        with self._lock:
            blocks = self._blocks
            if not fresh and any(b in blocks for b in block_ids):
                pairs = [(b, ln) for b, ln in zip(block_ids, lengths) if b not in blocks]
                new_ids, new_lens = [p[0] for p in pairs], [p[1] for p in pairs]
            else:
                new_ids, new_lens = list(block_ids), list(lengths)
            blocks.update(zip(new_ids, map(BlockMeta, new_lens)))
            if not new_ids:
                return 0
            self._bump_epoch()
            ctx = self._ctx()
            ctx.append(RawEntryBatch(lib().encode_block_info_batch(new_ids, new_lens), len(new_ids)))
        ctx.close()
        return len(new_ids)

    # ---- workers ------------------------------------------------------------------------------
    def get_worker_id(self, address) -> int:
        with self._lock:
            key = address_key(address)
            for s in (self._registered, self._temp):
                w = s.get_first_by_field("addr", key)
                if w is not None:
                    return w.id
            w = self._lost.get_first_by_field("addr", key)
            if w is not None:
                self._lost.remove(w)
                w.registered = False
                self._temp.add(w)
                return w.id
            wid = ids.get_random_non_negative_long()
            while self._registered.get_first_by_field("id", wid) or self._temp.get_first_by_field("id", wid):
                wid = ids.get_random_non_negative_long()
            self._temp.add(MasterWorkerInfo(wid, address))
            return wid

    def _find_worker(self, wid) -> MasterWorkerInfo | None:
        return self._registered.get_first_by_field("id", wid) or self._temp.get_first_by_field("id", wid)

    def worker_register(self, wid: int, tiers, total_on_tiers: dict, used_on_tiers: dict,
                        current_blocks: dict[tuple[str, str], list[int]], lost_storage: dict | None = None,
                        options=None) -> None:
        with self._lock:
            w = self._find_worker(wid)
            if w is None:
                w = self._lost.get_first_by_field("id", wid)
                if w is None:
                    raise NotFoundException(f"Could not find worker id: {wid} to register.")
                self._lost.remove(w)
            self._bump_epoch()
            self._temp.remove(w)
            self._registered.remove(w)
            w.registered = True
            w.storage_tiers = list(tiers)
            w.capacity = dict(total_on_tiers)
            w.used = dict(used_on_tiers)
            w.lost_storage = dict(lost_storage or {})
            w.last_updated_ms = int(time.time() * 1000)
            # replace the worker's block set with what it reports
            for bid in list(w.blocks):
                m = self._blocks.get(bid)
                if m is not None:
                    m.locations.pop(wid, None)
            w.blocks.clear()
            w.to_remove.clear()
            for (tier, medium), blist in current_blocks.items():
                for bid in blist:
                    self._add_location(w, bid, tier, medium)
            self._registered.add(w)
        for l in self.worker_registered_listeners:
            l(wid)
        LOG.info("registered worker %d at %s:%d", wid, w.address.host, w.address.rpcPort)

    def _add_location(self, w: MasterWorkerInfo, bid: int, tier: str, medium: str) -> None:
        m = self._blocks.get(bid)
        if m is None:
            # block unknown to the master (deleted meanwhile): ask the worker to drop it
            w.to_remove.add(bid)
            return
        if m.locations.get(w.id) != (tier, medium):
            m.locations[w.id] = (tier, medium)
            self._bump_epoch()
        w.blocks.add(bid)
        self._lost_blocks.discard(bid)

    def worker_heartbeat(self, wid: int, used_on_tiers: dict, removed: list[int],
                         added: dict[tuple[str, str], list[int]], metrics=None,
                         lost_storage: dict | None = None):
        """Returns (command_type, data) with command_type in Nothing/Register/Free."""
        with self._lock:
            w = self._registered.get_first_by_field("id", wid)
            if w is None:
                return "Register", []
            w.last_updated_ms = int(time.time() * 1000)
            w.used = dict(used_on_tiers)
            if lost_storage:
                w.lost_storage.update(lost_storage)
            if removed:
                self._bump_epoch()
            for bid in removed:
                m = self._blocks.get(bid)
                if m is not None:
                    m.locations.pop(wid, None)
                    if not m.locations:
                        self._lost_blocks.add(bid)
                w.blocks.discard(bid)
                w.to_remove.discard(bid)
            for (tier, medium), blist in added.items():
                for bid in blist:
                    self._add_location(w, bid, tier, medium)
            to_free = sorted(w.to_remove)
        if metrics and self.metrics is not None:
            self.metrics(w, metrics)
        if to_free:
            return "Free", to_free
        return "Nothing", []

    def commit_block(self, wid: int, used_on_tier: int, tier: str, medium: str, block_id: int,
                     length: int) -> None:
        ctx = None
        with self._lock:
            w = self._registered.get_first_by_field("id", wid)
            if w is None:
                raise NotFoundException(f"worker {wid} is not registered")
            m = self._blocks.get(block_id)
            if m is None or m.length != length:
                e = pb.journal.JournalEntry(block_info=pb.journal.BlockInfoEntry(block_id=block_id, length=length))
                self.process_journal_entry(e)
                ctx = self._ctx()
                ctx.append(e)
            self._add_location(w, block_id, tier, medium)
            w.used[tier] = used_on_tier
            w.last_updated_ms = int(time.time() * 1000)
        if ctx is not None:
            ctx.close()

    def commit_blocks(self, wid: int, block_ids, lengths, tier_index, tiers, mediums, used_on_tiers) -> None:
        """``commit_block`` for a batch from one worker (parallel arrays; ``tier_index[i]`` names
        ``tiers[k]`` / ``mediums[k]``): one lock section, one journal context (one flush) and one
        location-epoch bump for the lot -- the bulk-ingest commit path of ~100k blocks."""
        ctx = None
        changed = False
        with self._lock:
            w = self._registered.get_first_by_field("id", wid)
            if w is None:
                raise NotFoundException(f"worker {wid} is not registered")
            blocks, wblocks, lost = self._blocks, w.blocks, self._lost_blocks
            locs = [(t, m) for t, m in zip(tiers, mediums)]
            for bid, length, ti in zip(block_ids, lengths, tier_index):
                m = blocks.get(bid)
                if m is None or m.length != length:
                    e = pb.journal.JournalEntry(block_info=pb.journal.BlockInfoEntry(block_id=bid, length=length))
                    self.process_journal_entry(e)
                    if ctx is None:
                        ctx = self._ctx()
                    ctx.append(e)
                    m = blocks.get(bid)
                    if m is None:
                        w.to_remove.add(bid)
                        continue
                loc = locs[ti]
                if m.locations.get(w.id) != loc:
                    m.locations[w.id] = loc
                    changed = True
                wblocks.add(bid)
                lost.discard(bid)
            for t, used in used_on_tiers.items():
                w.used[t] = used
            w.last_updated_ms = int(time.time() * 1000)
            if changed:
                self._bump_epoch()
        if ctx is not None:
            ctx.close()

    def commit_block_in_ufs(self, block_id: int, length: int) -> None:
        self.commit_blocks_in_ufs([(block_id, length)])

    def commit_blocks_in_ufs(self, blocks) -> None:
        """Record (block id, length) pairs as stored in the UFS only: one journal context (one
        flush) for the whole batch (a metadata load of a big directory)."""
        ctx = None
        with self._lock:
            for block_id, length in blocks:
                if block_id in self._blocks:
                    continue
                e = pb.journal.JournalEntry(block_info=pb.journal.BlockInfoEntry(block_id=block_id, length=length))
                self.process_journal_entry(e)
                if ctx is None:
                    ctx = self._ctx()
                ctx.append(e)
        if ctx is not None:
            ctx.close()

    def remove_blocks(self, block_ids, delete: bool) -> None:
        """Remove replicas on workers; with ``delete`` also forget the block (journaled)."""
        ctx = None
        with self._lock:
            for bid in block_ids:
                m = self._blocks.get(bid)
                if m is None:
                    continue
                for wid in list(m.locations):
                    w = self._registered.get_first_by_field("id", wid)
                    if w is not None:
                        w.to_remove.add(bid)
                if delete:
                    e = pb.journal.JournalEntry(delete_block=pb.journal.DeleteBlockEntry(block_id=bid))
                    self.process_journal_entry(e)
                    if ctx is None:
                        ctx = self._ctx()
                    ctx.append(e)
                    self._lost_blocks.discard(bid)
        if ctx is not None:
            ctx.close()

    def remove_block_from_worker(self, block_id: int, wid: int) -> None:
        with self._lock:
            w = self._registered.get_first_by_field("id", wid)
            if w is not None:
                w.to_remove.add(block_id)

    def validate_block(self, block_id: int) -> bool:
        with self._lock:
            return block_id in self._blocks

    # ---- queries ------------------------------------------------------------------------------
    def block_info(self, block_id: int):
        with self._lock:
            m = self._blocks.get(block_id)
            if m is None:
                raise BlockDoesNotExistException(f"Block {block_id} does not exist")
            return self._gen_block_info(block_id, m)

    def block_info_or_none(self, block_id: int):
        with self._lock:
            m = self._blocks.get(block_id)
            return None if m is None else self._gen_block_info(block_id, m)

    def block_info_list(self, block_ids) -> list:
        with self._lock:
            out = []
            for bid in block_ids:
                m = self._blocks.get(bid)
                if m is not None:
                    out.append(self._gen_block_info(bid, m))
            return out

    def _gen_block_info(self, bid, m: BlockMeta):
        locs = []
        order = {t: i for i, t in enumerate(self.global_tiers)}
        for wid, (tier, medium) in sorted(m.locations.items(), key=lambda kv: order.get(kv[1][0], 99)):
            w = self._registered.get_first_by_field("id", wid)
            if w is None:
                continue
            locs.append(pb.grpc.BlockLocation(workerId=wid, workerAddress=w.address, tierAlias=tier,
                                              mediumType=medium))
        return pb.grpc.BlockInfo(blockId=bid, length=m.length, locations=locs)

    def block_length(self, block_id: int) -> int | None:
        with self._lock:
            m = self._blocks.get(block_id)
            return None if m is None else m.length

    def workers(self, live_only: bool = True) -> list[MasterWorkerInfo]:
        with self._lock:
            return list(self._registered) if live_only else list(self._registered) + list(self._lost)

    def worker_info_list(self):
        with self._lock:
            return [w.to_proto("In Service") for w in self._registered]

    def lost_workers_info_list(self):
        with self._lock:
            return [w.to_proto("Out of Service") for w in self._lost]

    def worker_count(self) -> int:
        return len(self._registered)

    def lost_worker_count(self) -> int:
        return len(self._lost)

    def capacity_bytes(self) -> int:
        return sum(w.capacity_bytes() for w in self.workers())

    def used_bytes(self) -> int:
        return sum(w.used_bytes() for w in self.workers())

    def capacity_on_tiers(self) -> dict:
        out: dict[str, int] = {}
        for w in self.workers():
            for k, v in w.capacity.items():
                out[k] = out.get(k, 0) + v
        return out

    def used_on_tiers(self) -> dict:
        out: dict[str, int] = {}
        for w in self.workers():
            for k, v in w.used.items():
                out[k] = out.get(k, 0) + v
        return out

    def lost_blocks(self) -> set[int]:
        with self._lock:
            return set(self._lost_blocks)

    def block_count(self) -> int:
        with self._lock:
            return len(self._blocks)

    def worker_lost_storage(self):
        out = []
        for w in self.workers():
            if w.lost_storage:
                info = pb.block.WorkerLostStorageInfo(address=w.address)
                for k, v in w.lost_storage.items():
                    info.lostStorage[k].storage.extend(v)
                out.append(info)
        return out

    # ---- failure detection --------------------------------------------------------------------
    def detect_lost_workers(self) -> list[int]:
        now = int(time.time() * 1000)
        lost = []
        with self._lock:
            for w in list(self._registered):
                if now - w.last_updated_ms > self.worker_timeout_ms:
                    LOG.warning("worker %d timed out after %d ms", w.id, now - w.last_updated_ms)
                    self._registered.remove(w)
                    self._process_lost(w)
                    self._lost.add(w)
                    lost.append(w.id)
        for wid in lost:
            for l in self.lost_worker_listeners:
                l(wid)
        return lost

    def _process_lost(self, w: MasterWorkerInfo) -> None:
        self._bump_epoch()
        for bid in w.blocks:
            m = self._blocks.get(bid)
            if m is not None:
                m.locations.pop(w.id, None)
                if not m.locations:
                    self._lost_blocks.add(bid)
        w.blocks.clear()
        w.registered = False

    def decommission_worker(self, wid: int) -> None:
        with self._lock:
            w = self._registered.get_first_by_field("id", wid)
            if w is not None:
                self._registered.remove(w)
                self._process_lost(w)
                self._lost.add(w)
