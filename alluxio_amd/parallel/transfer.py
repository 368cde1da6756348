"""Worker-to-worker block movement on one node: xGMI peer copies and RCCL collectives.

Reference data movement between workers is a gRPC ``ReadBlock`` stream copied chunk by chunk
(core/server/worker/.../block/RemoteBlockReader.java, AsyncCacheRequestManager.java:213-240,
job/server/.../plan/replicate/ReplicateDefinition.java + JobUtils.loadBlock).  On an MI355X node
every worker owns one GPU and the workers are ranks of one ``torch.distributed`` group, so:

* **on-demand moves** (async cache from a peer, replicate, passive cache) are *pulls over xGMI*:
  the destination asks the source for the block's device handle (``OpenDeviceBlock``: read lock +
  HIP IPC handle of the source arena + page list), reserves its own pages
  (``BlockStore.external_write``) and runs the batched page-gather kernel on its own GPU reading
  the peer's HBM directly.  No host staging, no RPC payload, and — unlike RCCL send/recv — no
  cross-process op ordering to get wrong: any number of pulls in any direction can be in flight.
* **bulk moves where every worker participates** (replicate a dataset onto every GPU, the
  ``distributedLoad --replication=all`` shape) are RCCL collectives: each rank contributes the
  blocks it holds to one ``all_gather_into_tensor`` per round, so all xGMI links carry traffic at
  once (C2/C4 in SURVEY §2.10).  Collectives are issued by every rank in the same order, so they
  cannot deadlock.

On CPU (gloo, DRAM tiers) pulls fall back to the gRPC block stream and collectives run on gloo,
which keeps the whole control flow testable without GPUs.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from datetime import timedelta

from ..proto import pb
from ..utils import ids

LOG = logging.getLogger(__name__)


def _addr_key(addr) -> str:
    if isinstance(addr, (tuple, list)):
        return f"{addr[0]}:{addr[1]}"
    if isinstance(addr, str):
        return addr
    return f"{addr.host}:{addr.rpcPort}"


def cross_page_segments(src_base: int, src_pages, src_ps: int, dst_base: int, dst_pages, dst_ps: int,
                        offset: int, length: int) -> list[tuple[int, int, int]]:
    """(src_ptr, dst_ptr, nbytes) segments copying block bytes [offset, offset+length) between two
    paged layouts (possibly different page sizes), merging runs contiguous on both sides."""
    segs: list[tuple[int, int, int]] = []
    pos, end = offset, offset + length
    while pos < end:
        spi, spo = divmod(pos, src_ps)
        dpi, dpo = divmod(pos, dst_ps)
        take = min(src_ps - spo, dst_ps - dpo, end - pos)
        s = src_base + src_pages[spi] * src_ps + spo
        d = dst_base + dst_pages[dpi] * dst_ps + dpo
        if segs and segs[-1][0] + segs[-1][2] == s and segs[-1][1] + segs[-1][2] == d:
            a, b, n = segs[-1]
            segs[-1] = (a, b, n + take)
        else:
            segs.append((s, d, take))
        pos += take
    return segs


class PlaneFailure(RuntimeError):
    """A transfer-plane collective did not complete: a member died, timed out, or another member
    already started rebuilding the group."""


def _new_group(backend: str, store, rank: int, world: int, timeout_s: float):
    """A process group for the plane's collectives with a bounded timeout.  RCCL groups are built
    with ``TORCH_NCCL_ASYNC_ERROR_HANDLING=2`` (CleanUpOnly): a failed or timed-out collective
    aborts the communicator and raises in the survivors instead of tearing their processes down
    (the default 3 kills the worker), so they can rebuild without the dead rank."""
    import os

    import torch.distributed as dist
    timeout = timedelta(seconds=timeout_s)
    if backend == "nccl":
        saved = {k: os.environ.get(k) for k in ("TORCH_NCCL_ASYNC_ERROR_HANDLING",)}
        os.environ["TORCH_NCCL_ASYNC_ERROR_HANDLING"] = "2"
        try:
            opts = dist.ProcessGroupNCCL.Options()
            try:
                opts._timeout = timeout
            except AttributeError:
                pass
            return dist.ProcessGroupNCCL(store, rank, world, opts)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    return dist.ProcessGroupGloo(store, rank, world, timeout)


class TransferPlane:
    """Peer block mover bound to one worker (one rank of the node's worker group).

    Collectives run on the plane's own process group (built over a prefixed view of the
    rendezvous store with a bounded timeout; :func:`_new_group`).  Every wait on a collective is
    bounded (:meth:`_await`: completion polling against ``timeout_s``, and against the store's
    rebuild marker, so a survivor blocked on a dead peer notices the others rebuilding within
    milliseconds); a failure aborts the communicator (``ProcessGroupNCCL.abort``) before the
    survivors agree on a new member list and build a new group (:meth:`_rebuild`)."""

    def __init__(self, worker, rank: int, world: int, addr_to_rank: dict[str, int], group=None, store=None,
                 rebuild_wait_s: float = 5.0, timeout_s: float = 60.0, batch_bytes: int = 256 << 20,
                 agree_every: int = 8):
        import torch.distributed as dist
        self.w = worker
        self.rank = rank
        self.world = world
        self.group = group
        self.addr_to_rank = dict(addr_to_rank)
        self.rank_to_addr = {r: a for a, r in self.addr_to_rank.items()}
        self.backend = dist.get_backend(group)
        self._collective_lock = threading.Lock()
        self.bytes_pulled = 0
        self.bytes_gathered = 0
        # membership: ``members`` are the original ranks of the current collective group, ``gen``
        # counts rebuilds; ``store`` (the rendezvous store) lets survivors of a dead rank agree on
        # a new group without it (None = a failed collective just raises)
        self.orig_rank = rank
        self.members = list(range(world))
        self.gen = 0
        self.store = store
        self.rebuild_wait_s = rebuild_wait_s
        self.timeout_s = timeout_s
        # ring rounds pack several blocks per owner up to batch_bytes; members agree on success
        # every agree_every rounds (one tiny all-reduce, no per-round host sync)
        self.batch_bytes = max(1, int(batch_bytes))
        self.agree_every = max(1, int(agree_every))
        self._pg = group if group is not None else dist.distributed_c10d._get_default_group()
        if group is None and store is not None:
            # the plane's own communicator: bounded timeout, survivable failures
            self._pg = _new_group(self.backend, dist.PrefixStore("alluxio/plane/gen0/pg/", store), rank, world,
                                  timeout_s)
        self.rebuilds = 0
        self.rounds = 0
        self.agreements = 0

    # ---- setup --------------------------------------------------------------------------------
    @classmethod
    def establish(cls, worker, group=None, store=None, rebuild_wait_s: float = 5.0,
                  timeout_s: float = 60.0, batch_bytes: int | None = None) -> "TransferPlane":
        """Collective: every rank of ``group`` calls this once after its worker has started.
        ``store`` defaults to the default group's rendezvous store (used to rebuild the group
        when a rank dies; see :meth:`_rebuild`)."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        allv = [None] * world
        dist.all_gather_object(allv, _addr_key(worker.address), group=group)
        if store is None and group is None:
            try:
                store = dist.distributed_c10d._get_default_store()
            except Exception:  # noqa: BLE001 - no store: no rebuild
                store = None
        if batch_bytes is None:
            batch_bytes = worker.conf.get_bytes("alluxio.worker.transfer.batch.bytes", "256MB")
        plane = cls(worker, rank, world, {a: r for r, a in enumerate(allv)}, group, store, rebuild_wait_s, timeout_s,
                    batch_bytes)
        worker.transfer_plane = plane
        if plane.backend == "nccl":
            import torch
            from ..ops.native import lib
            me = torch.cuda.current_device()
            for d in range(torch.cuda.device_count()):
                if d != me:
                    try:
                        lib().enable_peer_access(me, d)
                    except Exception:  # noqa: BLE001
                        LOG.debug("peer access %d->%d unavailable", me, d)
        return plane

    def rank_of(self, addr) -> int | None:
        return self.addr_to_rank.get(_addr_key(addr))

    def can_reach(self, addr) -> bool:
        r = self.rank_of(addr)
        return r is not None and r != self.orig_rank and r in self.members

    @property
    def device_plane(self) -> bool:
        """Pulls go GPU-to-GPU (IPC-mapped peer arena + copy kernel) when this worker has an HBM
        tier; independent of the collective backend, so gloo-coordinated workers sharing one
        GPU use it too."""
        return bool(self.w.store.has_device_tier) and self.w.conf.get_bool("alluxio.worker.ipc.enabled", "true")

    # ---- on-demand pulls ------------------------------------------------------------------------
    def pull_block(self, block_id: int, src, length: int, tier: int = 0, medium: str = "") -> int:
        """Copy ``block_id`` from peer worker ``src`` into this worker; returns bytes moved.
        Mapped (xGMI / shared-memory) pull with gRPC fallback: see :mod:`.peer`."""
        if not self.can_reach(src):
            raise ValueError(f"worker {_addr_key(src)} is not a peer in this transfer group")
        from .peer import pull_block
        n = pull_block(self.w, block_id, _addr_key(src), length, tier, medium, same_node=True)
        self.bytes_pulled += n
        return n

    def serve(self, req) -> None:
        """``PeerTransfer`` RPC: the requester (the block's holder, ``src_rank``) asks this worker to
        pull the block — used to fan a freshly written block out to replicas in parallel."""
        src = self.rank_to_addr.get(req.src_rank)
        if src is None:
            raise ValueError(f"unknown source rank {req.src_rank}")
        self.pull_block(req.block_id, src, req.length)

    # ---- bounded waits ---------------------------------------------------------------------------
    def _rebuild_requested(self) -> bool:
        """Another member started re-forming the group (a host-side store lookup, no GPU sync)."""
        if self.store is None:
            return False
        try:
            return bool(self.store.check([f"alluxio/plane/gen{self.gen + 1}/arrivals"]))
        except Exception:  # noqa: BLE001
            return False

    def _await(self, works, events=(), timeout_s: float | None = None) -> None:
        """Wait until every work (and CUDA event) completed, at most ``timeout_s``; raise
        :class:`PlaneFailure` on timeout, on a failed work, or once a rebuild has begun.
        RCCL works are polled (``is_completed`` queries their event), so a survivor blocked on a
        dead peer sees the others' rebuild marker within milliseconds.  gloo point-to-point works
        only complete inside ``wait``: they get one bounded wait each."""
        works = [w for w in works if w is not None]
        timeout_s = self.timeout_s if timeout_s is None else timeout_s
        if self.backend != "nccl":
            try:
                for w in works:
                    w.wait(timedelta(seconds=timeout_s))
            except Exception as e:  # noqa: BLE001 - a dead member fails (or stalls) the op
                raise PlaneFailure(str(e)) from e
            return
        deadline = time.monotonic() + timeout_s
        next_check = 0.0
        spin = 0
        while True:
            pending = [w for w in works if not w.is_completed()]
            if not pending and all(e.query() for e in events):
                for w in works:
                    w.wait()               # completed: returns at once, or raises its error
                return
            now = time.monotonic()
            if now > deadline:
                raise PlaneFailure(f"collective did not complete within {timeout_s:.0f}s")
            if now >= next_check:
                if self._rebuild_requested():
                    raise PlaneFailure("another member is rebuilding the transfer group")
                next_check = now + 0.02
            spin += 1
            time.sleep(0 if spin < 50 else 0.0002)

    def _abort_pg(self) -> None:
        """Abort the current communicator (RCCL: ncclCommAbort) so no kernel of the failed group
        stays queued behind a dead peer; then it is dropped for the rebuilt one."""
        pg = self._pg
        if self.group is not None and pg is self.group:
            return                      # a caller-owned group is the caller's to abort
        try:
            pg.abort()
        except Exception:  # noqa: BLE001 - gloo / already aborted
            LOG.debug("abort of the transfer group failed", exc_info=True)

    def _stream(self):
        import torch
        if self.backend == "nccl":
            return torch.cuda.current_stream()
        return None

    def _record(self):
        import torch
        if self.backend != "nccl":
            return None
        ev = torch.cuda.Event()
        ev.record()
        return ev

    # ---- collectives ----------------------------------------------------------------------------
    def replicate_all(self, blocks: list[tuple[int, int, int]]) -> int:
        """Collective: ``blocks`` = [(block_id, length, owner_rank)], identical on every rank.
        Afterwards every rank's worker holds every block.  One ``all_gather_into_tensor`` per
        round moves one batch (blocks packed up to ``batch_bytes``) from each owner to everyone
        (rounds = max batches per owner); the
        scatter of round k into pages is queued behind its all-gather on the stream and round k+1
        is issued before round k is waited for (two staging slots), so the GPU never idles
        between rounds.

        A rank that dies mid-way fails the round's collective on the others (bounded wait); with a
        rendezvous store they abort the communicator, rebuild the group among themselves
        (:meth:`_rebuild`) and redo the rounds from the earliest one any survivor failed in,
        without the dead rank's blocks (rounds are idempotent: blocks a rank already holds are
        skipped)."""
        by_owner: dict[int, list[tuple[int, int]]] = {}
        for bid, length, owner in blocks:
            by_owner.setdefault(owner, []).append((bid, length))
        moved = 0
        with self._collective_lock:
            k = 0
            while True:
                try:
                    moved += self._gather_rounds(by_owner, k)
                    break
                except Exception as e:  # noqa: BLE001
                    if self.store is None:
                        raise
                    moved += getattr(e, "moved", 0)
                    failed = getattr(e, "round", k)
                    LOG.warning("replicate_all: round %d failed (gen %d); rebuilding the group", failed, self.gen,
                                exc_info=True)
                    self._abort_pg()
                    k = self._rebuild(failed)
        self.bytes_gathered += moved
        return moved

    def _gather_rounds(self, by_owner, start: int) -> int:
        members = self.members
        # round k all-gathers every owner's k-th batch (consecutive blocks packed up to
        # batch_bytes): one collective per batch, not per block.  Batches depend only on
        # by_owner and batch_bytes, so the resume index stays valid across a rebuild.
        batches = [self._batches(by_owner.get(r, [])) for r in members]
        rounds = max((len(b) for b in batches), default=0)
        pending: list = []
        moved = 0
        k = start
        try:
            while k < rounds:
                if self._rebuild_requested():
                    raise PlaneFailure("another member is rebuilding the transfer group")
                entries = [batches[r][k] if k < len(batches[r]) else [] for r in range(len(members))]
                shard = max(sum(n for _, n in e) for e in entries)
                if shard == 0:
                    k += 1
                    continue
                send, out = self._staging(shard, slot=k % 2)
                if entries[self.rank]:     # bytes past a short batch are never read: no zero fill
                    self._copy_batch_out(entries[self.rank], send)
                work = self._pg._allgather_base(out, send)
                if self.backend == "nccl":
                    work.wait()            # the scatter queues behind the all-gather (no host wait)
                else:
                    self._await([work])    # host scatter needs the bytes; a gloo work is waited once
                    work = None
                opened = self._scatter_batches(out, shard, list(enumerate(entries)), skip_slot=self.rank)
                pending.append((k, [work], self._record(), opened))
                self.rounds += 1
                k += 1
                while len(pending) > 1:
                    moved += self._finish(pending.pop(0))
            while pending:
                moved += self._finish(pending.pop(0))
        except Exception as e:
            salvaged, failed = self._salvage(pending, k)
            if not isinstance(e, PlaneFailure):
                e = PlaneFailure(str(e))
            e.round, e.moved = failed, moved + salvaged
            raise e
        return moved

    def _salvage(self, pending, next_round: int) -> tuple[int, int]:
        """After a failure: commit the in-flight rounds that did complete (in order), abort the
        rest; returns (bytes committed, first round to redo)."""
        moved, failed = 0, next_round
        for i, item in enumerate(pending):
            k, works, ev, opened = item
            done = False
            if failed == next_round:
                try:
                    done = all(w.is_completed() for w in works if w is not None) and (ev is None or ev.query())
                    if done:
                        for w in works:
                            if w is not None:
                                w.wait()
                except Exception:  # noqa: BLE001 - the round's collective failed
                    done = False
            if done:
                moved += self._finish(item)
            else:
                failed = min(failed, k)
                self._abort_opened(opened)
        pending.clear()
        return moved, failed

    def replicate_ring(self, blocks: list[tuple[int, int, int]], copies: int) -> int:
        """Collective: ``blocks`` = [(block_id, length, owner_rank)], identical on every rank.
        Afterwards block b is held by its owner and the next ``copies - 1`` members after it (a
        ring).  Round k moves every owner's k-th *batch* (consecutive blocks packed up to
        ``batch_bytes``) with point-to-point RCCL send/recv: each rank sends to its ``copies - 1``
        successors and receives from its ``copies - 1`` predecessors, all posted in one coalesced
        group, so with copies=2 every xGMI link of the ring carries one batch per round in each
        direction and no rank receives bytes it will not keep (an all-gather would ship every
        block to all N ranks).  Rounds are pipelined two deep (round k+1 is posted before round k
        is waited for); failure is detected from the bounded wait itself, and the members agree
        on success with one all-reduce every ``agree_every`` rounds and at the end -- no
        per-round host sync.  The reference's replicate plan makes ``copies - 1`` separate gRPC
        block-stream copies per block (job/server/.../plan/replicate/ReplicateDefinition.java)."""
        copies = max(1, min(int(copies), len(self.members)))
        if copies == len(self.members):
            return self.replicate_all(blocks)
        by_owner: dict[int, list[tuple[int, int]]] = {}
        for bid, length, owner in blocks:
            by_owner.setdefault(owner, []).append((bid, length))
        moved = 0
        with self._collective_lock:
            while True:
                try:
                    moved += self._ring_rounds(by_owner, copies)
                    break
                except Exception as e:  # noqa: BLE001
                    if self.store is None:
                        raise
                    moved += getattr(e, "moved", 0)
                    LOG.warning("replicate_ring: round %s failed (gen %d); rebuilding the group",
                                getattr(e, "round", "?"), self.gen, exc_info=True)
                    self._abort_pg()
                    # the ring's neighbours changed: every round is redone over the new members
                    # (blocks a rank already holds are skipped when scattering)
                    self._rebuild(getattr(e, "round", 0))
        self.bytes_gathered += moved
        return moved

    def _batches(self, items: list[tuple[int, int]]) -> list[list[tuple[int, int]]]:
        out, cur, size = [], [], 0
        for bid, n in items:
            if cur and size + n > self.batch_bytes:
                out.append(cur)
                cur, size = [], 0
            cur.append((bid, n))
            size += n
        if cur:
            out.append(cur)
        return out

    def _ring_rounds(self, by_owner, copies: int) -> int:
        members, world, me = self.members, self.world, self.rank
        batches = [self._batches(by_owner.get(r, [])) for r in members]
        rounds = max((len(b) for b in batches), default=0)
        hops = range(1, min(copies, world))
        pending: list = []
        moved = 0
        k = 0
        failed_local = False
        # gloo point-to-point ops fail only on the dead rank's neighbours and cannot be polled:
        # there every round starts with the (cheap, host-side anyway) agreement all-reduce
        agree_every = 1 if self.backend != "nccl" else self.agree_every
        try:
            while k < rounds:
                if self._rebuild_requested():
                    raise PlaneFailure("another member is rebuilding the transfer group")
                entries = [batches[r][k] if k < len(batches[r]) else [] for r in range(world)]
                sizes = [sum(n for _, n in e) for e in entries]
                shard = max(sizes)
                if shard and hops:
                    send, out = self._staging(shard, slot=k % 2, nslots=len(hops))
                    if entries[me]:
                        self._copy_batch_out(entries[me], send)
                    works = self._ring_round(send, out, shard, sizes, hops, me, world, k)
                    if self.backend != "nccl":
                        self._await(works)     # gloo works complete inside wait, once
                        works = []
                    slots = [(h - 1, entries[(me - h) % world]) for h in hops]
                    opened = self._scatter_batches(out, shard, slots, skip_slot=-1)
                    pending.append((k, works, self._record(), opened))
                    self.rounds += 1
                    while len(pending) > 1:
                        moved += self._finish(pending.pop(0))
                k += 1
                if k % agree_every == 0 and k < rounds and self._agree(False):
                    raise PlaneFailure("a member failed a ring round")
            while pending:
                moved += self._finish(pending.pop(0))
        except Exception as e:
            failed_local = True
            salvaged, failed = self._salvage(pending, k)
            if not isinstance(e, PlaneFailure):
                e = PlaneFailure(str(e))
            e.round, e.moved = failed, moved + salvaged
            raise e
        # one agreement per call: a rank whose neighbour died must not be the only one to
        # rebuild while the others return as if nothing happened
        if not failed_local and self._agree(False):
            e = PlaneFailure("a member failed a ring round")
            e.round = 0
            raise e
        return moved

    def _agree(self, failed: bool) -> bool:
        """All-reduce of a failure flag over the members (bounded); True if any member failed.
        The flag is read on the host only after the bounded wait has seen it complete."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        flag = torch.tensor([1.0 if failed else 0.0], device=dev)
        w = self._pg.allreduce([flag])
        # bounded well below the rebuild window: a rank stuck on a dead reduction partner must
        # reach the rebuild while the others still wait for it
        self._await([w], [self._record()] if self.backend == "nccl" else (),
                    timeout_s=max(0.5, self.rebuild_wait_s / 2) if self.backend != "nccl" else None)
        self.agreements += 1
        return flag.item() > 0

    def _ring_round(self, send, out, shard, sizes, hops, me, world, k) -> list:
        # RCCL: one coalesced group on the group's communicator (ncclGroupStart/End), so no lazily
        # created per-pair communicator can deadlock the ring; gloo: receives are posted before
        # sends.  Returns the works (waited for by the caller, bounded).
        coalesce = send.is_cuda
        if coalesce:
            self._pg._start_coalescing(send.device)
        works = []
        for h in hops:      # receive slot h-1 <- predecessor me-h
            src = (me - h) % world
            if sizes[src]:
                works.append(self._pg.recv([out[(h - 1) * shard:(h - 1) * shard + sizes[src]]], src, k))
        if sizes[me]:
            for h in hops:
                works.append(self._pg.send([send[:sizes[me]]], (me + h) % world, k))
        if coalesce:
            works = [self._pg._end_coalescing(send.device)]
            for wk in works:
                if wk is not None:
                    wk.wait()          # stream dependency only: the scatter queues behind it
        return works

    def _finish(self, item) -> int:
        """Bounded wait for a round (its collective and its scatter), then commit its blocks."""
        _k, works, ev, opened = item
        self._await(works, [ev] if ev is not None else ())
        moved = 0
        while opened:
            session, bid, n = opened[0]
            self.w.commit_block(session, bid)
            opened.pop(0)
            moved += n
        return moved

    def _abort_opened(self, opened) -> None:
        for session, bid, _n in opened:
            try:
                self.w.abort_block(session, bid)
            except Exception:  # noqa: BLE001
                LOG.warning("abort of gathered block %d failed", bid, exc_info=True)
        opened.clear()

    def _rebuild(self, failed_round: int) -> int:
        """Re-form the collective group among the ranks still alive; returns the round to resume
        from.  Survivors check in under ``gen<g+1>/`` of the rendezvous store; the first to arrive
        waits up to ``rebuild_wait_s`` for the others, then publishes the member list and the
        resume round (the earliest any survivor failed in); everyone builds a new process group
        (bounded timeout, survivable errors: :func:`_new_group`) over a prefixed view of the store
        (no participation of the dead rank needed, unlike ``new_group``).  The caller aborted the
        old communicator first (:meth:`_abort_pg`)."""
        import torch.distributed as dist
        g = self.gen + 1
        st = self.store
        pre = f"alluxio/plane/gen{g}/"
        st.set(pre + f"alive/{self.orig_rank}", str(failed_round))
        if st.add(pre + "arrivals", 1) == 1:
            # sliding window: every new arrival extends the wait (stragglers blocked on a dead
            # peer reach this point a little later), up to 3x rebuild_wait_s in total
            t0 = time.time()
            deadline, seen = t0 + self.rebuild_wait_s, 1
            while time.time() < deadline:
                if all(st.check([pre + f"alive/{r}"]) for r in self.members):
                    break
                n = st.add(pre + "arrivals", 0)
                if n > seen:
                    seen = n
                    deadline = min(time.time() + self.rebuild_wait_s, t0 + 3 * self.rebuild_wait_s)
                time.sleep(0.05)
            alive = [r for r in self.members if st.check([pre + f"alive/{r}"])]
            resume = min(int(st.get(pre + f"alive/{r}")) for r in alive)
            st.set(pre + "members", json.dumps({"members": alive, "resume": resume}))
        else:
            st.wait([pre + "members"], timedelta(seconds=self.rebuild_wait_s * 2 + 30))
        plan = json.loads(st.get(pre + "members"))
        members = plan["members"]
        if self.orig_rank not in members:
            raise RuntimeError(f"rank {self.orig_rank} was left out of the rebuilt transfer group (gen {g})")
        rank = members.index(self.orig_rank)
        pg = _new_group(self.backend, dist.PrefixStore(pre + "pg/", st), rank, len(members), self.timeout_s)
        dead = [r for r in self.members if r not in members]
        self._pg = pg
        self.members = members
        self.rank, self.world, self.gen = rank, len(members), g
        self.rebuilds += 1
        LOG.warning("transfer group rebuilt (gen %d): members %s, lost %s, resuming at round %d", g, members, dead,
                    plan["resume"])
        return int(plan["resume"])

    def _staging(self, shard: int, slot: int = 0, nslots: int | None = None):
        """(send[shard], out[shard*nslots]) views of persistent buffers (two slots: round k+1 fills
        one while round k's scatter drains the other), grown geometrically: no allocation or
        zero-fill per round."""
        import torch
        nslots = self.world if nslots is None else nslots
        need = shard * (nslots + 1)
        bufs = getattr(self, "_stage", None)
        if bufs is None:
            bufs = self._stage = [None, None]
        buf = bufs[slot]
        if buf is None or buf.numel() < need:
            dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
            cap = max(need, 2 * (buf.numel() if buf is not None else 0))
            # gloo-coordinated workers with an HBM tier scatter out of this buffer with the GPU copy
            # kernel: it must be pinned (device-visible) host memory, never pageable
            pin = dev.type == "cpu" and bool(self.w.store.has_device_tier)
            buf = bufs[slot] = torch.empty(cap, dtype=torch.uint8, device=dev, pin_memory=pin)
        return buf[:shard], buf[shard:shard * (nslots + 1)]

    def _copy_batch_out(self, batch, dst) -> None:
        """Pack the blocks of ``batch`` back to back into ``dst`` with one batched read (queued on
        the current stream for a device buffer: the collective is ordered after it)."""
        kind = 1 if dst.is_cuda else 0
        base = dst.data_ptr()
        reqs, off = [], 0
        for bid, n in batch:
            reqs.append((bid, 0, n, base + off, kind))
            off += n
        if dst.is_cuda:
            import torch
            self.w.read_batch(reqs, torch.cuda.current_stream().cuda_stream, sync=False)
        else:
            self.w.read_batch(reqs, 0, sync=True)

    def _scatter_batches(self, out, shard: int, slots, skip_slot: int) -> list:
        """Reserve pages for every block received this round (``external_write``) and queue ONE
        batched page-scatter copy out of the staging buffer (device: on the current stream,
        behind the collective; host: synchronous).  ``slots`` = [(slot index, [(bid, n)...])] of
        packed batches; returns the opened temp blocks, committed by :meth:`_finish`."""
        from ..ops.native import lib
        base = out.data_ptr()
        segs, opened = [], []
        try:
            for slot, batch in slots:
                if slot == skip_slot:
                    continue
                off = 0
                for bid, n in batch:
                    at = off
                    off += n
                    if bid is None or self.w.has_block(bid):
                        continue
                    session = ids.create_session_id()
                    self.w.create_block(session, bid, 0, "", max(n, 1))
                    opened.append((session, bid, n))
                    pages = self.w.native.external_write(session, bid, 0, n)
                    _p, _d, dps, dbase = self.w.native.block_pages(bid)
                    segs.extend(cross_page_segments(base + slot * shard + at, [0], max(n, 1), dbase, list(pages),
                                                    dps, 0, n))
            if segs:
                if out.is_cuda:
                    import torch
                    with torch.cuda.device(out.device):
                        lib().batched_copy(segs, torch.cuda.current_stream().cuda_stream, False)
                else:
                    lib().batched_copy(segs, 0, True)
            return opened
        except Exception:
            self._abort_opened(opened)
            raise
