"""Embedded journal: the master journal replicated by Raft among the masters themselves.

Parity: core/server/common/src/main/java/alluxio/master/journal/raft/
  * RaftJournalSystem.java:150-860 — start/join quorum, gainPrimacy (catch-up protocol :542-615:
    write a unique primary-start id, wait until it is applied, then wait two election timeouts of
    quiet), losePrimacy (state rebuilt from the journal), checkpoint (:508 snapshot on demand),
    getQuorumServerInfoList (:686, AVAILABLE iff contacted within an election timeout),
    add/removeQuorumServer (:768-806), global sequence numbers (:461).
  * JournalStateMachine.java:83-620 — applies committed entries to the masters in order, drops
    duplicates by sequence number (:384-409), ignores applies while this master is primary
    (``upgrade``: the primary applied its own writes already), snapshot = every master's
    checkpoint + the last sequence number (:411), install resets and restores (:478).
  * RaftPrimarySelector.java — primacy follows Raft leadership.
  * RaftJournalWriter.java / AsyncJournalWriter — batched writes; a journal flush completes when
    the batch is committed by a majority (``write.timeout``).
  * RaftJournalServiceHandler / SnapshotUploader / SnapshotDownloader — snapshot transfer over
    ``RaftJournalService`` (see journal/raft.py).
Storage lives under ``<alluxio.master.journal.folder>/raft``.
"""
from __future__ import annotations

import logging
import os
import random
import shutil
import struct
import threading
import time

from ..proto import pb
from . import checkpoint as ck
from ..utils.exceptions import JournalClosedException, UnavailableException
from . import format as fmt
from .raft import (KIND_JOURNAL, KIND_PRIMARY_START, SVC_RAFT, SVC_RAFT_JOURNAL, LEADER, RaftNode,
                   RaftServiceHandler, RaftStorage)
from .system import JournalContext, JournalSystem, UfsJournalSystem

LOG = logging.getLogger(__name__)


def _hostport(a: str) -> str:
    a = a.strip()
    return a if ":" in a else f"{a}:19200"


class JournalStateMachine:
    def __init__(self, system: "RaftJournalSystem"):
        self.system = system
        self.next_sn = 0                 # next global sequence number expected
        self.ignore_applies = False
        self.last_primary_start = 0
        self.applied_entries = 0
        # delegated backup on a follower: entries are parked instead of applied, so the masters'
        # state can be brought to exactly the sequence the primary chose (JournalStateMachine
        # suspend / catchup / resume)
        self.suspended = False
        self._parked: list = []
        self._susp_lock = threading.Condition()

    def apply(self, index: int, payload: bytes) -> None:
        kind = payload[:1]
        if kind == KIND_JOURNAL:
            cmd = pb.raft.RaftCommand.FromString(payload[1:])
            for ne in cmd.entries:
                self._apply_entry(ne.master, ne.entry)
        elif kind == KIND_PRIMARY_START:
            self.last_primary_start = pb.raft.RaftCommand.FromString(payload[1:]).primaryStart

    def _apply_entry(self, master: str, e) -> None:
        sn = e.sequence_number
        if sn < self.next_sn:
            return                       # duplicate from a retried flush
        if sn > self.next_sn:
            LOG.error("journal gap: expected sequence number %d, got %d (%s)", self.next_sn, sn, master)
        self.next_sn = sn + 1
        self.applied_entries += 1
        if self.ignore_applies:
            return
        with self._susp_lock:
            if self.suspended:
                self._parked.append((master, e))
                self._susp_lock.notify_all()
                return
        self._apply_to_master(master, e)

    def _apply_to_master(self, master: str, e) -> None:
        comp = self.system._journaled.get(master)
        if comp is None:
            LOG.warning("journal entry for unknown master %s", master)
            return
        UfsJournalSystem._apply(comp, e)

    def suspend(self) -> None:
        with self._susp_lock:
            self.suspended = True

    def catchup(self, target_sn: int, timeout: float) -> None:
        """Apply parked entries with sequence number < ``target_sn``, waiting for them to arrive."""
        deadline = time.monotonic() + timeout
        with self._susp_lock:
            if not self.suspended:
                raise RuntimeError("catchup needs a suspended state machine")
            while True:
                keep = []
                for master, e in self._parked:
                    if e.sequence_number < target_sn:
                        self._apply_to_master(master, e)
                    else:
                        keep.append((master, e))
                self._parked = keep
                if self.next_sn >= target_sn:
                    return
                rem = deadline - time.monotonic()
                if rem <= 0:
                    raise TimeoutError(f"state machine catch-up to {target_sn} timed out at {self.next_sn}")
                self._susp_lock.wait(min(rem, 0.1))

    def resume(self) -> None:
        with self._susp_lock:
            for master, e in self._parked:
                self._apply_to_master(master, e)
            self._parked = []
            self.suspended = False

    def write_snapshot(self, path: str, index: int, term: int, peers) -> None:
        if self.suspended:
            raise RuntimeError("journal application is suspended (backup in progress)")
        comps = self.system.journaled
        hdr = pb.raft.RaftSnapshotHeader(index=index, term=term, peers=list(peers),
                                         nextSequenceNumber=self.next_sn, masters=sorted(comps))
        with open(path, "wb") as f:
            fmt.write_delimited(f, hdr)
            # JournalStateMachine snapshot: one COMPOUND over the masters, each master's own typed
            # checkpoint nested inside (JournalUtils.writeToCheckpoint(out, getStateMachines()))
            f.write(ck.compound([(fmt.CHECKPOINT_NAMES.get(n, n), ck.write_journaled(comps[n])) for n in sorted(comps)]))
            f.flush()
            os.fsync(f.fileno())

    def install_snapshot(self, path: str | None) -> list[str]:
        comps = self.system.journaled
        for c in comps.values():
            c.reset_state()
        if path is None:
            self.next_sn = 0
            return []
        with open(path, "rb") as f:
            hdr = fmt.read_delimited(f, pb.raft.RaftSnapshotHeader)
            pos = f.tell()
            head = f.read(8)
            f.seek(pos)
            typed = len(head) == 8 and 0 <= struct.unpack(">q", head)[0] <= max(fmt.CheckpointType)
            if typed:
                parts = fmt.read_compound(f)
            else:      # round-1 framing of this repo
                parts = [(n, ck.parse(ck.typed(fmt.CheckpointType.JOURNAL_ENTRY, d), n))
                         for n, d in fmt.read_legacy_compound(f)]
        for name, cp in parts:
            comp = comps.get(name)
            if comp is None:
                LOG.warning("snapshot has state for unknown master %s", name)
                continue
            ck.restore_journaled(comp, cp, UfsJournalSystem._apply)
        self.next_sn = hdr.nextSequenceNumber
        return list(hdr.peers)


class _RaftBatchWriter:
    """AsyncJournalWriter semantics over Raft: entries queue up, one flush thread batches them
    (``flush.batch.time``) into a single log entry and waits for its commit."""

    def __init__(self, system: "RaftJournalSystem", next_sn: int):
        self.system = system
        self.next_sn = next_sn
        self._cond = threading.Condition()
        self._queue: list = []
        self._appended = 0
        self._flushed = 0
        self._error: BaseException | None = None
        self._closed = False
        self._t = threading.Thread(target=self._run, daemon=True, name="raft-journal-flush")
        self._t.start()

    def append(self, master: str, entry) -> int:
        with self._cond:
            if self._closed:
                raise JournalClosedException("journal is closed")
            if self._error is not None:
                raise UnavailableException(f"journal write failed: {self._error}")
            if isinstance(entry, fmt.RawEntryBatch):
                e = entry.to_proto()
            else:
                e = pb.journal.JournalEntry()
                e.CopyFrom(entry)
            e.sequence_number = self.next_sn
            self.next_sn += 1
            self._queue.append(pb.raft.RaftNamedEntry(master=master, entry=e))
            self._appended += 1
            self._cond.notify_all()
            return self._appended

    def flush(self, counter: int) -> None:
        deadline = time.monotonic() + self.system.write_timeout + 5
        with self._cond:
            while self._flushed < counter:
                if self._error is not None:
                    raise UnavailableException(f"journal flush failed: {self._error}")
                if self._closed and self._flushed < counter and not self._queue:
                    raise JournalClosedException("journal closed before flush")
                rem = deadline - time.monotonic()
                if rem <= 0:
                    raise UnavailableException("journal flush timed out")
                self._cond.wait(min(rem, 0.05))

    def _run(self) -> None:
        while True:
            with self._cond:
                while not self._queue and not self._closed:
                    self._cond.wait(0.1)
                if not self._queue and self._closed:
                    return
            if self.system.flush_batch > 0:
                time.sleep(self.system.flush_batch)
            with self._cond:
                batch, self._queue = self._queue, []
            try:
                payload = KIND_JOURNAL + pb.raft.RaftCommand(entries=batch).SerializeToString()
                self.system.node.submit(payload, self.system.write_timeout)
                with self._cond:
                    self._flushed += len(batch)
                    self._cond.notify_all()
            except BaseException as e:  # noqa: BLE001
                LOG.warning("raft journal flush failed: %s", e)
                with self._cond:
                    self._error = e
                    self._cond.notify_all()
                self.system._on_write_failure(e)
                return

    def close(self) -> None:
        with self._cond:
            self._closed = True
            self._cond.notify_all()
        if self._t is not threading.current_thread():
            self._t.join(timeout=10)


class _ComponentWriter:
    def __init__(self, batch: _RaftBatchWriter, master: str):
        self.batch, self.master = batch, master

    def append(self, entry) -> int:
        return self.batch.append(self.master, entry)

    def flush(self, counter: int) -> None:
        self.batch.flush(counter)


class RaftPrimarySelector:
    """Primacy follows Raft leadership (RaftPrimarySelector.java)."""
    PRIMARY, SECONDARY = "PRIMARY", "SECONDARY"

    def __init__(self, system: "RaftJournalSystem"):
        self.system = system
        self._state = self.SECONDARY
        self._on_primary = self._on_secondary = None
        self._lock = threading.Lock()

    @property
    def state(self) -> str:
        return self._state

    def start(self, on_primary, on_secondary=None) -> None:
        self._on_primary, self._on_secondary = on_primary, on_secondary
        self.system.node.add_listener(self._changed)
        if self.system.node.is_leader():
            self._changed(True)

    def _changed(self, is_leader: bool) -> None:
        with self._lock:
            if is_leader and self._state != self.PRIMARY:
                self._state = self.PRIMARY
                try:
                    if self._on_primary is not None:
                        self._on_primary()
                except Exception:  # noqa: BLE001
                    LOG.exception("gaining primacy failed; stepping down")
                    self._state = self.SECONDARY
                    self.system.step_down()
                    if self._on_secondary is not None:
                        self._on_secondary()
            elif not is_leader and self._state == self.PRIMARY:
                self._state = self.SECONDARY
                if self._on_secondary is not None:
                    self._on_secondary()

    def wait_primary(self, timeout: float) -> bool:
        end = time.monotonic() + timeout
        while time.monotonic() < end:
            if self._state == self.PRIMARY and self.system.primary:
                return True
            time.sleep(0.02)
        return False

    def stop(self) -> None:
        self._on_primary = self._on_secondary = None
        self._state = self.SECONDARY

    halt = stop       # no lock to hold: just stop reacting to leadership changes


class RaftJournalSystem(JournalSystem):
    def __init__(self, root: str, local_address: str, cluster_addresses, *, conf=None, bind_host: str | None = None,
                 election_timeout_ms: float = 10_000, heartbeat_ms: float = 3_000, write_timeout_ms: float = 30_000,
                 flush_batch_ms: float = 5.0, snapshot_period_entries: int = 2_000_000,
                 append_batch_bytes: int = 512 << 10, snapshot_chunk_bytes: int = 4 << 20,
                 rpc_timeout_ms: float = 5_000, catchup_quiet_factor: float = 2.0, enable_grpc: bool = True,
                 fsync: bool = True, transport: str = "MESSAGING"):
        super().__init__()
        self.transport = transport
        self.root = root
        self.local = _hostport(local_address)
        self.single = not cluster_addresses
        self.cluster = [self.local] if self.single else sorted({_hostport(a) for a in cluster_addresses})
        self.conf = conf
        self.bind_host = bind_host
        self.election_timeout_ms = election_timeout_ms
        self.heartbeat_ms = heartbeat_ms
        self.write_timeout = write_timeout_ms / 1000.0
        self.flush_batch = flush_batch_ms / 1000.0
        self.snapshot_period = snapshot_period_entries
        self.append_batch_bytes = append_batch_bytes
        self.chunk = snapshot_chunk_bytes
        self.rpc_timeout_ms = rpc_timeout_ms
        self.quiet = catchup_quiet_factor
        self.enable_grpc = enable_grpc
        self.fsync = fsync
        self.sm = JournalStateMachine(self)
        self.node: RaftNode | None = None
        self.server = None
        self.selector = None
        self._writer: _RaftBatchWriter | None = None
        self._lock = threading.RLock()
        self._snapshot_allowed = True
        self._join_thread = None
        self._stopped = threading.Event()
        self.on_write_failure = None

    @classmethod
    def from_conf(cls, conf, folder: str, host: str | None = None, enable_grpc: bool = True,
                  ephemeral_port: bool = False):
        port = conf.get_int("alluxio.master.embedded.journal.port")
        host = host or conf.get_raw("alluxio.master.hostname") or "127.0.0.1"
        if host in ("0.0.0.0", ""):
            host = "127.0.0.1"
        addrs = conf.get_raw("alluxio.master.embedded.journal.addresses")
        cluster = [a for a in (addrs or "").split(",") if a.strip()]
        if ephemeral_port and not cluster:
            port = 0      # single master on an ephemeral RPC port (tests, embedded use)
        election = conf.get_ms("alluxio.master.embedded.journal.election.timeout")
        return cls(os.path.join(folder, "raft"), f"{host}:{port}", cluster, conf=conf,
                   bind_host=conf.get_raw("alluxio.master.embedded.journal.bind.host"),
                   election_timeout_ms=election,
                   heartbeat_ms=min(conf.get_ms("alluxio.master.embedded.journal.heartbeat.interval"), election / 2),
                   write_timeout_ms=conf.get_ms("alluxio.master.embedded.journal.write.timeout"),
                   flush_batch_ms=conf.get_ms("alluxio.master.journal.flush.batch.time"),
                   snapshot_period_entries=conf.get_int("alluxio.master.journal.checkpoint.period.entries"),
                   append_batch_bytes=conf.get_bytes("alluxio.master.embedded.journal.appender.batch.size"),
                   snapshot_chunk_bytes=conf.get_bytes("alluxio.master.embedded.journal.snapshot.replication.chunk.size"),
                   rpc_timeout_ms=conf.get_ms("alluxio.master.embedded.journal.transport.request.timeout.ms"),
                   enable_grpc=enable_grpc,
                   # consensus RPCs over MessagingService streams (the reference's transport) or
                   # one unary call each
                   transport=conf.get("alluxio.master.embedded.journal.transport.type", "MESSAGING"))

    # ---- format / state --------------------------------------------------------------------------
    def format(self) -> None:
        if os.path.isdir(self.root):
            shutil.rmtree(self.root)
        os.makedirs(self.root, exist_ok=True)

    def is_formatted(self) -> bool:
        return os.path.isdir(self.root)

    def is_empty(self) -> bool:
        if self.node is not None:
            # only the bootstrap entries (no-op / primary start) of this term so far
            return self.sm.next_sn == 0 and self.node.storage.snapshot_path is None
        return not os.path.isdir(self.root) or RaftStorage(self.root, fsync=False).is_empty()

    # ---- lifecycle -------------------------------------------------------------------------------
    def start(self) -> None:
        from ..rpc import Channel, RpcServer
        os.makedirs(self.root, exist_ok=True)
        self._stopped.clear()
        host, port = self.local.rsplit(":", 1)
        self.server = RpcServer(self.bind_host or host, int(port), max_workers=16, enable_grpc=self.enable_grpc,
                                conf=self.conf)
        handler = RaftServiceHandler(lambda: self.node, self._on_query)
        self.server.add_servicer(SVC_RAFT, handler)
        self.server.add_servicer(SVC_RAFT_JOURNAL, handler)
        from .messaging import SVC_MESSAGING, MessagingServiceHandler
        self.server.add_servicer(SVC_MESSAGING, MessagingServiceHandler(handler))
        addr = self.server.start()
        if self.single:
            # a lone master is the whole group, whatever address an earlier run recorded
            self.local = f"{host}:{addr.rsplit(':', 1)[1]}"
            self.cluster = [self.local]
        storage = RaftStorage(self.root, fsync=self.fsync)
        peers = self.sm.install_snapshot(storage.snapshot_path)
        initial = self.cluster if self.single else (peers or self.cluster)
        auth = None
        if self.conf is not None:
            from ..security.authentication import client_auth_from_conf
            auth = client_auth_from_conf(self.conf, None)

        def channel(addr):
            return Channel(addr, auth=auth) if auth is not None else Channel(addr, auth=None)

        self.node = RaftNode(self.local, initial, storage, self.sm, channel,
                             election_timeout_ms=self.election_timeout_ms, heartbeat_ms=self.heartbeat_ms,
                             rpc_timeout_ms=self.rpc_timeout_ms, append_batch_bytes=self.append_batch_bytes,
                             snapshot_chunk_bytes=self.chunk, snapshot_period_entries=self.snapshot_period,
                             snapshot_allowed=lambda: self._snapshot_allowed, transport=self.transport)
        if self.single:
            self.node._configs = [(storage.base_index, [self.local])]
        self.selector = RaftPrimarySelector(self)
        self.node.start()
        if self.local not in self.node.peers() and self.cluster:
            self._join_thread = threading.Thread(target=self._join_quorum, daemon=True, name="raft-join")
            self._join_thread.start()

    def _join_quorum(self) -> None:
        """A master outside the current configuration asks the leader to add it (joinQuorum)."""
        host, port = self.local.rsplit(":", 1)
        req = pb.meta.JournalQueryRequest(addQuorumServerRequest=pb.meta.AddQuorumServerRequest(
            serverAddress=pb.grpc.NetAddress(host=host, rpcPort=int(port))))
        while not self._stopped.is_set() and self.local not in self.node.peers():
            for peer in [p for p in self.node.peers() if p != self.local]:
                try:
                    self.node._call(peer, "JournalQuery", req)
                    break
                except Exception:  # noqa: BLE001
                    continue
            self._stopped.wait(self.election_timeout_ms / 1000.0)

    def _on_query(self, req):
        if req.HasField("addQuorumServerRequest"):
            a = req.addQuorumServerRequest.serverAddress
            self.add_quorum_server(f"{a.host}:{a.rpcPort}")
        if req.HasField("snapshotInfoRequest"):
            st = self.node.storage
            return pb.meta.JournalQueryResponse(snapshotInfoResponse=pb.meta.GetSnapshotInfoResponse(
                latest=pb.meta.SnapshotMetadata(snapshotTerm=st.base_term, snapshotIndex=st.base_index)))
        return pb.meta.JournalQueryResponse()

    def stop(self) -> None:
        self._stopped.set()
        self._close_writer()
        if self.server is not None:
            self.server.stop()
            self.server = None
        if self.node is not None:
            self.node.stop()

    # ---- primacy ---------------------------------------------------------------------------------
    def gain_primacy(self) -> None:
        """Catch up on everything committed before this term, then take over writing."""
        node = self.node
        timeout = max(30.0, 20 * node.T)
        if self.sm.suspended:           # a delegated backup was in flight on this follower
            self.sm.resume()
        self._snapshot_allowed = False
        while True:
            if not node.is_leader():
                raise UnavailableException("lost raft leadership while catching up")
            before = self.sm.applied_entries
            marker = random.randint(1, (1 << 62))
            payload = KIND_PRIMARY_START + pb.raft.RaftCommand(primaryStart=marker).SerializeToString()
            idx = node.submit(payload, timeout)
            if not node.wait_applied(idx, timeout):
                continue
            if node.peers() != [self.local]:      # alone in the group: nobody else can lead
                time.sleep(self.quiet * node.T)
            if self.sm.last_primary_start == marker and self.sm.applied_entries == before:
                break
        with self._lock:
            self.sm.ignore_applies = True
            self._writer = _RaftBatchWriter(self, self.sm.next_sn)
        super().gain_primacy()

    def lose_primacy(self) -> None:
        self._close_writer()
        super().lose_primacy()
        with self._lock:
            self.sm.ignore_applies = False
        # the masters may hold writes that never committed: rebuild them from the journal
        self.node.reset_applied_to_snapshot()
        self._snapshot_allowed = True

    def step_down(self) -> None:
        node = self.node
        with node._lock:
            if node.role == LEADER:
                node._become_follower(node.storage.term, None)

    def _on_write_failure(self, e) -> None:
        if self.on_write_failure is not None:
            threading.Thread(target=self.on_write_failure, args=(e,), daemon=True).start()
        else:
            self.step_down()

    def _close_writer(self) -> None:
        with self._lock:
            w, self._writer = self._writer, None
        if w is not None:
            w.close()

    def create_context(self, name: str, state_lock=None) -> JournalContext:
        w = self._writer
        if w is None:
            raise UnavailableException(f"journal for {name} is not writable (not primary)")
        return JournalContext(_ComponentWriter(w, name), state_lock)

    # ---- checkpoints -----------------------------------------------------------------------------
    def checkpoint(self) -> None:
        """Snapshot now.  On the primary the caller holds the master state lock exclusively, so
        every journaled change is flushed and the live state equals the committed log."""
        node = self.node
        w = self._writer
        if w is not None:
            w.flush(w._appended)
            with node._lock:
                last = node.storage.last_index()
            node.wait_applied(last, self.write_timeout)
            with node._apply_lock:
                with node._lock:
                    idx = node.last_applied
                    term = node.storage.term_at(idx)
                    peers = node._config_at(idx)
                    tmp = node.storage.new_snapshot_tmp()
                self.sm.write_snapshot(tmp, idx, term, peers)
                with node._lock:
                    if idx > node.storage.base_index:
                        node.storage.install_snapshot(tmp, idx, term)
                        node._configs = [(idx, peers)] + [c for c in node._configs if c[0] > idx]
                    elif os.path.exists(tmp):
                        os.remove(tmp)
        else:
            node.take_snapshot()

    def sequence_numbers(self) -> dict[str, int]:
        sn = (self._writer.next_sn if self._writer is not None else self.sm.next_sn)
        return {name: sn for name in self.journaled}

    def suspend(self) -> None:
        if self._writer is not None:
            raise RuntimeError("cannot suspend the primary's journal")
        self._snapshot_allowed = False
        self.sm.suspend()

    def catchup(self, sequences: dict[str, int], timeout: float = 60.0) -> None:
        # one global sequence across masters: the requested point is the largest of them
        self.sm.catchup(max(sequences.values(), default=0), timeout)

    def resume(self) -> None:
        self.sm.resume()
        self._snapshot_allowed = True

    # ---- quorum management -----------------------------------------------------------------------
    def quorum_info(self) -> list[tuple[str, bool]]:
        st = self.node.status()
        out = []
        for p in st["peers"]:
            if p == self.local:
                out.append((p, True))
            else:
                age = st["contact_s"].get(p)
                out.append((p, age is not None and age < 2 * self.node.T))
        return out

    def add_quorum_server(self, address: str) -> None:
        address = _hostport(address)
        peers = set(self.node.peers())
        if address in peers:
            return
        self.node.change_peers(peers | {address}, self.write_timeout)

    def remove_quorum_server(self, address: str) -> None:
        address = _hostport(address)
        peers = set(self.node.peers())
        if address not in peers:
            return
        self.node.change_peers(peers - {address}, self.write_timeout)

    def transfer_leadership(self, address: str, timeout: float = 10.0) -> bool:
        return self.node.transfer_leadership(_hostport(address), timeout)

    def is_leader(self) -> bool:
        return self.node is not None and self.node.is_leader()
