"""Raft consensus for the embedded journal: durable log + snapshots, elections, replication.

Parity: the reference embeds Apache Ratis (core/server/common/src/main/java/alluxio/master/
journal/raft/RaftJournalSystem.java:150-860 configures it: election timeout min/max, heartbeat,
appender batch size, snapshot chunking; SnapshotReplicationManager / SnapshotDownloader /
SnapshotUploader move snapshots over RaftJournalService).  Ratis is a Java library, so this
module is the consensus core itself, written for the master's control plane:

* ``RaftStorage`` — ``meta.json`` (current term + vote, fsynced before answering), one append-only
  ``log`` file of CRC-framed records (torn tails are cut on load), ``snapshot.<term>_<index>``
  files; a snapshot compacts the log prefix it covers.
* ``RaftNode`` — follower / candidate / leader with randomised election timeouts in [T, 2T],
  PreVote + leader stickiness (a partitioned node that comes back cannot depose a healthy leader),
  CheckQuorum (a leader that lost contact with a majority steps down), per-peer replicator threads
  with byte-bounded batches, conflict-index back-off, snapshot push (InstallSnapshot over
  ``RaftJournalService.UploadSnapshot``), single-server membership changes (config entries take
  effect when appended), leadership transfer (TimeoutNow) and an applier thread that feeds
  committed entries to the state machine in order.

Payloads are opaque bytes with a one-byte kind prefix (``J`` journal batch, ``P`` primary-start
marker, ``N`` no-op, ``C`` configuration) so membership changes are visible without parsing
journal batches.
"""
from __future__ import annotations

import json
import logging
import os
import random
import struct
import threading
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

from ..proto import pb
from ..utils.exceptions import UnavailableException

LOG = logging.getLogger(__name__)

FOLLOWER, CANDIDATE, LEADER = "FOLLOWER", "CANDIDATE", "LEADER"
KIND_JOURNAL, KIND_PRIMARY_START, KIND_NOOP, KIND_CONFIG = b"J", b"P", b"N", b"C"
SVC_RAFT = "alluxio.grpc.raft.RaftServerService"
SVC_RAFT_JOURNAL = "alluxio.grpc.meta.RaftJournalService"

_REC = struct.Struct("<IIQQ")   # payload length, crc32(payload), index, term


class NotLeaderException(UnavailableException):
    def __init__(self, leader: str | None):
        super().__init__(f"not the raft leader (leader: {leader})")
        self.leader = leader


def config_payload(peers) -> bytes:
    return KIND_CONFIG + pb.raft.RaftCommand(peers=sorted(peers)).SerializeToString()


def parse_config(payload: bytes) -> list[str]:
    return list(pb.raft.RaftCommand.FromString(payload[1:]).peers)


class RaftStorage:
    """Durable Raft state of one server."""

    def __init__(self, root: str, fsync: bool = True):
        self.root = root
        self.fsync = fsync
        os.makedirs(root, exist_ok=True)
        self.term = 0
        self.voted_for: str | None = None
        self.base_index = 0
        self.base_term = 0
        self.snapshot_path: str | None = None
        self._terms: list[int] = []
        self._payloads: list[bytes] = []
        self._offsets: list[int] = []
        self._f = None
        self._load()

    # ---- paths ---------------------------------------------------------------------------------
    @property
    def _meta(self) -> str:
        return os.path.join(self.root, "meta.json")

    @property
    def _log(self) -> str:
        return os.path.join(self.root, "log")

    def snapshots(self) -> list[tuple[int, int, str]]:
        out = []
        for n in os.listdir(self.root):
            if n.startswith("snapshot.") and not n.endswith(".tmp"):
                try:
                    t, i = n[len("snapshot."):].split("_")
                    out.append((int(i), int(t), os.path.join(self.root, n)))
                except ValueError:
                    continue
        return sorted(out)

    def _sync(self, f) -> None:
        f.flush()
        if self.fsync:
            os.fsync(f.fileno())

    # ---- load / persist ------------------------------------------------------------------------
    def _load(self) -> None:
        if os.path.exists(self._meta):
            with open(self._meta) as f:
                m = json.load(f)
            self.term, self.voted_for = int(m.get("term", 0)), m.get("votedFor")
        snaps = self.snapshots()
        if snaps:
            self.base_index, self.base_term, self.snapshot_path = snaps[-1]
        good = 0
        if os.path.exists(self._log):
            with open(self._log, "rb") as f:
                data = f.read()
            pos = 0
            while pos + _REC.size <= len(data):
                ln, crc, idx, term = _REC.unpack_from(data, pos)
                end = pos + _REC.size + ln
                if end > len(data):
                    break
                payload = data[pos + _REC.size:end]
                if zlib.crc32(payload) != crc:
                    break
                if idx > self.base_index:
                    if idx != self.last_index() + 1:
                        break
                    self._terms.append(term)
                    self._payloads.append(payload)
                    self._offsets.append(pos)
                pos = end
            good = pos
            if good < len(data):
                LOG.warning("raft log %s: cutting %d torn/corrupt tail bytes", self._log, len(data) - good)
                with open(self._log, "r+b") as f:
                    f.truncate(good)
        self._f = open(self._log, "ab")

    def save_meta(self, term: int, voted_for: str | None) -> None:
        self.term, self.voted_for = term, voted_for
        tmp = self._meta + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"term": term, "votedFor": voted_for}, f)
            self._sync(f)
        os.replace(tmp, self._meta)

    # ---- log -----------------------------------------------------------------------------------
    def last_index(self) -> int:
        return self.base_index + len(self._terms)

    def last_term(self) -> int:
        return self._terms[-1] if self._terms else self.base_term

    def term_at(self, i: int) -> int | None:
        if i == self.base_index:
            return self.base_term
        k = i - self.base_index - 1
        if k < 0 or k >= len(self._terms):
            return None
        return self._terms[k]

    def payload_at(self, i: int) -> bytes:
        return self._payloads[i - self.base_index - 1]

    def entries(self, start: int, end: int | None = None, max_bytes: int = 1 << 62) -> list[tuple[int, int, bytes]]:
        """[(index, term, payload)] for start..end inclusive, at least one entry, ≤ max_bytes."""
        end = self.last_index() if end is None else min(end, self.last_index())
        out, size = [], 0
        for i in range(max(start, self.base_index + 1), end + 1):
            p = self._payloads[i - self.base_index - 1]
            if out and size + len(p) > max_bytes:
                break
            out.append((i, self._terms[i - self.base_index - 1], p))
            size += len(p)
        return out

    def append(self, items, sync: bool = True) -> int:
        for term, payload in items:
            idx = self.last_index() + 1
            self._offsets.append(self._f.tell())
            self._f.write(_REC.pack(len(payload), zlib.crc32(payload), idx, term))
            self._f.write(payload)
            self._terms.append(term)
            self._payloads.append(payload)
        if sync:
            self._sync(self._f)
        return self.last_index()

    def truncate_from(self, i: int) -> None:
        """Drop entries with index ≥ i (conflict with the leader's log)."""
        k = i - self.base_index - 1
        if k < 0 or k >= len(self._terms):
            return
        self._f.flush()
        os.ftruncate(self._f.fileno(), self._offsets[k])
        self._f.seek(0, os.SEEK_END)
        del self._terms[k:], self._payloads[k:], self._offsets[k:]

    def _rewrite(self, keep_from: int) -> None:
        """Rewrite the log keeping entries with index ≥ keep_from (index > new base)."""
        k = max(0, keep_from - self.base_index - 1)
        terms, payloads = self._terms[k:], self._payloads[k:]
        first = self.base_index + 1 + k
        tmp = self._log + ".tmp"
        offsets = []
        with open(tmp, "wb") as f:
            for n, (t, p) in enumerate(zip(terms, payloads)):
                offsets.append(f.tell())
                f.write(_REC.pack(len(p), zlib.crc32(p), first + n, t))
                f.write(p)
            self._sync(f)
        self._f.close()
        os.replace(tmp, self._log)
        self._f = open(self._log, "ab")
        self._terms, self._payloads, self._offsets = terms, payloads, offsets

    def install_snapshot(self, tmp_path: str, index: int, term: int) -> None:
        """Adopt ``tmp_path`` as the snapshot at (index, term); compact the log it covers."""
        path = os.path.join(self.root, f"snapshot.{term}_{index}")
        os.replace(tmp_path, path)
        if self.fsync:
            fd = os.open(self.root, os.O_RDONLY)
            try:
                os.fsync(fd)
            finally:
                os.close(fd)
        if self.term_at(index) == term:
            self._rewrite(index + 1)            # keep the suffix after the snapshot
        else:
            self._rewrite(self.last_index() + 1)   # log diverges or is behind: discard it all
        self.base_index, self.base_term, self.snapshot_path = index, term, path
        for i, _t, p in self.snapshots()[:-2]:   # keep the newest two
            if p != path:
                try:
                    os.remove(p)
                except OSError:
                    pass

    def new_snapshot_tmp(self) -> str:
        return os.path.join(self.root, f"snapshot.{os.getpid()}.{threading.get_ident()}.tmp")

    def is_empty(self) -> bool:
        return self.snapshot_path is None and not self._terms

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None


class RaftNode:
    """One Raft server.

    ``state_machine`` provides ``apply(index, payload)``, ``write_snapshot(path, index, term, peers)``
    and ``install_snapshot(path) -> peers``; ``channel_factory(address)`` returns a
    ``rpc.Channel``-like object with ``stub(service)``.
    """

    def __init__(self, self_id: str, initial_peers, storage: RaftStorage, state_machine, channel_factory, *,
                 election_timeout_ms: float = 10_000, heartbeat_ms: float = 3_000,
                 rpc_timeout_ms: float = 5_000, append_batch_bytes: int = 512 << 10,
                 snapshot_chunk_bytes: int = 4 << 20, snapshot_period_entries: int = 2_000_000,
                 snapshot_allowed=None, transport: str = "UNARY"):
        self.id = self_id
        # "MESSAGING": consensus RPCs go through one MessagingService.connect stream per peer
        # (journal/messaging.py, the reference's transport); "UNARY": one gRPC call each
        self.transport = transport.upper()
        self._msg_conns: dict = {}
        self.storage = storage
        self.sm = state_machine
        self._channel_factory = channel_factory
        self.T = election_timeout_ms / 1000.0
        self.heartbeat = heartbeat_ms / 1000.0
        self.rpc_timeout = rpc_timeout_ms / 1000.0
        self.batch_bytes = append_batch_bytes
        self.chunk = snapshot_chunk_bytes
        self.snapshot_period = snapshot_period_entries
        self.snapshot_allowed = snapshot_allowed or (lambda: True)
        self._lock = threading.RLock()
        self._cond = threading.Condition(self._lock)
        self._apply_lock = threading.Lock()
        self._stop = threading.Event()
        self.role = FOLLOWER
        self.leader_id: str | None = None
        self.commit_index = storage.base_index
        self.last_applied = storage.base_index
        self._configs: list[tuple[int, list[str]]] = [(storage.base_index, sorted(set(initial_peers)))]
        for idx, _t, p in storage.entries(storage.base_index + 1):
            if p[:1] == KIND_CONFIG:
                self._configs.append((idx, parse_config(p)))
        self._next: dict[str, int] = {}
        self._match: dict[str, int] = {}
        self._contact: dict[str, float] = {}
        self._replicators: dict[str, threading.Thread] = {}
        self._transfer_target: str | None = None
        self._last_heard = time.monotonic()
        self._deadline = 0.0
        self._reset_deadline()
        self._channels: dict[str, object] = {}
        self._pool = ThreadPoolExecutor(max_workers=32, thread_name_prefix=f"raft-{self_id}")
        self._listeners = []
        self._events: list[bool] = []
        self._threads: list[threading.Thread] = []
        self.snapshot_installs = 0

    # ---- configuration -------------------------------------------------------------------------
    def peers(self) -> list[str]:
        return self._configs[-1][1]

    def set_base_config(self, peers) -> None:
        """Peers recorded in the snapshot the state machine was restored from."""
        with self._lock:
            tail = [c for c in self._configs if c[0] > self.storage.base_index]
            self._configs = [(self.storage.base_index, sorted(set(peers)))] + tail

    def _config_at(self, index: int) -> list[str]:
        peers = self._configs[0][1]
        for i, p in self._configs:
            if i <= index:
                peers = p
        return peers

    def _others(self) -> list[str]:
        return [p for p in self.peers() if p != self.id]

    def _quorum(self, voters) -> int:
        return len(voters) // 2 + 1

    # ---- lifecycle -----------------------------------------------------------------------------
    def add_listener(self, fn) -> None:
        """``fn(is_leader: bool)`` — called in order from one notifier thread."""
        self._listeners.append(fn)

    def start(self) -> None:
        self._stop.clear()
        for name, fn in (("tick", self._tick_loop), ("apply", self._apply_loop), ("notify", self._notify_loop)):
            t = threading.Thread(target=fn, name=f"raft-{name}-{self.id}", daemon=True)
            t.start()
            self._threads.append(t)
        with self._lock:
            # a one-member group elects itself at once (no other voter can exist)
            if self.peers() == [self.id]:
                self._become_candidate(pre_vote=False)
                self._become_leader()

    def stop(self) -> None:
        self._stop.set()
        with self._lock:
            self._cond.notify_all()
        for t in self._threads + list(self._replicators.values()):
            if t is not threading.current_thread():
                t.join(timeout=5)
        self._threads.clear()
        self._pool.shutdown(wait=False, cancel_futures=True)
        for ch in list(self._channels.values()):
            try:
                ch.close()
            except Exception:  # noqa: BLE001
                pass
        self._channels.clear()
        for c in list(self._msg_conns.values()):
            c.close()
        self._msg_conns.clear()
        with self._lock:
            self.role = FOLLOWER
            self._replicators.clear()
        self.storage.close()

    # ---- transport -----------------------------------------------------------------------------
    def _call(self, peer: str, method: str, req, service: str = SVC_RAFT):
        ch = self._channels.get(peer)
        if ch is None:
            ch = self._channels[peer] = self._channel_factory(peer)
        if self.transport == "MESSAGING" and service == SVC_RAFT and method != "JournalQuery":
            from .messaging import MessagingConnection
            conn = self._msg_conns.get(peer)
            try:
                if conn is None or conn.closed:
                    conn = self._msg_conns[peer] = MessagingConnection(ch)
                return conn.call(method, req, self.rpc_timeout)
            except Exception:
                c = self._msg_conns.pop(peer, None)
                if c is not None:
                    c.close()
                self._channels.pop(peer, None)     # a restarted peer needs a fresh channel
                try:
                    ch.close()
                except Exception:  # noqa: BLE001
                    pass
                raise
        try:
            return getattr(ch.stub(service), method)(req, timeout=self.rpc_timeout)
        except Exception:
            self._channels.pop(peer, None)
            try:
                ch.close()
            except Exception:  # noqa: BLE001
                pass
            raise

    # ---- timers & elections --------------------------------------------------------------------
    def _reset_deadline(self) -> None:
        self._deadline = time.monotonic() + random.uniform(self.T, 2 * self.T)

    def _tick_loop(self) -> None:
        tick = max(0.005, min(0.05, self.T / 10))
        while not self._stop.wait(tick):
            start = None
            with self._lock:
                now = time.monotonic()
                if self.role == LEADER:
                    # CheckQuorum: a leader cut off from a majority steps down
                    voters = self.peers()
                    alive = sum(1 for p in voters if p == self.id or now - self._contact.get(p, 0) < 2 * self.T)
                    if alive < self._quorum(voters) and now - self._leader_since > 2 * self.T:
                        LOG.warning("raft %s: lost contact with a majority, stepping down", self.id)
                        self._become_follower(self.storage.term, None)
                elif now >= self._deadline and self.id in self.peers():
                    self._reset_deadline()
                    start = self.storage.term
            if start is not None:
                self._pool.submit(self._election, True, False)

    def _election(self, pre_vote: bool, transfer: bool) -> None:
        with self._lock:
            if self.role == LEADER or self._stop.is_set():
                return
            if pre_vote:
                term = self.storage.term + 1      # the term we would campaign in (nothing persisted)
            else:
                self._become_candidate(pre_vote=False)
                term = self.storage.term
            voters = self.peers()
            if len(voters) == 1 and voters[0] == self.id:
                if pre_vote:
                    self._become_candidate(pre_vote=False)
                self._become_leader()
                return
            req = pb.raft.RequestVotePRequest(term=term, candidateId=self.id, lastLogIndex=self.storage.last_index(),
                                              lastLogTerm=self.storage.last_term(), preVote=pre_vote,
                                              transfer=transfer)
        votes = 1 if self.id in voters else 0
        need = self._quorum(voters)
        futs = [self._pool.submit(self._call, p, "RequestVote", req) for p in voters if p != self.id]
        deadline = time.monotonic() + self.rpc_timeout
        for f in futs:
            try:
                r = f.result(timeout=max(0.0, deadline - time.monotonic()))
            except Exception:  # noqa: BLE001
                continue
            with self._lock:
                if (r.term >= term) if pre_vote else (r.term > self.storage.term):
                    self._become_follower(r.term, None)     # we are behind: adopt the newer term
                    return
                if r.granted:
                    votes += 1
            if votes >= need:
                break
        with self._lock:
            if votes < need or self._stop.is_set():
                return
            if pre_vote:
                if self.role != FOLLOWER and self.role != CANDIDATE:
                    return
                # pre-vote won: campaign for real (in a fresh task to keep lock scopes short)
                self._pool.submit(self._election, False, transfer)
                return
            if self.role == CANDIDATE and self.storage.term == term:
                self._become_leader()

    def _become_candidate(self, pre_vote: bool) -> None:
        self.role = CANDIDATE
        self.leader_id = None
        self.storage.save_meta(self.storage.term + 1, self.id)
        self._reset_deadline()

    def _become_follower(self, term: int, leader: str | None) -> None:
        was_leader = self.role == LEADER
        if term > self.storage.term:
            self.storage.save_meta(term, None)
        self.role = FOLLOWER
        self.leader_id = leader
        self._transfer_target = None
        self._replicators.clear()
        self._reset_deadline()
        self._cond.notify_all()
        if was_leader:
            self._emit(False)

    def _become_leader(self) -> None:
        LOG.info("raft %s: leader for term %d", self.id, self.storage.term)
        self.role = LEADER
        self.leader_id = self.id
        self._leader_since = time.monotonic()
        last = self.storage.last_index()
        now = time.monotonic()
        for p in self._others():
            self._next[p] = last + 1
            self._match[p] = 0
            self._contact[p] = now
        # a no-op in the new term commits everything before it (Raft §5.4.2)
        self.storage.append([(self.storage.term, KIND_NOOP)])
        self._advance_commit()
        self._sync_replicators()
        self._emit(True)

    def _sync_replicators(self) -> None:
        term = self.storage.term
        for p in self._others():
            t = self._replicators.get(p)
            if t is None or not t.is_alive():
                self._next.setdefault(p, self.storage.last_index() + 1)
                self._match.setdefault(p, 0)
                self._contact.setdefault(p, time.monotonic())
                t = threading.Thread(target=self._replicate, args=(p, term), daemon=True,
                                     name=f"raft-repl-{self.id}->{p}")
                self._replicators[p] = t
                t.start()
        self._cond.notify_all()

    def _emit(self, is_leader: bool) -> None:
        self._events.append(is_leader)
        self._cond.notify_all()

    def _notify_loop(self) -> None:
        while not self._stop.is_set():
            with self._lock:
                while not self._events and not self._stop.is_set():
                    self._cond.wait(0.1)
                if self._stop.is_set():
                    return
                ev = self._events.pop(0)
            for fn in self._listeners:
                try:
                    fn(ev)
                except Exception:  # noqa: BLE001
                    LOG.exception("raft listener failed")

    # ---- leader: replication -------------------------------------------------------------------
    def _replicate(self, peer: str, term: int) -> None:
        while not self._stop.is_set():
            snap = None
            with self._lock:
                if self.role != LEADER or self.storage.term != term or peer not in self._others() \
                        or self._replicators.get(peer) is not threading.current_thread():
                    return
                nxt = self._next[peer]
                if nxt <= self.storage.base_index and self.storage.snapshot_path:
                    snap = (self.storage.snapshot_path, self.storage.base_index, self.storage.base_term)
                    req = None
                else:
                    nxt = max(nxt, self.storage.base_index + 1)
                    prev = nxt - 1
                    ents = [pb.raft.RaftLogEntry(term=t, index=i, command=p)
                            for i, t, p in self.storage.entries(nxt, max_bytes=self.batch_bytes)]
                    req = pb.raft.AppendEntriesPRequest(term=term, leaderId=self.id, prevLogIndex=prev,
                                                        prevLogTerm=self.storage.term_at(prev) or 0,
                                                        entries=ents, leaderCommit=self.commit_index)
            if snap is not None:
                ok = self._push_snapshot(peer, term, *snap)
                with self._lock:
                    if ok:
                        self._contact[peer] = time.monotonic()
                        self._match[peer] = max(self._match.get(peer, 0), snap[1])
                        self._next[peer] = self._match[peer] + 1
                        self._advance_commit()
                    else:
                        self._cond.wait(self.heartbeat)
                continue
            try:
                r = self._call(peer, "AppendEntries", req)
            except Exception:  # noqa: BLE001
                with self._lock:
                    self._cond.wait(min(self.heartbeat, self.T / 2))
                continue
            with self._lock:
                if r.term > self.storage.term:
                    self._become_follower(r.term, None)
                    return
                if self.role != LEADER or self.storage.term != term:
                    return
                self._contact[peer] = time.monotonic()
                if r.success:
                    self._match[peer] = max(self._match.get(peer, 0), r.matchIndex)
                    self._next[peer] = self._match[peer] + 1
                    self._advance_commit()
                    if self._transfer_target == peer and self._match[peer] == self.storage.last_index():
                        self._pool.submit(self._send_timeout_now, peer, term)
                else:
                    back = r.conflictIndex if r.conflictIndex > 0 else nxt - 1
                    self._next[peer] = max(1, min(nxt - 1, back))
                    continue
                # idle: wait for new entries, a commit to propagate, or the heartbeat interval
                if self._next[peer] > self.storage.last_index() and r.matchIndex >= 0:
                    sent_commit = req.leaderCommit
                    end = time.monotonic() + self.heartbeat
                    while (not self._stop.is_set() and self.role == LEADER and self.storage.term == term
                           and self._next[peer] > self.storage.last_index()
                           and self.commit_index == sent_commit):
                        rem = end - time.monotonic()
                        if rem <= 0:
                            break
                        self._cond.wait(rem)

    def _push_snapshot(self, peer: str, term: int, path: str, index: int, sterm: int) -> bool:
        LOG.info("raft %s: sending snapshot %d to %s", self.id, index, peer)

        def chunks():
            off = 0
            with open(path, "rb") as f:
                while True:
                    b = f.read(self.chunk)
                    eof = len(b) < self.chunk
                    yield pb.meta.UploadSnapshotPRequest(data=pb.meta.SnapshotData(
                        snapshotTerm=sterm, snapshotIndex=index, chunk=b, offset=off, eof=eof,
                        leaderTerm=term, leaderId=self.id))
                    off += len(b)
                    if eof:
                        return
        try:
            size = os.path.getsize(path)
            rs = self._call(peer, "UploadSnapshot", chunks(), service=SVC_RAFT_JOURNAL)
            rs = list(rs)
            return bool(rs) and rs[-1].offsetReceived == size
        except Exception as e:  # noqa: BLE001
            LOG.warning("raft %s: snapshot push to %s failed: %s", self.id, peer, e)
            return False

    def _advance_commit(self) -> None:
        voters = self.peers()
        matches = sorted((self.storage.last_index() if p == self.id else self._match.get(p, 0) for p in voters),
                         reverse=True)
        if not matches:
            return
        n = matches[self._quorum(voters) - 1]
        if n > self.commit_index and self.storage.term_at(n) == self.storage.term:
            self.commit_index = n
            self._cond.notify_all()
            if self.id not in voters and self._configs[-1][0] <= n:
                LOG.info("raft %s: removed from the group, stepping down", self.id)
                self._become_follower(self.storage.term, None)

    # ---- leader: client API --------------------------------------------------------------------
    def is_leader(self) -> bool:
        return self.role == LEADER

    def propose(self, payload: bytes) -> tuple[int, int]:
        with self._lock:
            if self.role != LEADER:
                raise NotLeaderException(self.leader_id)
            if self._transfer_target is not None:
                raise UnavailableException("raft leadership transfer in progress")
            idx = self.storage.append([(self.storage.term, payload)])
            if payload[:1] == KIND_CONFIG:
                self._configs.append((idx, parse_config(payload)))
                self._sync_replicators()
            self._advance_commit()
            self._cond.notify_all()
            return idx, self.storage.term

    def wait_committed(self, index: int, term: int, timeout: float) -> None:
        end = time.monotonic() + timeout
        with self._lock:
            while True:
                if self.commit_index >= index:
                    t = self.storage.term_at(index)
                    if t is None and index <= self.storage.base_index and self.storage.term == term:
                        return
                    if t == term:
                        return
                    raise UnavailableException(f"raft entry {index} was overwritten (leadership lost)")
                if self.storage.term != term or self.role != LEADER:
                    raise UnavailableException("raft leadership lost before the entry committed")
                if self._stop.is_set():
                    raise UnavailableException("raft server stopped")
                rem = end - time.monotonic()
                if rem <= 0:
                    raise UnavailableException(f"raft entry {index} not committed within {timeout}s")
                self._cond.wait(min(rem, 0.1))

    def submit(self, payload: bytes, timeout: float) -> int:
        idx, term = self.propose(payload)
        self.wait_committed(idx, term, timeout)
        return idx

    def wait_applied(self, index: int, timeout: float) -> bool:
        end = time.monotonic() + timeout
        with self._lock:
            while self.last_applied < index:
                rem = end - time.monotonic()
                if rem <= 0 or self._stop.is_set():
                    return False
                self._cond.wait(min(rem, 0.1))
        return True

    def change_peers(self, peers, timeout: float) -> None:
        with self._lock:
            if self.role != LEADER:
                raise NotLeaderException(self.leader_id)
            if self._configs[-1][0] > self.commit_index:
                raise UnavailableException("another membership change is in progress")
            cur = set(self.peers())
            new = set(peers)
            if len(cur ^ new) > 1:
                raise ValueError("one server may be added or removed at a time")
            if cur == new:
                return
        self.submit(config_payload(new), timeout)

    def transfer_leadership(self, target: str, timeout: float) -> bool:
        """Catch ``target`` up, then tell it to campaign at once (TimeoutNow)."""
        with self._lock:
            if self.role != LEADER or target not in self._others():
                return False
            self._transfer_target = target
            term = self.storage.term
            if self._match.get(target, 0) == self.storage.last_index():
                self._pool.submit(self._send_timeout_now, target, term)
            self._cond.notify_all()
        end = time.monotonic() + timeout
        with self._lock:
            while self.role == LEADER and self.storage.term == term and time.monotonic() < end:
                self._cond.wait(0.05)
            if self.role == LEADER:
                self._transfer_target = None
                return False
        return True

    def _send_timeout_now(self, peer: str, term: int) -> None:
        try:
            self._call(peer, "TimeoutNow", pb.raft.TimeoutNowPRequest(term=term, leaderId=self.id))
        except Exception as e:  # noqa: BLE001
            LOG.warning("raft %s: TimeoutNow to %s failed: %s", self.id, peer, e)

    # ---- follower: RPC handlers ----------------------------------------------------------------
    def handle_request_vote(self, req):
        with self._lock:
            now = time.monotonic()
            term = self.storage.term
            sticky = not req.transfer and (self.role == LEADER or (
                self.leader_id is not None and now - self._last_heard < self.T))
            up_to_date = (req.lastLogTerm, req.lastLogIndex) >= (self.storage.last_term(), self.storage.last_index())
            if req.preVote:      # would a real vote succeed?  (no state changes)
                granted = req.term > term and up_to_date and not sticky
                return pb.raft.RequestVotePResponse(term=term, granted=bool(granted))
            if req.term < term or sticky:
                return pb.raft.RequestVotePResponse(term=term, granted=False)
            if req.term > term:
                self._become_follower(req.term, None)
            granted = self.storage.voted_for in (None, req.candidateId) and up_to_date
            if granted:
                self.storage.save_meta(self.storage.term, req.candidateId)
                self._reset_deadline()
            return pb.raft.RequestVotePResponse(term=self.storage.term, granted=granted)

    def handle_append_entries(self, req):
        with self._lock:
            st = self.storage
            if req.term < st.term:
                return pb.raft.AppendEntriesPResponse(term=st.term, success=False)
            if req.term > st.term or self.role != FOLLOWER:
                self._become_follower(req.term, req.leaderId)
            self.leader_id = req.leaderId
            self._last_heard = time.monotonic()
            self._reset_deadline()
            prev = req.prevLogIndex
            if prev > st.last_index():
                return pb.raft.AppendEntriesPResponse(term=st.term, success=False, conflictIndex=st.last_index() + 1)
            if prev >= st.base_index and st.term_at(prev) != req.prevLogTerm:
                bad = st.term_at(prev)
                i = prev
                while i > st.base_index + 1 and st.term_at(i - 1) == bad:
                    i -= 1
                return pb.raft.AppendEntriesPResponse(term=st.term, success=False, conflictIndex=max(1, i))
            new = []
            for e in req.entries:
                if e.index <= st.base_index:
                    continue
                if e.index <= st.last_index():
                    if st.term_at(e.index) == e.term:
                        continue
                    st.truncate_from(e.index)
                    self._configs = [c for c in self._configs if c[0] < e.index] or self._configs[:1]
                new.append(e)
            if new:
                st.append([(e.term, e.command) for e in new])
                for e in new:
                    if e.command[:1] == KIND_CONFIG:
                        self._configs.append((e.index, parse_config(e.command)))
            last_new = prev + len(req.entries)
            if req.leaderCommit > self.commit_index:
                self.commit_index = min(req.leaderCommit, max(last_new, st.base_index))
                self._cond.notify_all()
            return pb.raft.AppendEntriesPResponse(term=st.term, success=True, matchIndex=last_new)

    def handle_timeout_now(self, req):
        with self._lock:
            if req.term < self.storage.term or self.id not in self.peers():
                return pb.raft.TimeoutNowPResponse(accepted=False)
            self.leader_id = None
        self._pool.submit(self._election, False, True)
        return pb.raft.TimeoutNowPResponse(accepted=True)

    def handle_upload_snapshot(self, request_iter):
        """InstallSnapshot: receive chunks into a temp file, then install atomically."""
        tmp = self.storage.new_snapshot_tmp()
        received = 0
        meta = None
        try:
            with open(tmp, "wb") as f:
                for r in request_iter:
                    d = r.data
                    if meta is None:
                        with self._lock:
                            if d.leaderTerm < self.storage.term:
                                raise UnavailableException("stale snapshot sender")
                            if d.leaderTerm > self.storage.term or self.role != FOLLOWER:
                                self._become_follower(d.leaderTerm, d.leaderId)
                            self.leader_id = d.leaderId
                        meta = (d.snapshotIndex, d.snapshotTerm, d.leaderTerm)
                    if d.offset != received:
                        raise UnavailableException(f"snapshot chunk at {d.offset}, expected {received}")
                    f.write(d.chunk)
                    received += len(d.chunk)
                    with self._lock:
                        self._last_heard = time.monotonic()
                        self._reset_deadline()
                    if d.eof:
                        break
                f.flush()
                os.fsync(f.fileno())
            if meta is not None:
                self.install_snapshot_file(tmp, meta[0], meta[1])
            yield pb.meta.UploadSnapshotPResponse(offsetReceived=received)
        finally:
            if os.path.exists(tmp):
                os.remove(tmp)

    def install_snapshot_file(self, tmp: str, index: int, term: int) -> None:
        with self._apply_lock:
            with self._lock:
                if index <= self.storage.base_index:
                    return
                if index <= self.last_applied:
                    # state is already past it: adopt the file only to compact the log
                    self.storage.install_snapshot(tmp, index, term)
                    return
            peers = self.sm.install_snapshot(tmp)
            with self._lock:
                self.storage.install_snapshot(tmp, index, term)
                self._configs = [(index, sorted(set(peers)))] + [c for c in self._configs if c[0] > index]
                self.last_applied = index
                self.commit_index = max(self.commit_index, index)
                self.snapshot_installs += 1
                self._cond.notify_all()
        LOG.info("raft %s: installed snapshot %d (term %d)", self.id, index, term)

    def snapshot_chunks(self, start: int = 0):
        """DownloadSnapshot: stream the latest local snapshot."""
        with self._lock:
            path, index, term = self.storage.snapshot_path, self.storage.base_index, self.storage.base_term
        if path is None:
            yield pb.meta.DownloadSnapshotPResponse(data=pb.meta.SnapshotData(snapshotIndex=0, eof=True))
            return
        with open(path, "rb") as f:
            f.seek(start)
            off = start
            while True:
                b = f.read(self.chunk)
                eof = len(b) < self.chunk
                yield pb.meta.DownloadSnapshotPResponse(data=pb.meta.SnapshotData(
                    snapshotTerm=term, snapshotIndex=index, chunk=b, offset=off, eof=eof))
                off += len(b)
                if eof:
                    return

    # ---- applier & snapshots -------------------------------------------------------------------
    def _apply_loop(self) -> None:
        while not self._stop.is_set():
            with self._lock:
                while self.commit_index <= self.last_applied and not self._stop.is_set():
                    self._cond.wait(0.1)
                if self._stop.is_set():
                    return
                batch = self.storage.entries(self.last_applied + 1, self.commit_index, max_bytes=64 << 20)
            with self._apply_lock:
                for idx, _term, payload in batch:
                    with self._lock:
                        if idx != self.last_applied + 1:
                            break
                    try:
                        self.sm.apply(idx, payload)
                    except Exception:  # noqa: BLE001
                        LOG.exception("raft %s: applying entry %d failed", self.id, idx)
                    with self._lock:
                        self.last_applied = idx
                        self._cond.notify_all()
            if (self.snapshot_period > 0 and self.last_applied - self.storage.base_index >= self.snapshot_period
                    and self.snapshot_allowed()):
                try:
                    self.take_snapshot()
                except Exception:  # noqa: BLE001
                    LOG.exception("raft %s: snapshot failed", self.id)

    def take_snapshot(self) -> int:
        """Snapshot the state machine at ``last_applied`` and compact the log before it."""
        with self._apply_lock:
            with self._lock:
                idx = self.last_applied
                if idx <= self.storage.base_index:
                    return self.storage.base_index
                term = self.storage.term_at(idx)
                peers = self._config_at(idx)
                tmp = self.storage.new_snapshot_tmp()
            self.sm.write_snapshot(tmp, idx, term, peers)
            with self._lock:
                self.storage.install_snapshot(tmp, idx, term)
                self._configs = [(idx, peers)] + [c for c in self._configs if c[0] > idx]
        LOG.info("raft %s: snapshot at index %d (term %d)", self.id, idx, term)
        return idx

    def reset_applied_to_snapshot(self) -> None:
        """Rebuild the state machine from the local snapshot; committed entries after it are
        re-applied by the applier (used when a primary steps down)."""
        with self._apply_lock:
            with self._lock:
                path = self.storage.snapshot_path
                base = self.storage.base_index
            peers = self.sm.install_snapshot(path)
            with self._lock:
                if path is not None and peers:
                    self._configs = [(base, sorted(set(peers)))] + [c for c in self._configs if c[0] > base]
                self.last_applied = base
                self._cond.notify_all()

    # ---- introspection -------------------------------------------------------------------------
    def status(self) -> dict:
        with self._lock:
            now = time.monotonic()
            return {"id": self.id, "role": self.role, "term": self.storage.term, "leader": self.leader_id,
                    "commit": self.commit_index, "applied": self.last_applied,
                    "last": self.storage.last_index(), "base": self.storage.base_index,
                    "peers": list(self.peers()),
                    "contact_s": {p: (now - self._contact[p]) for p in self._others() if p in self._contact}}


class RaftServiceHandler:
    """RaftServerService + RaftJournalService servicers bound to one node."""

    def __init__(self, node_fn, on_query=None):
        self._node = node_fn
        self._on_query = on_query

    def RequestVote(self, req, ctx):
        return self._node().handle_request_vote(req)

    def AppendEntries(self, req, ctx):
        return self._node().handle_append_entries(req)

    def TimeoutNow(self, req, ctx):
        return self._node().handle_timeout_now(req)

    def JournalQuery(self, req, ctx):
        if self._on_query is None:
            return pb.meta.JournalQueryResponse()
        return self._on_query(req)

    def UploadSnapshot(self, request_iter, ctx):
        yield from self._node().handle_upload_snapshot(request_iter)

    def DownloadSnapshot(self, request_iter, ctx):
        start = 0
        for r in request_iter:
            start = r.offsetReceived
            break
        yield from self._node().snapshot_chunks(start)
