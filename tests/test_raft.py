"""Embedded (Raft) journal.

Reference coverage model: core/server/common/src/test/.../journal/raft/*Test (RaftJournalSystem,
JournalStateMachine, snapshot replication) and tests/src/test/java/alluxio/server/ft/journal/raft/
EmbeddedJournalIntegrationTest* (failover, restart catch-up, quorum info/remove, snapshot
transfer to a lagging master).  Consensus nodes here run over the in-process RPC transport; a
filtering channel cuts links to model partitions.
"""
import io
import json
import os
import time

import pytest

from alluxio_amd.journal.raft import (KIND_JOURNAL, LEADER, SVC_RAFT, SVC_RAFT_JOURNAL, RaftNode,
                                      RaftServiceHandler, RaftStorage)
from alluxio_amd.proto import pb
from alluxio_amd.rpc import Channel, RpcServer, _alloc_local_port
from alluxio_amd.utils.exceptions import UnavailableException


class ListSM:
    def __init__(self):
        self.items = []

    def apply(self, index, payload):
        v = payload[1:].decode()
        if payload[:1] == KIND_JOURNAL and v not in self.items:    # retried submits (like SN dedup)
            self.items.append(v)

    def write_snapshot(self, path, index, term, peers):
        with open(path, "w") as f:
            json.dump({"items": self.items, "peers": list(peers)}, f)

    def install_snapshot(self, path):
        if path is None:
            self.items = []
            return []
        with open(path) as f:
            d = json.load(f)
        self.items = list(d["items"])
        return d["peers"]


class _Cut:
    def __init__(self):
        self.cut = set()

    def isolate(self, a, ids):
        for b in ids:
            if b != a:
                self.cut.add(frozenset((a, b)))

    def heal(self):
        self.cut.clear()


class FilteredChannel:
    def __init__(self, src, dst, net):
        self.src, self.dst, self.net = src, dst, net
        self.ch = Channel(dst, auth=None)

    def stub(self, svc):
        if frozenset((self.src, self.dst)) in self.net.cut:
            raise UnavailableException(f"link {self.src}->{self.dst} is cut")
        return self.ch.stub(svc)

    def raw_stream(self, svc, method):
        if frozenset((self.src, self.dst)) in self.net.cut:
            raise UnavailableException(f"link {self.src}->{self.dst} is cut")
        return self.ch.raw_stream(svc, method)

    def close(self):
        self.ch.close()


class Group:
    def __init__(self, root, n=3, T=150, period=0, ids=None, transport="UNARY"):
        self.root, self.T, self.period = root, T, period
        self.transport = transport
        self.ids = ids or [f"127.0.0.1:{_alloc_local_port()}" for _ in range(n)]
        self.net = _Cut()
        self.nodes, self.servers = {}, {}

    def start(self, nid, peers=None):
        storage = RaftStorage(os.path.join(self.root, nid.replace(":", "_")), fsync=False)
        sm = ListSM()
        got = sm.install_snapshot(storage.snapshot_path)
        node = RaftNode(nid, got or peers or self.ids, storage, sm,
                        lambda a, s=nid: FilteredChannel(s, a, self.net),
                        election_timeout_ms=self.T, heartbeat_ms=self.T / 5, rpc_timeout_ms=500,
                        snapshot_chunk_bytes=64, snapshot_period_entries=self.period, transport=self.transport)
        srv = RpcServer("127.0.0.1", int(nid.rsplit(":", 1)[1]), enable_grpc=False)
        h = RaftServiceHandler(lambda: node)
        srv.add_servicer(SVC_RAFT, h)
        srv.add_servicer(SVC_RAFT_JOURNAL, h)
        from alluxio_amd.journal.messaging import SVC_MESSAGING, MessagingServiceHandler
        srv.add_servicer(SVC_MESSAGING, MessagingServiceHandler(h))
        srv.start()
        node.start()
        self.nodes[nid], self.servers[nid] = node, srv
        return node

    def start_all(self):
        for i in self.ids:
            self.start(i)
        return self

    def kill(self, nid):
        self.servers.pop(nid).stop()
        self.nodes.pop(nid).stop()

    def leader(self, timeout=10.0, exclude=()):
        end = time.time() + timeout
        while time.time() < end:
            ls = [n for i, n in self.nodes.items() if n.role == LEADER and i not in exclude]
            if len(ls) == 1:
                return ls[0]
            time.sleep(0.01)
        raise TimeoutError("no single leader")

    def submit(self, node, values):
        for v in values:
            for _ in range(20):       # a just-elected leader can still be deposed by a racing election
                try:
                    node.submit(KIND_JOURNAL + v.encode(), timeout=5)
                    break
                except UnavailableException:
                    node = self.leader()

    def wait_items(self, expected, nodes=None, timeout=10.0):
        end = time.time() + timeout
        nodes = nodes or list(self.nodes.values())
        while time.time() < end:
            if all(n.sm.items == expected for n in nodes):
                return
            time.sleep(0.01)
        raise AssertionError({n.id: n.sm.items[-3:] + [len(n.sm.items)] for n in nodes})

    def stop(self):
        for nid in list(self.nodes):
            self.kill(nid)


@pytest.fixture
def group(tmp_path):
    g = Group(str(tmp_path))
    yield g
    g.stop()


def test_storage_roundtrip_and_torn_tail(tmp_path):
    st = RaftStorage(str(tmp_path / "s"), fsync=False)
    st.save_meta(3, "a")
    st.append([(1, b"J1"), (1, b"J2"), (2, b"J3")])
    st.truncate_from(3)
    st.append([(3, b"J3b")])
    st.close()
    with open(tmp_path / "s" / "log", "ab") as f:
        f.write(b"\x05\x00\x00\x00garbage")            # torn record
    st = RaftStorage(str(tmp_path / "s"), fsync=False)
    assert (st.term, st.voted_for) == (3, "a")
    assert [(i, t, p) for i, t, p in st.entries(1)] == [(1, 1, b"J1"), (2, 1, b"J2"), (3, 3, b"J3b")]
    tmp = st.new_snapshot_tmp()
    open(tmp, "w").write("{}")
    st.install_snapshot(tmp, 2, 1)                     # compacts 1..2, keeps 3
    assert (st.base_index, st.last_index(), st.term_at(3)) == (2, 3, 3)
    st.close()
    st = RaftStorage(str(tmp_path / "s"), fsync=False)
    assert (st.base_index, st.base_term, [e[0] for e in st.entries(1)]) == (2, 1, [3])


def test_election_replication_and_failover(group):
    group.start_all()
    lead = group.leader()
    group.submit(lead, [f"a{i}" for i in range(30)])
    group.wait_items([f"a{i}" for i in range(30)])
    old = lead.id
    group.kill(old)
    lead2 = group.leader()
    assert lead2.id != old and lead2.storage.term > 0
    group.submit(lead2, ["b0", "b1"])
    # the old leader restarts from its own log and catches up from the new leader
    group.start(old)
    group.wait_items([f"a{i}" for i in range(30)] + ["b0", "b1"])


def test_lagging_follower_gets_snapshot(tmp_path):
    g = Group(str(tmp_path), period=10)
    try:
        g.start_all()
        lead = g.leader()
        lag = [i for i in g.ids if i != lead.id][0]
        g.kill(lag)
        vals = [f"v{i}" for i in range(40)]
        g.submit(lead, vals)
        end = time.time() + 10
        while lead.storage.base_index < 20 and time.time() < end:   # leader compacted its log
            time.sleep(0.01)
        assert lead.storage.base_index >= 20
        n = g.start(lag)
        g.wait_items(vals)
        end = time.time() + 5
        while n.snapshot_installs < 1 and time.time() < end:    # counted just after the state swap
            time.sleep(0.01)
        assert n.snapshot_installs >= 1
    finally:
        g.stop()


def test_partitioned_node_does_not_disrupt_leader(group):
    group.start_all()
    lead = group.leader()
    term = lead.storage.term
    other = [i for i in group.ids if i != lead.id][0]
    group.net.isolate(other, group.ids)
    time.sleep(group.T * 8 / 1000)
    assert group.nodes[other].storage.term == term      # PreVote: no term inflation while cut off
    group.net.heal()
    group.submit(lead, ["x"])
    group.wait_items(["x"])
    assert lead.role == LEADER and lead.storage.term == term


def test_minority_leader_steps_down_and_diverged_entries_are_dropped(group):
    group.start_all()
    lead = group.leader()
    group.submit(lead, ["c0"])
    group.net.isolate(lead.id, group.ids)
    # the cut-off leader accepts a write it can never commit
    idx, term = lead.propose(KIND_JOURNAL + b"lost")
    new = group.leader(exclude=(lead.id,))
    group.submit(new, ["c1"])
    end = time.time() + 10
    while lead.role == LEADER and time.time() < end:     # CheckQuorum
        time.sleep(0.01)
    assert lead.role != LEADER
    group.net.heal()
    group.wait_items(["c0", "c1"])


def test_membership_change_and_transfer(tmp_path):
    g = Group(str(tmp_path))
    try:
        g.start_all()
        lead = g.leader()
        g.submit(lead, ["m0", "m1"])
        newcomer = f"127.0.0.1:{_alloc_local_port()}"
        g.start(newcomer, peers=g.ids)                   # not a voter yet: stays passive
        lead.change_peers(set(g.ids) | {newcomer}, timeout=5)
        g.wait_items(["m0", "m1"])
        assert all(sorted(n.peers()) == sorted(g.ids + [newcomer]) for n in g.nodes.values())
        victim = [i for i in g.ids if i != lead.id][0]
        lead.change_peers(set(lead.peers()) - {victim}, timeout=5)
        g.kill(victim)
        g.submit(lead, ["m2"])
        g.wait_items(["m0", "m1", "m2"])
        assert victim not in lead.peers() and len(lead.peers()) == 3
        assert lead.transfer_leadership(newcomer, timeout=5)
        assert g.leader().id == newcomer
        g.submit(g.nodes[newcomer], ["m3"])
        g.wait_items(["m0", "m1", "m2", "m3"])
    finally:
        g.stop()


# ---- masters on the embedded journal ----------------------------------------------------------

def test_embedded_journal_master_failover(tmp_path):
    from alluxio_amd.cli.fsadmin import FileSystemAdminShell
    from alluxio_amd.minicluster import MultiMasterLocalAlluxioCluster
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "dram"}
    with MultiMasterLocalAlluxioCluster(num_masters=3, num_workers=1, conf=conf, journal_type="EMBEDDED",
                                        work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        for i in range(5):
            fs.write_file(f"/ej/f{i}", bytes([i]) * 1000, write_type="MUST_CACHE")
        fs.create_directory("/ej/dir")
        old = c.primary()
        idx = c.masters.index(old)
        new = c.kill_primary()
        assert new is not old
        names = sorted(s.info.name for s in fs.list_status("/ej"))
        assert names == ["dir"] + [f"f{i}" for i in range(5)]
        c.heartbeat_workers()          # the worker re-registers with the new primary
        c.heartbeat_workers()
        assert fs.read_file("/ej/f3") == bytes([3]) * 1000
        fs.write_file("/ej/after", b"z" * 10, write_type="MUST_CACHE")
        # fsadmin journal quorum info: 3 members, the killed one UNAVAILABLE
        out = io.StringIO()
        assert FileSystemAdminShell(fs, out=out).run(["journal", "quorum", "info"]) == 0
        text = out.getvalue()
        assert "Quorum size    : 3" in text and text.count("AVAILABLE") == 3 and "UNAVAILABLE" in text
        # the killed master restarts as a standby and replays what it missed
        m = c.start_master(idx)
        end = time.time() + 15
        while time.time() < end:
            if m.fs_master.tree.root is not None and not m.fs_master.tree.resolve("/ej/after")[1]:
                break
            time.sleep(0.05)
        assert not m.fs_master.tree.resolve("/ej/after")[1] and not m.primary
        # checkpoint on the primary (fsadmin journal checkpoint) compacts its raft log
        new.checkpoint()
        assert new.journal.node.storage.base_index > 0
        fs.close()


def test_single_master_embedded_restart_checkpoint_and_dump(tmp_path):
    from alluxio_amd.cli.journal_tool import dump_raft_journal
    from alluxio_amd.minicluster import LocalAlluxioCluster
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "dram", "alluxio.master.journal.type": "EMBEDDED"}
    with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=str(tmp_path / "c")) as c:
        from alluxio_amd.journal.raft_system import RaftJournalSystem
        assert isinstance(c.master.journal, RaftJournalSystem)
        fs = c.client()
        fs.write_file("/s/a", b"a" * 100, write_type="CACHE_THROUGH")
        fs.close()
        c.restart_master()                                # replays the raft log
        fs = c.client()
        assert fs.read_file("/s/a") == b"a" * 100
        c.master.checkpoint()                             # snapshot + log compaction
        fs.create_directory("/s/after_cp")
        fs.close()
        c.restart_master()                                # snapshot + log suffix
        fs = c.client()
        assert fs.exists("/s/after_cp") and fs.get_status("/s/a").length == 100
        fs.close()
        jdir = c.master.conf.get("alluxio.master.journal.folder")
    out = io.StringIO()
    n = dump_raft_journal(jdir, "FileSystemMaster", str(tmp_path / "dump"), out=out)
    assert n >= 1 and "Snapshot at raft index" in out.getvalue()
    assert "after_cp" in (tmp_path / "dump" / "edits.txt").read_text()


def test_consensus_over_messaging_streams(tmp_path):
    """The reference's transport: vote / append / timeout-now tunnelled through one
    MessagingService.connect stream per peer (journal/messaging.py), with failover, a cut link
    (the stream breaks and reconnects) and a restarted node catching up."""
    g = Group(str(tmp_path), transport="MESSAGING").start_all()
    try:
        lead = g.leader()
        g.submit(lead, [f"m{i}" for i in range(20)])
        g.wait_items([f"m{i}" for i in range(20)])
        assert any(lead._msg_conns.values()) and not any(c.closed for c in lead._msg_conns.values())
        old = lead.id
        g.kill(old)
        lead2 = g.leader()
        g.submit(lead2, ["n0"])
        g.start(old)
        g.wait_items([f"m{i}" for i in range(20)] + ["n0"])
    finally:
        g.stop()


def test_messaging_reports_remote_failure():
    from alluxio_amd.journal.messaging import MessagingConnection, MessagingServiceHandler

    class _H:
        def RequestVote(self, req, ctx):
            raise RuntimeError("boom")

        def AppendEntries(self, req, ctx):
            return pb.raft.AppendEntriesPResponse(term=req.term, success=True, matchIndex=7)

    class _Ch:
        def raw_stream(self, svc, method):
            return lambda it: MessagingServiceHandler(_H()).connect(it, None)

    c = MessagingConnection(_Ch())
    r = c.call("AppendEntries", pb.raft.AppendEntriesPRequest(term=3), 5)
    assert r.success and r.matchIndex == 7 and r.term == 3
    with pytest.raises(UnavailableException, match="boom"):
        c.call("RequestVote", pb.raft.RequestVotePRequest(term=1), 5)
    c.close()
    with pytest.raises(UnavailableException):
        c.call("AppendEntries", pb.raft.AppendEntriesPRequest(term=3), 1)
