"""Typed master checkpoints: golden bytes of every CheckpointType and the FileSystemMaster tree.

Golden bytes are derived by hand from the reference writers (core/server/common/src/main/java/
alluxio/master/journal/): CheckpointOutputStream (8-byte big-endian type id), LongsCheckpointFormat
/ CheckpointedIdHashSet.writeToCheckpoint (DataOutputStream longs), LongCheckpointFormat /
InodeCounter.writeToCheckpoint (one long), InodeProtosCheckpointFormat / HeapInodeStore
(delimited InodeMeta.Inode), and JournalUtils.writeToCheckpoint (COMPOUND: Kryo writeString +
the component stream inside OutputChunked, zero-length chunk per component).  No JVM is
available here, so byte-for-byte interop with a Java master stays "parity unpinned"; these tests
pin the layout the reference code defines.
"""
import io
import os

from alluxio_amd.journal import checkpoint as ck
from alluxio_amd.journal import format as fmt
from alluxio_amd.journal.format import CheckpointType
from alluxio_amd.proto import pb


def _q(v):
    return v.to_bytes(8, "big", signed=True)


def test_leaf_formats_golden_bytes():
    assert ck.longs([1, -2]) == _q(2) + _q(1) + _q(-2)
    assert ck.long_(7) == _q(5) + _q(7)
    inode = pb.metastore.Inode(id=1)
    assert ck.inode_protos([inode]) == _q(4) + b"\x02\x08\x01"
    e = pb.journal.JournalEntry(sequence_number=3)
    assert ck.journal_entries([e]) == _q(0) + b"\x02\x08\x03"
    for data, t in ((ck.longs([5, 6]), CheckpointType.LONGS), (ck.long_(9), CheckpointType.LONG),
                    (ck.inode_protos([inode]), CheckpointType.INODE_PROTOS),
                    (ck.journal_entries([e]), CheckpointType.JOURNAL_ENTRY),
                    (ck.typed(CheckpointType.ROCKS, b"tarball"), CheckpointType.ROCKS)):
        assert ck.parse(data).type == t
    assert ck.parse(ck.longs([5, 6])).longs() == [5, 6]
    assert ck.parse(ck.long_(9)).long() == 9
    assert ck.parse(ck.inode_protos([inode])).inodes()[0].id == 1


def test_nested_compound_golden_bytes():
    # INODE_COUNTER (13 ASCII chars: Kryo writes them with bit 7 set on the last one)
    counter = ck.long_(7)
    inner = ck.compound([("INODE_COUNTER", counter)])
    name = b"INODE_COUNTE" + bytes([ord("R") | 0x80])
    assert inner == _q(1) + bytes([len(name) + len(counter)]) + name + counter + b"\x00"
    outer = ck.compound([("INODE_TREE", inner)])
    tname = b"INODE_TRE" + bytes([ord("E") | 0x80])
    assert outer == _q(1) + bytes([len(tname) + len(inner)]) + tname + inner + b"\x00"
    cp = ck.parse(outer)
    assert cp.type == CheckpointType.COMPOUND and [p.name for p in cp.parts] == ["INODE_TREE"]
    sub = cp.parts[0]
    assert sub.type == CheckpointType.COMPOUND and sub.component("INODE_COUNTER").long() == 7


def test_compound_chunks_at_64k():
    big = ck.longs(range(20_000))            # 160 KB body -> three chunks
    data = ck.compound([("TTL_BUCKET_LIST", big)])
    cp = ck.parse(data)
    assert cp.parts[0].longs() == list(range(20_000))
    payload = fmt.kryo_string("TTL_BUCKET_LIST") + big
    assert data[8:8 + 3] == fmt.kryo_varint(65536)
    assert data.endswith(fmt.kryo_varint(len(payload) - 2 * 65536) + payload[2 * 65536:] + b"\x00")


def _master(tmp_path, journal="journal"):
    from alluxio_amd.conf import Configuration
    from alluxio_amd.master.process import AlluxioMasterProcess
    conf = Configuration({"alluxio.master.journal.folder": str(tmp_path / journal),
                          "alluxio.master.journal.type": "UFS",
                          "alluxio.security.authorization.permission.enabled": "false"})
    m = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    return m


def _populate(fsm):
    fsm.create_directory("/a/b", recursive=True)
    fsm.create_file("/a/b/f", block_size=1 << 20, replication_min=1)
    fsm.get_new_block_id_for_file("/a/b/f")
    fsm.create_file("/a/g")
    fsm.complete_file("/a/g")
    fsm.set_attribute("/a/g", pinned=True, ttl=3_600_000, ttl_action="FREE", mode=0o640)
    fsm.create_directory("/p", write_type="CACHE_THROUGH")
    fsm.set_attribute("/a", owner="alice", group="staff")
    from alluxio_amd.security.acl import AclEntry, AclEntryType
    fsm.set_acl("/a/b", "MODIFY", [AclEntry(AclEntryType.NAMED_USER, "bob", 5, False)])


def _snapshot(fsm):
    out = {}
    with fsm.tree.lock.read():
        for n in [fsm.tree.root] + fsm.tree.descendants(fsm.tree.root):
            p = fsm.tree.path_of(n)
            out[p] = (n.id, n.is_directory, n.owner, n.group, n.mode, n.pinned, n.ttl, n.ttl_action,
                      n.persistence_state, getattr(n, "block_ids", None), getattr(n, "completed", None),
                      getattr(n, "replication_min", None),
                      sorted((n.acl.named_users if n.acl else {}).items()))
    return out


def test_file_system_master_checkpoint_tree_and_restart(tmp_path):
    """FileSystemMaster writes the reference's nested component tree; a checkpoint-only restart
    (every log below the checkpoint garbage-collected) restores the namespace exactly."""
    m = _master(tmp_path)
    fsm = m.fs_master
    _populate(fsm)
    before = _snapshot(fsm)
    cp = ck.parse(fsm.write_checkpoint(), "FILE_SYSTEM_MASTER")
    assert [p.name for p in cp.parts] == ["INODE_TREE", "INODE_DIRECTORY_ID_GENERATOR", "MOUNT_TABLE",
                                          "MASTER_UFS_MANAGER", "ACTIVE_SYNC_MANAGER"]
    tree = cp.component("INODE_TREE")
    assert [p.name for p in tree.parts] == ["HEAP_INODE_STORE", "PINNED_INODE_FILE_IDS",
                                            "REPLICATION_LIMITED_FILE_IDS", "TO_BE_PERSISTED_FILE_IDS",
                                            "TTL_BUCKET_LIST", "INODE_COUNTER"]
    assert [p.type for p in tree.parts] == [CheckpointType.INODE_PROTOS] + [CheckpointType.LONGS] * 4 + \
        [CheckpointType.LONG]
    inodes = tree.component("HEAP_INODE_STORE").inodes()
    assert tree.component("INODE_COUNTER").long() == len(inodes) == len(before)
    g = fsm.tree.get("/a/g")
    f = fsm.tree.get("/a/b/f")          # replicationMin > 0 pins a file (applyCreateInode)
    assert tree.component("PINNED_INODE_FILE_IDS").longs() == sorted([f.id, g.id])
    assert tree.component("TTL_BUCKET_LIST").longs() == [g.id]
    assert tree.component("REPLICATION_LIMITED_FILE_IDS").longs() == []     # no replicationMax set
    # owner/group/mode live in the access ACL (OWNING_USER_KEY "" entries + otherActions)
    gp = next(p for p in inodes if p.id == g.id)
    assert [(a.name, list(a.actions.actions)) for a in gp.access_acl.userActions] == [("", [0, 1])]
    assert [(a.name, list(a.actions.actions)) for a in gp.access_acl.groupActions] == [("", [0])]
    assert list(gp.access_acl.otherActions.actions) == [] and not gp.access_acl.isEmpty
    root = next(p for p in inodes if p.parent_id == -1)
    assert root.is_directory and root.default_acl.isDefault and root.default_acl.isEmpty
    # checkpoint through the journal system, GC the logs, restart from the checkpoint alone
    m.journal.checkpoint()
    jdir = tmp_path / "journal" / "FileSystemMaster" / "v1"
    assert os.listdir(jdir / "checkpoints") and not [f for f in os.listdir(jdir / "logs")
                                                     if not f.endswith("-0x7fffffffffffffff")]
    with open(jdir / "checkpoints" / os.listdir(jdir / "checkpoints")[0], "rb") as f:
        assert fmt.read_checkpoint_header(f) == CheckpointType.COMPOUND
    m.stop()
    m2 = _master(tmp_path)
    assert _snapshot(m2.fs_master) == before
    # the restored namespace keeps working (ids, dir id generator, mounts)
    m2.fs_master.create_file("/a/h")
    assert m2.fs_master.get_status("/a/h").fileId not in {v[0] for v in before.values()}
    m2.stop()


def test_restore_accepts_caching_inode_store_and_rejects_rocks(tmp_path):
    m = _master(tmp_path)
    fsm = m.fs_master
    _populate(fsm)
    before = _snapshot(fsm)
    cp = ck.parse(fsm.write_checkpoint())
    tree = cp.component("INODE_TREE")
    heap = ck.typed(tree.parts[0].type, tree.parts[0].body)
    # CachingInodeStore.writeToCheckpoint writes its backing store's checkpoint under its own name
    caching = ck.compound([("CACHING_INODE_STORE", heap)] +
                          [(p.name, ck.typed(p.type, p.body)) for p in tree.parts[1:]])
    rebuilt = ck.compound([("INODE_TREE", caching)] + [(p.name, ck.typed(p.type, p.body)) for p in cp.parts[1:]])
    fsm.restore_checkpoint(ck.parse(rebuilt))
    assert _snapshot(fsm) == before
    rocks = ck.compound([("INODE_TREE", ck.compound([("ROCKS_INODE_STORE", ck.typed(CheckpointType.ROCKS, b"x"))]))])
    import pytest
    with pytest.raises(ValueError, match="RocksDB"):
        fsm.restore_checkpoint(ck.parse(rocks))
    m.stop()


def test_raft_snapshot_nests_master_checkpoints_and_reads_legacy(tmp_path):
    """Embedded-journal snapshots (JournalStateMachine.write_snapshot / install_snapshot): one
    COMPOUND over the masters with each master's own typed checkpoint nested (FILE_SYSTEM_MASTER
    is itself COMPOUND); round-1 snapshots (4-byte count framing) still install."""
    import struct
    import types
    from alluxio_amd.journal.raft_system import JournalStateMachine
    m = _master(tmp_path)
    _populate(m.fs_master)
    before = _snapshot(m.fs_master)
    comps = {"FileSystemMaster": m.fs_master, "BlockMaster": m.block_master}
    sm = JournalStateMachine(types.SimpleNamespace(journaled=comps))
    snap = str(tmp_path / "snap")
    sm.write_snapshot(snap, 10, 2, ["a:1"])
    with open(snap, "rb") as f:
        fmt.read_delimited(f, pb.raft.RaftSnapshotHeader)
        parts = fmt.read_compound(f)
    assert [(n, p.type) for n, p in parts] == [("BlockMaster", CheckpointType.JOURNAL_ENTRY),
                                               ("FileSystemMaster", CheckpointType.COMPOUND)]
    m.fs_master.reset_state()
    assert sm.install_snapshot(snap) == ["a:1"]
    assert _snapshot(m.fs_master) == before
    # legacy framing: header, then a count and (name, journal entries) per master
    entries = fmt.entries_to_bytes(m.fs_master.journal_entries())
    legacy = str(tmp_path / "legacy")
    with open(legacy, "wb") as f:
        fmt.write_delimited(f, pb.raft.RaftSnapshotHeader(index=3, term=1, peers=["b:2"], nextSequenceNumber=5,
                                                          masters=["FileSystemMaster"]))
        f.write(struct.pack(">i", 1))
        f.write(struct.pack(">i", len(b"FileSystemMaster")) + b"FileSystemMaster")
        f.write(struct.pack(">q", len(entries)) + entries)
    m.fs_master.reset_state()
    assert sm.install_snapshot(legacy) == ["b:2"] and sm.next_sn == 5
    assert _snapshot(m.fs_master) == before
    m.stop()
