"""HDFS UFS over the native Hadoop IPC + DataTransferProtocol client, against the in-process
mini HDFS in ``tests/hdfs_fake.py`` (the reference tests HdfsUnderFileSystem against a
MiniDFSCluster; no JVM here, so Java interop is parity unpinned).

Covers the UFS contract (integration/tools/validation/.../UnderFileSystemContractTest.java), multi-
block files with a 3-DataNode write pipeline, positioned reads that start mid-chunk, failover to a
second replica, checksum corruption detection, paged listings, and golden bytes of the IPC
preamble / call frame.
"""
import io
import os
import socket
import struct
import sys
import threading

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from hdfs_fake import MiniDfs  # noqa: E402

from alluxio_amd.cli import ufs_contract  # noqa: E402
from alluxio_amd.underfs import hadoop_rpc as H  # noqa: E402
from alluxio_amd.underfs.base import DeleteOptions, MkdirsOptions, OpenOptions, SpaceType  # noqa: E402
from alluxio_amd.underfs.registry import create as create_ufs  # noqa: E402


@pytest.fixture
def dfs():
    d = MiniDfs(num_datanodes=3, ls_limit=7)
    yield d
    d.stop()


def _ufs(d, **props):
    p = {"dfs.blocksize": "256k", "dfs.replication": "1"}
    p.update(props)
    return create_ufs(f"hdfs://127.0.0.1:{d.port}/", properties=p)


def test_hdfs_contract(dfs):
    res = ufs_contract.run(f"hdfs://127.0.0.1:{dfs.port}/", properties={"dfs.blocksize": "256k"},
                           out=io.StringIO(), large_file_size=1 << 20)
    assert res["failed"] == [], res["failed"]
    assert len(res["passed"]) >= 40


def test_multiblock_pipeline_positioned_reads_and_failover(dfs):
    ufs = _ufs(dfs, **{"dfs.replication": "3"})
    data = np.random.default_rng(1).integers(0, 256, (1 << 20) + 777, dtype=np.uint8).tobytes()
    with ufs.create("/d/big.bin") as f:
        for i in range(0, len(data), 100_003):          # writes straddle packet and block edges
            f.write(data[i:i + 100_003])
    st = ufs.get_status("/d/big.bin")
    assert st.content_length == len(data) and st.block_size == 256 << 10
    assert all(len(dn.blocks) == 5 for dn in dfs.datanodes)   # 5 blocks, every replica on all 3
    with ufs.open("/d/big.bin") as f:
        assert f.read() == data
    for off in (0, 1, 511, 513, (256 << 10) - 3, 600_001, len(data) - 5):
        with ufs.open("/d/big.bin", OpenOptions(offset=off)) as f:
            assert f.read(9000) == data[off:off + 9000], off
    with ufs.open("/d/big.bin") as f:
        f.seek(300_000)
        assert f.read(1000) == data[300_000:301_000]
        f.seek(10)
        assert f.read(10) == data[10:20]
    dfs.datanodes[0].fail_reads = True                  # first replica refuses: next one serves
    with ufs.open("/d/big.bin", OpenOptions(offset=12345)) as f:
        assert f.read(70_000) == data[12345:12345 + 70_000]
    assert ufs.get_file_locations("/d/big.bin") == ["localhost"] * 3
    assert ufs.get_space("/", SpaceType.SPACE_USED) == 3 * len(data)


def test_checksum_corruption_is_detected(dfs):
    ufs = _ufs(dfs, **{"dfs.replication": "1"})     # one replica: nothing to fail over to
    with ufs.create("/c.bin") as f:
        f.write(b"x" * 5000)
    dfs.datanodes[0].corrupt_reads = True
    with pytest.raises(IOError, match="checksum"):
        with ufs.open("/c.bin") as f:
            f.read()
    dfs.datanodes[0].corrupt_reads = False
    with ufs.open("/c.bin") as f:
        assert f.read() == b"x" * 5000


def test_truncated_or_corrupt_replica_fails_over_mid_stream(dfs):
    """A DataNode that ends a block early, or whose bytes fail their checksum, is never a silent
    short read: the reader moves to the block's next replica at the current position
    (DFSInputStream deadNodes + seekToNewSource); with every replica bad the read raises."""
    ufs = _ufs(dfs, **{"dfs.replication": "3"})
    data = np.random.default_rng(9).integers(0, 256, (600 << 10) + 17, dtype=np.uint8).tobytes()
    with ufs.create("/ft.bin") as f:
        f.write(data)
    dfs.datanodes[0].truncate_reads = True          # first replica: lastPacketInBlock after 1 packet
    dfs.datanodes[1].corrupt_reads = True           # second replica: flipped bits
    try:
        with ufs.open("/ft.bin") as f:
            assert f.read() == data
        with ufs.open("/ft.bin", OpenOptions(offset=300_001)) as f:
            assert f.read(100_000) == data[300_001:400_001]
        dfs.datanodes[2].truncate_reads = True      # no good replica left
        with pytest.raises(IOError):
            with ufs.open("/ft.bin") as f:
                f.read()
    finally:
        for dn in dfs.datanodes:
            dn.truncate_reads = dn.corrupt_reads = False


def test_listing_pages_mkdirs_delete_rename_semantics(dfs):
    ufs = _ufs(dfs)
    for i in range(20):
        with ufs.create(f"/ls/f{i:02d}") as f:
            f.write(b"%d" % i)
    names = [s.name for s in ufs.list_status("/ls")]
    assert names == [f"f{i:02d}" for i in range(20)]       # 3 pages of ls_limit=7
    assert dfs.calls.count("getListing") >= 3
    assert not ufs.mkdirs("/a/b/c", MkdirsOptions(create_parent=False))
    assert ufs.mkdirs("/a/b/c")
    assert not ufs.mkdirs("/a/b/c")
    assert not ufs.delete_directory("/ls")                  # non-empty, non-recursive
    assert ufs.rename_directory("/ls", "/ls2") and ufs.list_status("/ls") is None
    assert not ufs.rename_file("/ls2/f01", "/ls2/f02")      # destination exists
    assert ufs.delete_directory("/ls2", DeleteOptions(recursive=True))
    ufs.set_mode("/a/b", 0o700)
    ufs.set_owner("/a/b", "alice", "staff")
    st = ufs.get_status("/a/b")
    assert (st.mode, st.owner, st.group) == (0o700, "alice", "staff")
    with pytest.raises(FileNotFoundError):
        ufs.open("/nope")


def test_ipc_wire_golden_bytes():
    """Connection preamble and the first call frame, byte-for-byte (RpcHeader.proto/ProtobufRpcEngine)."""
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    got = {}

    def serve():
        c, _ = srv.accept()
        got["pre"] = bytes(H.recv_exact(c, 7))
        (n,) = struct.unpack(">I", bytes(H.recv_exact(c, 4)))
        got["ctx"] = bytes(H.recv_exact(c, n))
        (n,) = struct.unpack(">I", bytes(H.recv_exact(c, 4)))
        got["call"] = bytes(H.recv_exact(c, n))
        hdr = H.common.RpcResponseHeaderProto(callId=0, status=1, exceptionClassName="java.io.FileNotFoundException",
                                              errorMsg="nope")
        p = H.delimited(hdr)
        c.sendall(struct.pack(">I", len(p)) + p)
        c.close()

    t = threading.Thread(target=serve)
    t.start()
    nn = H.NameNodeClient("127.0.0.1", srv.getsockname()[1], user="bob")
    nn.client_id = bytes(range(16))
    with pytest.raises(H.RemoteException) as ei:
        nn.get_file_info("/x")
    t.join()
    srv.close()
    assert ei.value.short_name == "FileNotFoundException"
    assert got["pre"] == b"hrpc\x09\x00\x00"
    # RpcRequestHeaderProto{rpcKind=2, rpcOp=0, callId=-3 (zigzag 5), clientId, retryCount=-1 (zigzag 1)}
    hdr = b"\x08\x02\x10\x00\x18\x05\x22\x10" + bytes(range(16)) + b"\x28\x01"
    ctx = b"\x12\x05\x0a\x03bob\x1a" + bytes([len(H.CLIENT_PROTOCOL)]) + H.CLIENT_PROTOCOL.encode()
    assert got["ctx"] == bytes([len(hdr)]) + hdr + bytes([len(ctx)]) + ctx
    hdr0 = b"\x08\x02\x10\x00\x18\x00\x22\x10" + bytes(range(16)) + b"\x28\x00"
    rh = b"\x0a\x0bgetFileInfo\x12" + bytes([len(H.CLIENT_PROTOCOL)]) + H.CLIENT_PROTOCOL.encode() + b"\x18\x01"
    req = b"\x0a\x02/x"
    assert got["call"] == bytes([len(hdr0)]) + hdr0 + bytes([len(rh)]) + rh + bytes([len(req)]) + req


def test_packet_golden_bytes():
    """DataTransferProtocol packet: PLEN (incl. itself), HLEN, PacketHeaderProto, BE CRC32C sums, data."""
    a, b = socket.socketpair()
    H.write_packet(a, 512, 3, b"123456789", False)
    raw = b.recv(100)
    a.close()
    b.close()
    hdr = b"\x09" + struct.pack("<q", 512) + b"\x11" + struct.pack("<q", 3) + b"\x18\x00" + b"\x25" + \
        struct.pack("<i", 9)
    assert raw == struct.pack(">IH", 4 + 4 + 9, len(hdr)) + hdr + bytes.fromhex("e3069283") + b"123456789"


def test_hdfs_mount_through_cluster(dfs, tmp_path):
    """Mount hdfs:// into the namespace: CACHE_THROUGH write persists to HDFS blocks, free + read
    goes back to the DataNodes, UFS-only files are loaded by metadata sync."""
    from alluxio_amd.minicluster import LocalAlluxioCluster
    props = {"dfs.blocksize": "128k", "dfs.replication": "2"}
    ufs = _ufs(dfs, **props)
    ufs.mkdirs("/warehouse")
    with ufs.create("/warehouse/pre.bin") as f:
        f.write(b"p" * 300_000)
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"},
                             work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        fs.mount("/h", f"hdfs://127.0.0.1:{dfs.port}/warehouse", properties=props)
        assert fs.read_file("/h/pre.bin") == b"p" * 300_000
        data = os.urandom(400_000)
        fs.write_file("/h/new.bin", data, write_type="CACHE_THROUGH")
        assert fs.get_status("/h/new.bin").is_persisted
        assert ufs.get_status("/warehouse/new.bin").content_length == len(data)
        fs.free("/h/new.bin")
        assert fs.read_file("/h/new.bin") == data
        assert sorted(s.name for s in fs.list_status("/h")) == ["new.bin", "pre.bin"]
        fs.unmount("/h")


def test_active_sync_follows_inotify(dfs, tmp_path):
    """startSync on an HDFS mount: the heartbeat follows the NameNode's edit stream (getEditsFromTxid)
    and re-syncs only the touched paths; the txid is journaled (ActiveSyncTxIdEntry)."""
    from alluxio_amd.minicluster import LocalAlluxioCluster
    ufs = _ufs(dfs)
    ufs.mkdirs("/w/a")
    ufs.mkdirs("/w/b")
    with ufs.create("/w/a/f1") as f:
        f.write(b"1")
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"},
                             work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        fs.mount("/h", f"hdfs://127.0.0.1:{dfs.port}/w", properties={"dfs.blocksize": "256k"})
        m = c.master.fs_master
        m.start_sync("/h/a")
        m.active_sync_heartbeat()                       # first round: full sync, feed starts now
        mid = m.sync_points["/h/a"]
        tx0 = m.active_sync_txids[mid]
        assert tx0 == len(dfs.edits)
        with ufs.create("/w/a/f2") as f:
            f.write(b"22")
        ufs.rename_file("/w/a/f1", "/w/a/f1r")
        with ufs.create("/w/b/outside") as f:           # not under the sync point: ignored
            f.write(b"x")
        before = dfs.calls.count("getListing")
        m.active_sync_heartbeat()
        assert m.active_sync_txids[mid] == len(dfs.edits) > tx0
        assert dfs.calls.count("getListing") > before
        names = sorted(s.name for s in fs.list_status("/h/a", load_metadata="NEVER"))
        assert names == ["f1r", "f2"]
        assert fs.read_file("/h/a/f2") == b"22"
        ents = list(m.journal_entries())
        assert any(e.HasField("active_sync_tx_id") and e.active_sync_tx_id.tx_id == len(dfs.edits) for e in ents)
        ufs.delete_file("/w/a/f2")
        m.active_sync_heartbeat()
        assert sorted(s.name for s in fs.list_status("/h/a", load_metadata="NEVER")) == ["f1r"]
        fs.unmount("/h")


def test_hdfs_acls_roundtrip_and_master_propagation(dfs, tmp_path):
    """setAcl/getAclStatus through the UFS (SupportedHdfsAclProvider), and an Alluxio setfacl on a
    persisted file propagating the full ACL to HDFS."""
    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.security.acl import AclEntry
    ufs = _ufs(dfs)
    with ufs.create("/acl/f") as f:
        f.write(b"x")
    spec = [AclEntry.parse(x) for x in ("user::rw-", "user:alice:r-x", "group::r--", "mask::r-x", "other::---",
                                        "default:user::rwx", "default:group::r-x", "default:other::r--")]
    ufs.set_acl_entries("/acl/f", spec)
    acl, dacl = ufs.get_acl_pair("/acl/f")
    assert acl.named_users == {"alice": 5} and acl.mask == 5 and (acl.mode >> 6) & 7 == 6 and acl.mode & 7 == 0
    assert dacl is not None and (dacl.mode >> 6) & 7 == 7
    assert ufs.get_acl_pair("/acl/none") is None
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"},
                             work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        fs.mount("/h", f"hdfs://127.0.0.1:{dfs.port}/acl", properties={"dfs.blocksize": "256k"})
        fs.write_file("/h/g", b"data", write_type="CACHE_THROUGH")
        c.master.fs_master.set_acl("/h/g", "MODIFY", [AclEntry.parse("user:bob:rw-")])
        acl2, _ = ufs.get_acl_pair("/acl/g")
        assert acl2.named_users == {"bob": 6}
        fs.unmount("/h")


def test_ha_nameservice_fails_over_from_standby(dfs):
    """hdfs://<nameservice>/ with two NameNodes: calls to the standby (StandbyException) and to a
    dead address fail over to the active one (ConfiguredFailoverProxyProvider semantics)."""
    from alluxio_amd.proxy.hdfs_gateway import IpcServer, RpcError

    def standby(method, body, user):
        raise RpcError("org.apache.hadoop.ipc.StandbyException",
                       "Operation category READ is not supported in state standby")
    sb = IpcServer(standby)
    try:
        props = {"dfs.ha.namenodes.mycluster": "nn1,nn2,nn3",
                 "dfs.namenode.rpc-address.mycluster.nn1": f"127.0.0.1:{sb.port}",
                 "dfs.namenode.rpc-address.mycluster.nn2": "127.0.0.1:1",          # nothing listens
                 "dfs.namenode.rpc-address.mycluster.nn3": f"127.0.0.1:{dfs.port}",
                 "dfs.blocksize": "256k", "dfs.replication": "1"}
        ufs = create_ufs("hdfs://mycluster/", properties=props)
        assert ufs.mkdirs("/ha/d")
        with ufs.create("/ha/d/f") as f:
            f.write(b"ha" * 1000)
        with ufs.open("/ha/d/f") as f:
            assert f.read() == b"ha" * 1000
        assert ufs.nn.active == 2 and ufs.nn.port == dfs.port
    finally:
        sb.stop()
