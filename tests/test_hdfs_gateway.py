"""HDFS-protocol gateway (proxy/hdfs_gateway.py): Hadoop clients reach the Alluxio namespace as
``hdfs://gateway:port/`` over Hadoop IPC + DataTransferProtocol, the surface the reference
provides with ``alluxio.hadoop.FileSystem`` (core/client/hdfs/.../AbstractFileSystem.java).  The
client here is this repo's native Hadoop client; Java DFSClient interop is parity unpinned.
"""
import io

import numpy as np
import pytest

from alluxio_amd.cli import ufs_contract
from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.proxy.hdfs_gateway import HdfsGateway
from alluxio_amd.underfs import hadoop_rpc as H
from alluxio_amd.underfs.base import OpenOptions
from alluxio_amd.underfs.registry import create as create_ufs


@pytest.fixture
def gw(tmp_path):
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                                                  "alluxio.user.block.size.bytes.default": "1MB"},
                             work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        g = HdfsGateway(fs)
        try:
            yield g, fs
        finally:
            g.stop()


def test_ufs_contract_through_gateway(gw):
    g, fs = gw
    fs.create_directory("/contract")
    res = ufs_contract.run(f"hdfs://127.0.0.1:{g.port}/contract", properties={"dfs.blocksize": "1m"},
                           out=io.StringIO(), large_file_size=3 << 20)
    assert res["failed"] == [], res["failed"]
    assert len(res["passed"]) >= 40
    assert g.calls.get("addBlock", 0) > 0 and g.calls.get("getBlockLocations", 0) > 0


def test_hadoop_client_reads_and_writes_alluxio_files(gw):
    g, fs = gw
    data = np.random.default_rng(3).integers(0, 256, (5 << 20) + 1234, dtype=np.uint8)
    fs.write_file("/ds/part-0", data, write_type="CACHE_THROUGH")
    ufs = create_ufs(f"hdfs://127.0.0.1:{g.port}/", properties={"dfs.blocksize": "1m"})
    st = ufs.get_status("/ds/part-0")
    assert st.content_length == data.size and st.block_size == 1 << 20
    with ufs.open("/ds/part-0") as f:
        assert f.read() == data.tobytes()                      # 6 Alluxio blocks = 6 HDFS blocks
    with ufs.open("/ds/part-0", OpenOptions(offset=(3 << 20) - 7)) as f:
        assert f.read(100_000) == data[(3 << 20) - 7:(3 << 20) - 7 + 100_000].tobytes()
    # written by the Hadoop client -> visible to Alluxio clients, block by block
    out = np.random.default_rng(4).integers(0, 256, (2 << 20) + 99, dtype=np.uint8).tobytes()
    with ufs.create("/ds/from-hadoop") as f:
        for i in range(0, len(out), 300_001):
            f.write(out[i:i + 300_001])
    assert fs.read_file("/ds/from-hadoop") == out
    assert fs.get_status("/ds/from-hadoop").is_completed
    # namespace calls
    nn = ufs.nn
    d = nn.get_server_defaults()
    assert d.checksumType == H.CHECKSUM_CRC32C and d.bytesPerChecksum == 512
    cs = nn.get_content_summary("/ds")
    assert (cs.fileCount, cs.directoryCount, cs.length) == (2, 1, data.size + len(out))
    assert sorted(s.name for s in ufs.list_status("/ds")) == ["from-hadoop", "part-0"]
    assert ufs.rename_file("/ds/from-hadoop", "/ds/moved") and fs.exists("/ds/moved")
    ufs.set_mode("/ds/moved", 0o600)
    assert fs.get_status("/ds/moved").info.mode & 0o777 == 0o600
    assert ufs.delete_file("/ds/moved") and not fs.exists("/ds/moved")
    with pytest.raises(H.RemoteException, match="RpcNoSuchMethodException"):
        nn.call("getSnapshottableDirListing", H.hdfs.GetFsStatusRequestProto(), H.hdfs.GetFsStatsResponseProto)


def test_block_cut_off_mid_stream_fails_the_file(gw):
    """A WRITE_BLOCK connection that dies mid-block cannot be taken back out of the Alluxio out
    stream: complete() reports an IOException and the partial file is discarded."""
    import time
    g, fs = gw
    nn = H.NameNodeClient("127.0.0.1", g.port, user="u")
    st = nn.create("/cut", 0o644, True, True, 1, 1 << 20)
    lb = nn.add_block("/cut", None, st.fileId)
    w = H.BlockWriter(lb, nn.client_name)
    w.write(b"z" * 200_000)
    w.abort()                                  # connection dropped: no last packet
    deadline = time.time() + 10
    while not g.open_files["/cut"].broken and time.time() < deadline:
        time.sleep(0.02)
    with pytest.raises(H.RemoteException, match="failed mid-stream"):
        nn.complete("/cut", None, st.fileId)
    assert not fs.exists("/cut")


def test_gateway_calls_run_as_the_hadoop_caller(tmp_path):
    """NameNode calls run as the IpcConnectionContext user, not the proxy's: a Hadoop client
    connecting as alice owns what she creates and is refused what she may not touch."""
    from alluxio_amd.utils import exceptions as ex
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.security.authorization.permission.enabled": "true"}
    with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        fs.create_directory("/shared")
        fs.set_attribute("/shared", mode=0o777)          # (create applies the umask)
        fs.create_directory("/private", mode=0o755)
        g = HdfsGateway(fs)
        nn = H.NameNodeClient("127.0.0.1", g.port, user="alice")
        try:
            assert nn.mkdirs("/shared/a", 0o755, False)
            assert fs.get_status("/shared/a").info.owner == "alice"
            with pytest.raises(Exception) as ei:
                nn.mkdirs("/private/b", 0o755, False)
            assert "ermission" in str(ei.value) or "AccessControl" in str(ei.value), ei.value
            assert not fs.exists("/private/b")
            with pytest.raises(Exception):
                nn.delete("/private", True)
            assert fs.exists("/private")
        finally:
            nn.close()
            g.stop()
            fs.close()


def test_gateway_refuses_oversized_rpc_frames(gw):
    import socket
    import struct
    g, _fs = gw
    s = socket.create_connection(("127.0.0.1", g.port))
    try:
        s.sendall(b"hrpc" + bytes([H.IPC_VERSION, 0, H.AUTH_NONE]) + struct.pack(">I", 1 << 30))
        s.settimeout(5)
        assert s.recv(1) == b""                  # closed without reading (or allocating) 1 GiB
    finally:
        s.close()
