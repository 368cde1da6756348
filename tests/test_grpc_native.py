"""gRPC served by the native front end (csrc/frame_rpc.cpp, H2): a stock grpcio client -- the
protocol a Java Alluxio client speaks -- authenticates over SaslAuthenticationService and calls the
FileSystemMaster on the native port; unary and server-streaming calls, errors (grpc-status /
grpc-message), unknown methods and the reply cache all go through the C++ HTTP/2 path.
Reference: core/common/src/main/proto/grpc/file_system_master.proto (FileSystemMasterClientService),
sasl_server.proto (SaslAuthenticationService.authenticate)."""
import grpc
import pytest

from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.ops.native import lib
from alluxio_amd.proto import SERVICES, pb
from alluxio_amd.rpc import Channel
from alluxio_amd.utils import exceptions as ex

FS = "alluxio.grpc.file.FileSystemMasterClientService"

pytestmark = pytest.mark.skipif(not lib().FrameRpcServer.grpc_available(), reason="libnghttp2 not present")


@pytest.fixture
def cluster(tmp_path):
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                                                  "alluxio.security.authorization.permission.enabled": "false"},
                             work_dir=str(tmp_path / "c")) as c:
        yield c


def _status(fs, path, user):
    return fs.get_status(path)


def test_grpc_client_on_native_port(cluster):
    m = cluster.master
    port = m.native_rpc.port
    fs = cluster.client()
    fs.create_directory("/d")
    fs.write_file("/d/a", b"x" * 100)
    srv = m.native_rpc.server
    before = srv.grpc_requests
    ch = Channel(f"127.0.0.1:{port}", user="alice", force_grpc=True, native=False)
    try:
        st = ch.stub(FS)
        r = st.GetStatus(pb.file.GetStatusPRequest(path="/d/a"))
        assert r.fileInfo.path == "/d/a" and r.fileInfo.length == 100
        assert ch.channel_id is not None                    # the SASL handshake ran natively
        # server streaming: ListStatus
        items = [fi.path for resp in st.ListStatus(pb.file.ListStatusPRequest(path="/d")) for fi in resp.fileInfos]
        assert items == ["/d/a"]
        # a mutation as the authenticated channel user
        st.CreateDirectory(pb.file.CreateDirectoryPRequest(path="/d/byalice"))
        assert fs.get_status("/d/byalice").info.owner == "alice"
        # errors travel as grpc-status / grpc-message
        with pytest.raises(ex.NotFoundException) as ei:
            st.GetStatus(pb.file.GetStatusPRequest(path="/d/missing-é"))
        assert "missing" in str(ei.value)
        # repeat lookups: answered from the native reply cache on the I/O thread
        hits = srv.cache_hits
        for _ in range(5):
            st.GetStatus(pb.file.GetStatusPRequest(path="/d/a"))
        assert srv.cache_hits >= hits + 4
        assert srv.grpc_requests >= before + 9
    finally:
        ch.close()
    # unknown method, and a call without an authenticated channel
    raw = grpc.insecure_channel(f"127.0.0.1:{port}")
    try:
        bogus = raw.unary_unary("/alluxio.grpc.file.FileSystemMasterClientService/NoSuchMethod",
                                lambda b: b, lambda b: b)
        with pytest.raises(grpc.RpcError) as ei:
            bogus(b"")
        assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
        spec = SERVICES[FS]["GetStatus"]
        call = raw.unary_unary(spec.path, spec.request.SerializeToString, spec.response.FromString)
        with pytest.raises(grpc.RpcError) as ei:
            call(pb.file.GetStatusPRequest(path="/d/a"))
        assert ei.value.code() == grpc.StatusCode.UNAUTHENTICATED
        # a large server-streaming reply crosses the HTTP/2 flow-control window
        for i in range(3000):
            fs.create_directory(f"/big/dir-with-a-long-name-{i:05d}", recursive=True)
        ch2 = Channel(f"127.0.0.1:{port}", user="alice", force_grpc=True, native=False)
        try:
            n = sum(len(r.fileInfos) for r in ch2.stub(FS).ListStatus(pb.file.ListStatusPRequest(path="/big")))
            assert n == 3000
        finally:
            ch2.close()
    finally:
        raw.close()
        fs.close()


def test_master_port_served_natively(tmp_path):
    """alluxio.master.rpc.native.grpc.enabled: the master RPC port is the native front end; gRPC
    and framed-RPC clients share it (protocol detected per connection)."""
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                                                  "alluxio.master.rpc.native.grpc.enabled": "true"},
                             work_dir=str(tmp_path / "c")) as c:
        m = c.master
        assert m.native_rpc is not None and m.server.port == m.native_rpc.port
        assert m.server._server is None                      # no grpcio server on the master
        addr = f"127.0.0.1:{m.server.port}"
        fs = c.client()
        fs.write_file("/f", b"abc")
        g = Channel(addr, user="bob", force_grpc=True, native=False)
        n = Channel(addr, user="bob", force_grpc=True)      # probes over gRPC, then framed RPC
        try:
            assert g.stub(FS).GetStatus(pb.file.GetStatusPRequest(path="/f")).fileInfo.length == 3
            g.stub(FS).CreateDirectory(pb.file.CreateDirectoryPRequest(path="/viagrpc"))
            assert n.stub(FS).GetStatus(pb.file.GetStatusPRequest(path="/viagrpc")).fileInfo.folder
            assert n._native is not None
            assert m.native_rpc.server.grpc_requests >= 3
        finally:
            g.close()
            n.close()
            fs.close()
