"""Channel authentication (reference core/common/src/test/.../authentication/*: SIMPLE accepts any
user, CUSTOM consults the provider, unauthenticated channels are rejected, the server takes the user
from the authenticated channel rather than per-call claims)."""
import grpc
import pytest

from alluxio_amd.conf import Configuration
from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.proto import SERVICES, pb
from alluxio_amd.rpc import Channel
from alluxio_amd.utils.exceptions import UnauthenticatedException


def check_password(user, password):
    return password == "s3cret"


def test_simple_auth_and_rejects_unauthenticated():
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"}) as c:
        fs = c.client()
        fs.write_file("/a/f", b"x", write_type="MUST_CACHE")   # SIMPLE handshake under the hood
        # a raw gRPC call without a channel id is refused
        ch = grpc.insecure_channel(c.master.address)
        spec = SERVICES["alluxio.grpc.file.FileSystemMasterClientService"]["GetStatus"]
        call = ch.unary_unary(spec.path, spec.request.SerializeToString, spec.response.FromString)
        with pytest.raises(grpc.RpcError) as e:
            call(pb.file.GetStatusPRequest(path="/a/f"), metadata=(("alluxio-user", "root"),))
        assert e.value.code() == grpc.StatusCode.UNAUTHENTICATED
        ch.close()
        # the owner is the authenticated user of the channel
        ch2 = Channel(c.master.address, user="carol", force_grpc=True)
        ch2.stub("alluxio.grpc.file.FileSystemMasterClientService").CreateDirectory(
            pb.file.CreateDirectoryPRequest(path="/carol", options=pb.file.CreateDirectoryPOptions()))
        assert fs.get_status("/carol").info.owner == "carol"
        fs.close()


def test_custom_auth_provider():
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.security.authentication.type": "CUSTOM",
            "alluxio.security.authentication.custom.provider.class": "tests.test_auth:check_password",
            "alluxio.security.login.password": "s3cret"}
    with LocalAlluxioCluster(num_workers=1, conf=conf) as c:
        fs = c.client()
        fs.write_file("/ok", b"y", write_type="MUST_CACHE")
        assert fs.read_file("/ok") == b"y"
        bad = Channel(c.master.address, user="mallory", force_grpc=True, auth=("CUSTOM", "mallory", "nope"))
        with pytest.raises(UnauthenticatedException):
            bad.stub("alluxio.grpc.file.FileSystemMasterClientService").GetStatus(pb.file.GetStatusPRequest(path="/"))
        fs.close()


def test_nosasl_trusts_header():
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                                                  "alluxio.security.authentication.type": "NOSASL"}) as c:
        fs = c.client()
        fs.write_file("/n", b"z", write_type="MUST_CACHE")
        assert fs.read_file("/n") == b"z"
        fs.close()
    assert Configuration().get("alluxio.security.authentication.type") == "SIMPLE"
