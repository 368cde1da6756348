"""HA masters: FILE_LOCK election, standby journal tailing, failover with client + worker
retargeting (reference tests/.../master/MasterFaultToleranceIntegrationTest: kill the leader,
a standby takes over, namespace and cached data survive)."""
import os

import pytest

from alluxio_amd.master.ha import FileLockPrimarySelector
from alluxio_amd.minicluster import MultiMasterLocalAlluxioCluster
from alluxio_amd.utils.exceptions import UnavailableException


def test_file_lock_selector(tmp_path):
    lock = str(tmp_path / "primary.lock")
    got = []
    a, b = FileLockPrimarySelector(lock, 0.01), FileLockPrimarySelector(lock, 0.01)
    a.start(lambda: got.append("a"))
    assert a.wait_primary(5)
    b.start(lambda: got.append("b"))
    assert not b.wait_primary(0.2)
    a.stop()
    assert b.wait_primary(5)
    assert got == ["a", "b"]
    b.stop()


@pytest.mark.parametrize("grpc", [False, True])
def test_failover(grpc):
    with MultiMasterLocalAlluxioCluster(num_masters=2, num_workers=1, grpc=grpc,
                                        conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                                              "alluxio.user.block.size.bytes.default": "1MB"}) as c:
        fs = c.client()
        standby = [m for m in c.masters if not m.primary][0]
        # a standby refuses RPCs
        from alluxio_amd.rpc import Channel
        from alluxio_amd.proto import pb
        with pytest.raises(UnavailableException):
            Channel(standby.address).stub("alluxio.grpc.file.FileSystemMasterClientService").GetStatus(
                pb.file.GetStatusPRequest(path="/"))
        data = os.urandom(3 << 20)
        fs.write_file("/ha/f", data, write_type="MUST_CACHE")
        fs.create_directory("/ha/d/e", recursive=True)
        old = c.primary()
        new = c.kill_primary()
        assert new is not old and new.primary
        # namespace survived (journal replay on the new primary); the client followed it
        assert fs.get_status("/ha/f").length == len(data)
        assert fs.exists("/ha/d/e")
        # worker re-registers with the new primary on its next heartbeat, then data is served
        c.heartbeat_workers()
        c.heartbeat_workers()
        assert fs.get_status("/ha/f").in_alluxio_percentage == 100
        assert fs.read_file("/ha/f") == data
        fs.write_file("/ha/g", b"after failover", write_type="MUST_CACHE")
        assert fs.read_file("/ha/g") == b"after failover"
        fs.close()
