"""Masters and workers as separate OS processes (reference MultiProcessCluster-based tests such as
tests/.../server/ft/journal/raft/EmbeddedJournalIntegrationTestFaultTolerance)."""
import os

import pytest

from alluxio_amd.minicluster.multi_process import MultiProcessCluster


@pytest.mark.timeout(300)
def test_processes_kill_primary_and_restart(tmp_path):
    with MultiProcessCluster(num_masters=3, num_workers=1, work_dir=str(tmp_path / "mpc")) as c:
        fs = c.client()
        data = os.urandom(1 << 20)
        fs.write_file("/mp/f", data, write_type="CACHE_THROUGH")
        assert fs.read_file("/mp/f") == data
        old = c.primary_index()
        c.stop_master(old)                          # SIGKILL the primary process
        new = c.wait_for_primary()
        assert new != old
        assert fs.read_file("/mp/f") == data        # the client follows the new primary
        c.wait_for_workers(1)                       # the worker re-registers with the new primary
        fs.write_file("/mp/g", b"after", write_type="CACHE_THROUGH")
        c.start_master(old)                         # comes back as a standby and catches up
        fs.close()
        fs = c.client()
        assert sorted(s.info.name for s in fs.list_status("/mp")) == ["f", "g"]
        fs.close()
