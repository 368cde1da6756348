"""ReplicationChecker parity with the reference's ReplicationCheckerTest
(core/server/master/src/test/java/alluxio/master/file/replication/ReplicationCheckerTest.java:254-406)
plus the durable-replication, lost/persisted, safe-mode and job-service back-off rules of
ReplicationChecker.java:127-317.  In-process master, no workers: block locations are made by
registering fake workers and committing / heartbeating blocks into the block master."""
import pytest

from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.master.replication import (JobServiceBusy, ReplicationChecker, ReplicationHandler)
from alluxio_amd.proto import pb


class MockHandler(ReplicationHandler):
    def __init__(self):
        self.evicts, self.replicates, self.migrates = {}, {}, {}
        self.busy = False

    def evict(self, path, block_id, num_replicas):
        if self.busy:
            raise JobServiceBusy("busy")
        self.evicts[block_id] = num_replicas
        return 0

    def replicate(self, path, block_id, num_replicas):
        if self.busy:
            raise JobServiceBusy("busy")
        self.replicates[block_id] = num_replicas
        return 0

    def migrate(self, path, block_id, worker_host, medium):
        self.migrates[block_id] = (worker_host, medium)
        return 0


class _NoSafeMode:
    on = False

    def in_safe_mode(self):
        return self.on


@pytest.fixture
def env(tmp_path):
    conf = Configuration({"alluxio.master.journal.folder": str(tmp_path / "journal"),
                          "alluxio.security.authorization.permission.enabled": "false"})
    m = AlluxioMasterProcess(conf, port=0, enable_grpc=False, root_ufs=str(tmp_path / "ufs"))
    m.start(start_heartbeats=False)
    h = MockHandler()
    sm = _NoSafeMode()
    checker = ReplicationChecker(m.fs_master, h, safe_mode=sm)
    checker.sleep = lambda s: None
    workers = {}

    def worker(i):
        if i not in workers:
            bm = m.block_master
            wid = bm.get_worker_id(pb.grpc.WorkerNetAddress(host=f"host{i}", rpcPort=1000, dataPort=2000))
            bm.worker_register(wid, ["MEM"], {"MEM": 100 << 20}, {"MEM": 0}, {})
            workers[i] = wid
        return workers[i]

    def create(path, rmin=0, rmax=-1, durable=1, pin_medium="", write_type="MUST_CACHE", locations=0,
               medium="MEM"):
        """A completed one-block file; its block on `locations` workers (0: known only to the UFS)."""
        fs = m.fs_master
        fs.create_file(path, block_size=1024, replication_min=rmin, replication_max=rmax,
                       replication_durable=durable, write_type=write_type)
        bid = fs.get_new_block_id_for_file(path)
        if locations:
            add_locations(bid, locations, medium)
        else:
            m.block_master.commit_block_in_ufs(bid, 20)
        fs.complete_file(path, ufs_length=20 if write_type in ("THROUGH", "CACHE_THROUGH") else 0)
        if pin_medium:
            fs.set_attribute(path, pinned=True, pinned_media=[pin_medium])
        return bid

    def add_locations(bid, n, medium="MEM", start=0):
        bm = m.block_master
        for i in range(start, start + n):
            wid = worker(i)
            if i == start and bm.block_info_or_none(bid) is None:
                bm.commit_block(wid, 50, "MEM", medium, bid, 20)
            else:
                bm.worker_heartbeat(wid, {"MEM": 0}, [], {("MEM", medium): [bid]})

    yield m, checker, h, sm, create, add_locations, worker
    m.stop()


def test_heartbeat_when_tree_is_empty(env):
    m, checker, h, *_ = env
    checker.heartbeat()
    assert h.evicts == {} and h.replicates == {}


def test_file_within_range(env):
    m, checker, h, sm, create, add, worker = env
    bid = create("/test1", rmin=1, rmax=3, locations=1)
    checker.heartbeat()
    assert h.evicts == {} and h.replicates == {}
    add(bid, 1, start=1)                       # two replicas
    checker.heartbeat()
    assert h.evicts == {} and h.replicates == {}
    add(bid, 1, start=2)                       # three: meets the max
    checker.heartbeat()
    assert h.evicts == {} and h.replicates == {}


def test_file_under_replicated_by_1(env):
    m, checker, h, sm, create, *_ = env
    bid = create("/test1", rmin=1)
    checker.heartbeat()
    assert h.evicts == {} and h.replicates == {bid: 1}


def test_file_needs_move(env):
    m, checker, h, sm, create, *_ = env
    bid = create("/test1", rmin=1, pin_medium="SSD", locations=1)
    checker.heartbeat()
    assert h.evicts == {} and h.replicates == {}
    assert h.migrates == {bid: ("host0", "SSD")}


def test_file_does_not_need_move(env):
    m, checker, h, sm, create, *_ = env
    create("/test1", rmin=1, pin_medium="MEM", locations=1)
    checker.heartbeat()
    assert h.evicts == {} and h.replicates == {} and h.migrates == {}


def test_pin_to_hbm_moves_dram_copies(env):
    """The MI355X case: `pin /ds HBM` on a file cached in DRAM asks the holder to move it."""
    m, checker, h, sm, create, *_ = env
    bid = create("/ds", locations=1, medium="MEM")
    m.fs_master.set_attribute("/ds", pinned=True, pinned_media=["HBM", "NOPE"])
    st = m.fs_master.get_status("/ds")
    assert st.replicationMin == 1 and st.pinned
    with m.fs_master.tree.lock.read():
        assert m.fs_master.tree.get("/ds").medium_types == ["HBM"]
    checker.heartbeat()
    assert h.migrates == {bid: ("host0", "HBM")}
    m.fs_master.set_attribute("/ds", pinned=False)         # unpinned: min back to 0, no more moves
    h.migrates.clear()
    checker.heartbeat()
    assert h.migrates == {} and m.fs_master.get_status("/ds").replicationMin == 0


def test_file_under_replicated_by_10(env):
    m, checker, h, sm, create, *_ = env
    bid = create("/test1", rmin=10)
    checker.heartbeat()
    assert h.evicts == {} and h.replicates == {bid: 10}


def test_multiple_files_under_replicated(env):
    m, checker, h, sm, create, *_ = env
    b1 = create("/test1", rmin=1)
    b2 = create("/test2", rmin=2)
    checker.heartbeat()
    assert h.evicts == {} and h.replicates == {b1: 1, b2: 2}


def test_file_under_replicated_and_lost(env):
    m, checker, h, sm, create, add, worker = env
    bid = create("/test1", rmin=2, locations=1)
    m.block_master.worker_heartbeat(worker(0), {"MEM": 0}, [bid], {})     # the only copy is gone
    assert bid in m.block_master.lost_blocks()
    checker.heartbeat()
    assert h.evicts == {} and h.replicates == {}


def test_lost_block_of_persisted_file_is_recached(env):
    """A persisted file's lost block is re-replicated: the replicate job reads it from the UFS."""
    m, checker, h, sm, create, add, worker = env
    bid = create("/p", rmin=1, locations=1, write_type="CACHE_THROUGH")
    m.block_master.worker_heartbeat(worker(0), {"MEM": 0}, [bid], {})
    checker.heartbeat()
    assert h.replicates == {bid: 1}


def test_file_over_replicated_by_1(env):
    m, checker, h, sm, create, *_ = env
    bid = create("/test1", rmax=1, locations=2)
    checker.heartbeat()
    assert h.evicts == {bid: 1} and h.replicates == {}


def test_file_over_replicated_by_10(env):
    m, checker, h, sm, create, *_ = env
    bid = create("/test1", rmax=1, locations=11)
    checker.heartbeat()
    assert h.evicts == {bid: 10} and h.replicates == {}


def test_multiple_files_over_replicated(env):
    m, checker, h, sm, create, *_ = env
    b1 = create("/test1", rmax=1, locations=2)
    b2 = create("/test2", rmax=2, locations=4)
    checker.heartbeat()
    assert h.evicts == {b1: 1, b2: 2} and h.replicates == {}


def test_files_under_and_over_replicated(env):
    m, checker, h, sm, create, *_ = env
    b1 = create("/test1", rmin=2, rmax=-1, locations=1)
    b2 = create("/test2", rmin=0, rmax=3, locations=5)
    checker.heartbeat()
    assert h.evicts == {b2: 2} and h.replicates == {b1: 1}


def test_durable_replication_while_to_be_persisted(env):
    """ASYNC_THROUGH before its persist job finished: the minimum (and maximum) is
    replicationDurable; once persisted, replicationMin again."""
    m, checker, h, sm, create, *_ = env
    fs = m.fs_master
    fs.create_file("/a", block_size=1024, replication_min=1, replication_durable=3, write_type="ASYNC_THROUGH")
    bid = fs.get_new_block_id_for_file("/a")
    env[5](bid, 1)
    fs.complete_file("/a", async_persist=True)
    assert fs.get_status("/a").persistenceState == "TO_BE_PERSISTED"
    checker.heartbeat()
    assert h.replicates == {bid: 2}
    fs.set_attribute("/a", persisted=True)
    h.replicates.clear()
    checker.heartbeat()
    assert h.replicates == {}


def test_safe_mode_skips_and_busy_job_service_backs_off(env):
    m, checker, h, sm, create, *_ = env
    bid = create("/test1", rmin=2)
    sm.on = True
    assert checker.heartbeat() == 0 and h.replicates == {}
    sm.on = False
    h.busy = True
    slept = []
    checker.sleep = slept.append
    checker.heartbeat()
    assert checker.quiet_period_s == 1
    checker.heartbeat()
    assert slept == [1] and checker.quiet_period_s == 2
    h.busy = False
    checker.heartbeat()
    assert h.replicates == {bid: 2} and checker.quiet_period_s == 1
