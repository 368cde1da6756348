"""Job service + stress benches on an in-process cluster (CPU; DRAM tiers).

Mirrors the reference's job integration tests (tests/.../job/plan/*IntegrationTest: load,
persist, replicate, evict, migrate; JobMaster status/cancel) and the stress-bench smoke tests
(stress/shell/src/test: each bench runs end-to-end with tiny parameters)."""
import os
import time

import pytest

from alluxio_amd.job import (CompositeConfig, EvictConfig, JobConfig, LoadConfig, MigrateConfig,
                             PersistConfig, ReplicateConfig, StressBenchConfig)
from alluxio_amd.minicluster import LocalAlluxioCluster

MB = 1 << 20
CONF = {"alluxio.worker.tieredstore.level0.dirs.path": "dram",
        "alluxio.user.block.size.bytes.default": "1MB"}


@pytest.fixture
def cluster():
    with LocalAlluxioCluster(num_workers=2, conf=CONF) as c:
        yield c


def test_job_config_roundtrip():
    cfg = CompositeConfig(jobs=[LoadConfig(path="/a", replication=2), PersistConfig(path="/b")], sequential=True)
    back = JobConfig.from_bytes(cfg.to_bytes())
    assert isinstance(back, CompositeConfig) and back.sequential
    assert isinstance(back.jobs[0], LoadConfig) and back.jobs[0].replication == 2
    assert isinstance(back.jobs[1], PersistConfig) and back.jobs[1].path == "/b"


def test_job_workers_register(cluster):
    assert len(cluster.master.job_master.workers) == 2
    from alluxio_amd.job import JobClient
    from alluxio_amd.rpc import Channel
    cluster.drive_jobs()
    assert len(JobClient(Channel(cluster.master.address)).worker_health()) == 2


def test_load_job(cluster):
    fs = cluster.client()
    data = os.urandom(3 * MB + 17)
    fs.write_file("/load/f", data, write_type="THROUGH")
    assert fs.get_status("/load/f").in_alluxio_percentage == 0
    status, result, err = cluster.run_job(LoadConfig(path="/load", replication=1))
    assert status == "COMPLETED", err
    assert result["bytes_loaded"] == len(data)
    cluster.heartbeat_workers()
    assert fs.get_status("/load/f").in_alluxio_percentage == 100
    assert fs.read_file("/load/f", read_type="NO_CACHE") == data
    fs.close()


def test_persist_job_via_scheduler(cluster):
    fs = cluster.client()
    fs.write_file("/p/f", b"async bytes" * 1000, write_type="ASYNC_THROUGH")
    assert fs.get_status("/p/f").info.persistenceState == "TO_BE_PERSISTED"
    fsm = cluster.master.fs_master
    assert fsm.persistence_scheduler_heartbeat() == 1
    for _ in range(500):
        cluster.drive_jobs()
        time.sleep(0.01)
        if fs.get_status("/p/f").info.persistenceState == "PERSISTED":
            break
    assert fs.get_status("/p/f").info.persistenceState == "PERSISTED"
    with open(os.path.join(cluster.ufs_root, "p", "f"), "rb") as f:
        assert f.read() == b"async bytes" * 1000
    fs.close()


def test_replicate_and_evict(cluster):
    fs = cluster.client()
    fs.write_file("/r/f", os.urandom(MB), write_type="MUST_CACHE")
    cluster.heartbeat_workers()
    bid = fs.get_status("/r/f").block_ids[0]
    assert len(fs.get_block_locations("/r/f")[0].locations) == 1 if hasattr(
        fs.get_block_locations("/r/f")[0], "locations") else True
    status, _, err = cluster.run_job(ReplicateConfig(block_id=bid, replicas=1, path="/r/f"))
    assert status == "COMPLETED", err
    cluster.heartbeat_workers()
    holders = [w for w in cluster.workers if w.worker.has_block(bid)]
    assert len(holders) == 2
    status, _, err = cluster.run_job(EvictConfig(block_id=bid, replicas=1))
    assert status == "COMPLETED", err
    assert sum(w.worker.has_block(bid) for w in cluster.workers) == 1
    fs.close()


def test_migrate_copy_and_move(cluster):
    fs = cluster.client()
    for i in range(3):
        fs.write_file(f"/src/d/f{i}", bytes([i]) * (MB + i), write_type="CACHE_THROUGH")
    status, result, err = cluster.run_job(MigrateConfig(source="/src", destination="/dst", write_type="CACHE_THROUGH"))
    assert status == "COMPLETED", err
    assert result["files"] == 3
    for i in range(3):
        assert fs.read_file(f"/dst/d/f{i}") == bytes([i]) * (MB + i)
    status, _, err = cluster.run_job(MigrateConfig(source="/dst/d/f0", destination="/moved", delete_source=True,
                                                   write_type="MUST_CACHE"))
    assert status == "COMPLETED", err
    assert not fs.exists("/dst/d/f0") and fs.read_file("/moved") == bytes([0]) * MB
    fs.close()


def test_failed_job_and_composite(cluster):
    status, _, err = cluster.run_job(MigrateConfig(source="/nope", destination="/x"))
    assert status == "FAILED" and "nope" in err
    fs = cluster.client()
    fs.write_file("/c/a", b"a" * 100, write_type="THROUGH")
    status, _, err = cluster.run_job(CompositeConfig(jobs=[LoadConfig(path="/c/a"),
                                                           MigrateConfig(source="/c/a", destination="/c/b")],
                                                     sequential=True))
    assert status == "COMPLETED", err
    assert fs.read_file("/c/b") == b"a" * 100
    jm = cluster.master.job_master
    summary = jm.summary()
    assert sum(s.count for s in summary.summaryPerStatus) >= 3
    assert jm.purge_finished(0.0) >= 3
    fs.close()


def test_lost_job_worker_fails_tasks(cluster):
    jm = cluster.master.job_master
    jm.worker_timeout = 0.0
    assert len(jm.detect_lost_workers()) == 2
    assert not jm.workers
    cluster.drive_jobs()   # job workers get a Register command and come back
    cluster.drive_jobs()
    assert len(jm.workers) == 2


@pytest.mark.parametrize("op", ["CreateFile", "GetFileStatus", "ListDir", "CreateDir", "RenameFile", "DeleteFile",
                                "OpenFile", "GetBlockLocations"])
def test_master_bench_ops(cluster, op):
    from alluxio_amd.stress.master_bench import main
    fs = cluster.client()
    extra = []
    if op in ("RenameFile", "DeleteFile"):
        # as in the reference: they consume the paths a preceding CreateFile run made
        c = main(["--operation", "CreateFile", "--threads", "4", "--duration", "10s", "--warmup", "0ms",
                  "--fixed-count", "5", "--stop-count", "40"], fs=fs, print_result=False)
        assert not c["errors"] and c["completed"] == 40
        extra = ["--stop-count", "40"]
    r = main(["--operation", op, "--threads", "4", "--duration", "300ms", "--warmup", "0ms" if extra else "50ms",
              "--fixed-count", "5"] + extra, fs=fs, print_result=False)
    assert not r["errors"], r["errors"]
    assert r["ops"] > 0 and r["throughput_ops"] > 0
    if op == "DeleteFile":
        assert fs.list_status("/stress-master-base/fixed") == [] and r["completed"] == 40
    fs.close()


def test_master_bench_stop_count_and_rate(cluster):
    from alluxio_amd.stress.master_bench import main
    fs = cluster.client()
    r = main(["--operation", "CreateFile", "--threads", "4", "--duration", "5s", "--warmup", "0s",
              "--stop-count", "40"], fs=fs, print_result=False)
    assert r["ops"] == 40
    r = main(["--operation", "GetFileStatus", "--threads", "2", "--duration", "500ms", "--warmup", "0s",
              "--target-throughput", "100", "--fixed-count", "2"], fs=fs, print_result=False)
    assert r["throughput_ops"] < 150
    fs.close()


def test_worker_and_client_io_bench(cluster):
    from alluxio_amd.stress.client_io_bench import main as cio
    from alluxio_amd.stress.worker_bench import main as wb
    fs = cluster.client(metadata_cache=True)
    r = wb(["--threads", "4", "--file-size", "2m", "--buffer-size", "64k", "--block-size", "1m",
            "--duration", "300ms", "--warmup", "50ms"], fs=fs, print_result=False)
    assert not r["errors"] and r["bytes"] > 0
    r = wb(["--threads", "8", "--file-size", "2m", "--buffer-size", "64k", "--block-size", "1m",
            "--duration", "300ms", "--warmup", "50ms", "--mode", "batched"], fs=fs, print_result=False)
    assert r["bytes"] > 0
    for op in ("Write", "Read", "ReadFully", "PosReadFully"):
        r = cio(["--operation", op, "--threads", "1,2", "--file-size", "1m", "--buffer-size", "256k",
                 "--duration", "200ms"], fs=fs, print_result=False)
        assert not r["errors"], r["errors"]
        assert r["bytes"] > 0
    fs.close()


def test_ufs_io_bench(tmp_path):
    from alluxio_amd.stress.ufs_io_bench import main
    r = main(["--path", str(tmp_path / "ufsio"), "--threads", "2", "--io-size", "1m", "--buffer-size", "256k"],
             print_result=False)
    assert not r["errors"] and r["read"]["MBps"] > 0 and r["write"]["MBps"] > 0


def test_stress_via_job_service(cluster):
    status, result, err = cluster.run_job(StressBenchConfig(
        bench="master", args=["--operation", "CreateFile", "--threads", "2", "--duration", "200ms",
                              "--warmup", "0s"]))
    assert status == "COMPLETED", err
    assert result["workers"] == 2 and result["ops"] > 0 and not result["errors"]


def test_max_throughput(cluster):
    from alluxio_amd.stress.max_throughput import main
    fs = cluster.client()
    r = main(["--operation", "GetFileStatus", "--threads", "2", "--duration", "200ms", "--lo", "10",
              "--hi", "400", "--iterations", "3"], fs=fs, print_result=False)
    assert r["max_ops"] > 0 and len(r["trace"]) >= 1
    fs.close()


def test_replicated_write_pulls_from_primary(cluster):
    """replication_min=2: the write lands on two workers at once (reference
    AlluxioBlockStore.getOutStream initialReplicas); the second copy is pulled out of the primary's
    shared arena by the replica (PeerTransfer), not streamed by the client."""
    fs = cluster.client()
    data = os.urandom(MB + 17)
    fs.write_file("/rep/w", data, write_type="MUST_CACHE", replication_min=2)
    cluster.heartbeat_workers()
    bid = fs.get_status("/rep/w").block_ids[0]
    assert sum(w.worker.has_block(bid) for w in cluster.workers) == 2
    pulled = sum(w.worker.metrics.counter("PeerSharedBytesReceived").count for w in cluster.workers)
    assert pulled >= len(data)
    assert fs.read_file("/rep/w") == data
    fs.close()


def test_replication_checker(cluster):
    fs = cluster.client()
    fs.write_file("/rep/f", os.urandom(MB), write_type="MUST_CACHE")
    fs.set_attribute("/rep/f", replication_min=2)
    cluster.heartbeat_workers()
    bid = fs.get_status("/rep/f").block_ids[0]
    rc = cluster.master.replication_checker
    assert rc.heartbeat() == 1
    for _ in range(300):
        cluster.drive_jobs()
        if sum(w.worker.has_block(bid) for w in cluster.workers) == 2:
            break
        time.sleep(0.01)
    assert sum(w.worker.has_block(bid) for w in cluster.workers) == 2
    for _ in range(300):         # the copy landed; let the job report COMPLETED before re-checking
        if not rc.handler._running(("replicate", bid)):
            break
        cluster.drive_jobs()
        time.sleep(0.01)
    cluster.heartbeat_workers()
    assert rc.heartbeat() == 0   # satisfied
    fs.set_attribute("/rep/f", replication_min=0, replication_max=1)
    assert rc.heartbeat() == 1
    for _ in range(300):
        cluster.drive_jobs()
        if sum(w.worker.has_block(bid) for w in cluster.workers) == 1:
            break
        time.sleep(0.01)
    assert sum(w.worker.has_block(bid) for w in cluster.workers) == 1
    fs.close()


def _drive_until(cluster, cond, n=500):
    for _ in range(n):
        cluster.drive_jobs()
        if cond():
            return True
        time.sleep(0.01)
    return cond()


def test_replication_checker_pins_to_medium_and_recaches_from_ufs(tmp_path):
    """Mis-replication: a file pinned to SSD whose block sits in MEM is moved into the SSD tier by a
    move job (ReplicationChecker.checkMisreplicated -> migrate).  Under-replication at 0 copies: a
    persisted file's freed block is re-cached from the UFS by the replicate job."""
    conf = {"alluxio.worker.tieredstore.levels": "2",
            "alluxio.worker.tieredstore.level0.alias": "MEM",
            "alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": "16MB",
            "alluxio.worker.tieredstore.level1.alias": "SSD",
            "alluxio.worker.tieredstore.level1.dirs.path": str(tmp_path / "ssd"),
            "alluxio.worker.tieredstore.level1.dirs.quota": "64MB",
            "alluxio.worker.tieredstore.level1.dirs.mediumtype": "SSD",
            "alluxio.worker.hbm.page.size": "256KB",
            "alluxio.user.block.size.bytes.default": "1MB"}
    os.makedirs(tmp_path / "ssd", exist_ok=True)
    with LocalAlluxioCluster(num_workers=1, conf=conf) as c:
        fs = c.client()
        w = c.workers[0].worker
        rc = c.master.replication_checker
        data = os.urandom(MB)
        fs.write_file("/pin/f", data, write_type="CACHE_THROUGH")
        bid = fs.get_status("/pin/f").block_ids[0]
        assert w.native.block_info(bid).medium == "DRAM"
        fs.set_attribute("/pin/f", pinned=True, pinned_media=["SSD"])
        assert rc.heartbeat() == 1                        # one move job
        assert _drive_until(c, lambda: w.native.block_info(bid).medium == "SSD")
        c.heartbeat_workers()
        assert fs.read_file("/pin/f") == data
        assert _drive_until(c, lambda: not rc.handler._running(("move", bid)))
        assert rc.heartbeat() == 0                        # in place now
        # the cached copy is freed: the pinned, persisted file is re-cached from the UFS
        fs.set_attribute("/pin/f", pinned=False)
        fs.set_attribute("/pin/f", replication_min=1)
        w.remove_block(1, bid)
        c.heartbeat_workers()
        assert fs.get_status("/pin/f").in_alluxio_percentage == 0
        assert rc.heartbeat() == 1
        assert _drive_until(c, lambda: w.has_block(bid))
        assert fs.read_file("/pin/f") == data
        fs.close()
