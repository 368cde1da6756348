"""Metadata backups: local backup + restore, async status, delegation to a standby master
(UFS-journal FILE_LOCK HA and embedded Raft), delegation refusal / allowLeader fallback, daily
backup scheduling and retention.

Reference tests: tests/src/test/java/alluxio/server/ft/journal/BackupIntegrationTest /
BackupDelegationIntegrationTest (backup taken on a standby, restore from it), core/server/master
DailyMetadataBackupTest (retention).
"""
import datetime
import os
import time

import pytest

from alluxio_amd.conf import Configuration
from alluxio_amd.master.backup import COMPLETED, INITIATING, DailyMetadataBackup
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.minicluster import LocalAlluxioCluster, MultiMasterLocalAlluxioCluster
from alluxio_amd.proto import pb
from alluxio_amd.utils.exceptions import FailedPreconditionException


def _restore(tmp_path, backup_path, name="restored"):
    c = Configuration(load_site=False)
    c.set("alluxio.master.journal.type", "UFS")
    c.set("alluxio.master.journal.folder", str(tmp_path / name))
    c.set("alluxio.web.server.enabled", "false")
    c.set("alluxio.master.journal.init.from.backup", str(backup_path))
    m = AlluxioMasterProcess(c, port=0, enable_grpc=False, root_ufs=str(tmp_path / f"{name}_ufs"))
    m.start(start_heartbeats=False)
    return m


def _meta(cluster_or_fs):
    return cluster_or_fs.ctx.meta_master() if hasattr(cluster_or_fs, "ctx") else cluster_or_fs


def test_local_backup_and_restore(tmp_path):
    with LocalAlluxioCluster(num_workers=1, grpc=False, work_dir=str(tmp_path / "c")) as cluster:
        fs = cluster.client()
        for i in range(5):
            fs.create_directory(f"/dir{i}/sub", recursive=True)
        fs.write_file("/dir0/f", b"hello", write_type="MUST_CACHE")
        st = _meta(fs).Backup(pb.meta.BackupPRequest(targetDirectory=str(tmp_path / "bk")))
        assert st.backupState == COMPLETED and st.entryCount > 0
        assert os.path.basename(st.backupUri).startswith("alluxio-backup-")
        # async: Initiating first, then Completed through GetBackupStatus
        st2 = _meta(fs).Backup(pb.meta.BackupPRequest(targetDirectory=str(tmp_path / "bk"),
                                                      options=pb.meta.BackupPOptions(runAsync=True)))
        assert st2.backupState == INITIATING
        deadline = time.time() + 20
        while time.time() < deadline:
            s = _meta(fs).GetBackupStatus(pb.meta.BackupStatusPRequest(backupId=st2.backupId))
            if s.backupState == COMPLETED:
                break
            time.sleep(0.02)
        assert s.backupState == COMPLETED and s.backupUri
        fs.close()
    m = _restore(tmp_path, st.backupUri)
    try:
        for i in range(5):
            assert m.fs_master.exists(f"/dir{i}/sub")
        assert m.fs_master.get_status("/dir0/f").length == 5
    finally:
        m.stop()


def _ha_conf(extra=None):
    c = {"alluxio.master.backup.delegation.enabled": "true",
         "alluxio.master.standby.heartbeat.interval": "50ms",
         "alluxio.master.backup.heartbeat.interval": "50ms"}
    c.update(extra or {})
    return c


def _wait_standby_registered(cluster, timeout=20.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        p = cluster.primary()
        if p is not None and p.backup_leader.standby_addresses():
            return p
        time.sleep(0.02)
    raise TimeoutError("standby never registered with the primary")


@pytest.mark.parametrize("journal", ["UFS", "EMBEDDED"])
def test_delegated_backup_on_standby(tmp_path, journal):
    n = 2 if journal == "UFS" else 3
    cluster = MultiMasterLocalAlluxioCluster(num_masters=n, num_workers=0, conf=_ha_conf(), grpc=False,
                                             journal_type=journal, work_dir=str(tmp_path / "c"))
    cluster.start()
    try:
        cluster.conf.set("alluxio.master.rpc.addresses", cluster.master_addresses)
        for c in cluster.master_confs:
            c.set("alluxio.master.rpc.addresses", cluster.master_addresses)
        primary = _wait_standby_registered(cluster)
        fs = cluster.client()
        for i in range(20):
            fs.create_directory(f"/ha/d{i}", recursive=True)
        st = fs.ctx.meta_master().Backup(pb.meta.BackupPRequest(targetDirectory=str(tmp_path / "bk")))
        assert st.backupState == COMPLETED, st
        standbys = [m for m in cluster.masters if m is not primary]
        ran_on = [m for m in standbys if st.backupId in m.backup_worker._statuses]
        assert len(ran_on) == 1, "backup was not delegated to a standby"
        # the standby resumed applying the journal: a later write reaches it
        fs.create_directory("/ha/after")
        deadline = time.time() + 20
        while time.time() < deadline and not ran_on[0].fs_master.tree.exists("/ha/after"):
            time.sleep(0.05)
        assert ran_on[0].fs_master.tree.exists("/ha/after")
        assert not ran_on[0].backup_worker._suspended
        fs.close()
    finally:
        cluster.stop()
    m = _restore(tmp_path, st.backupUri)
    try:
        # tree lookups only: the restored root mount points at the old cluster's UFS, where
        # later directories exist and would be loaded on demand
        assert all(m.fs_master.tree.exists(f"/ha/d{i}") for i in range(20))
        assert not m.fs_master.tree.exists("/ha/after")
    finally:
        m.stop()


def test_delegation_without_standby(tmp_path):
    cluster = MultiMasterLocalAlluxioCluster(num_masters=1, num_workers=0, conf=_ha_conf(), grpc=False,
                                             work_dir=str(tmp_path / "c"))
    cluster.start()
    try:
        fs = cluster.client()
        with pytest.raises(FailedPreconditionException):
            fs.ctx.meta_master().Backup(pb.meta.BackupPRequest(targetDirectory=str(tmp_path / "bk")))
        st = fs.ctx.meta_master().Backup(pb.meta.BackupPRequest(
            targetDirectory=str(tmp_path / "bk"), options=pb.meta.BackupPOptions(allowLeader=True)))
        assert st.backupState == COMPLETED
        fs.close()
    finally:
        cluster.stop()


def test_suspend_without_request_resumes(tmp_path):
    """A standby whose journal was suspended resumes by itself after the transport timeout."""
    cluster = MultiMasterLocalAlluxioCluster(num_masters=2, num_workers=0, grpc=False, work_dir=str(tmp_path / "c"),
                                             conf=_ha_conf({"alluxio.master.backup.transport.timeout": "200ms"}))
    cluster.start()
    try:
        primary = cluster.primary()
        standby = next(m for m in cluster.masters if m is not primary)
        standby.backup_worker.SuspendJournals(pb.meta.BackupSuspendPRequest(), None)
        assert standby.journal._suspended
        deadline = time.time() + 10
        while time.time() < deadline and standby.journal._suspended:
            time.sleep(0.02)
        assert not standby.journal._suspended
    finally:
        cluster.stop()


def test_daily_backup_schedule_and_retention(tmp_path):
    c = Configuration(load_site=False)
    c.set("alluxio.master.daily.backup.time", "05:30")
    c.set("alluxio.master.daily.backup.files.retained", "2")
    c.set("alluxio.master.backup.directory", str(tmp_path))

    class Leader:
        calls = 0

        def backup(self, req):
            Leader.calls += 1
            name = f"alluxio-backup-2026-01-0{Leader.calls}-000000000000-aaaaaa.gz"
            open(os.path.join(req.targetDirectory, name), "wb").close()
            return pb.meta.BackupPStatus(backupState=COMPLETED, backupUri=name)
    d = DailyMetadataBackup(Leader(), c)
    now = datetime.datetime(2026, 1, 1, 5, 0, tzinfo=datetime.timezone.utc)
    assert d.seconds_until_next(now) == 30 * 60
    now = datetime.datetime(2026, 1, 1, 6, 0, tzinfo=datetime.timezone.utc)
    assert d.seconds_until_next(now) == 23.5 * 3600
    for _ in range(4):
        d.run_once()
    left = sorted(os.listdir(tmp_path))
    assert left == ["alluxio-backup-2026-01-03-000000000000-aaaaaa.gz", "alluxio-backup-2026-01-04-000000000000-aaaaaa.gz"]
