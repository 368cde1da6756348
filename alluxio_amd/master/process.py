"""Master process: journal system + masters + RPC server + background heartbeats.

Parity: core/server/master/src/main/java/alluxio/master/AlluxioMasterProcess.java (ctor :97-127,
start :156-161 — journal start, gainPrimacy, startMasters :197-221, startServingRPCServer
:300-340), Factory.create :387-401 (journal type selection), FaultTolerantAlluxioMasterProcess
(standby tails the journal until it gains primacy), SafeModeManager, StateLockManager (blocks
mutations while a backup/checkpoint snapshot is taken), and the heartbeat executors started by
DefaultFileSystemMaster.start / DefaultBlockMaster.start.
"""
from __future__ import annotations

import logging
import os
import sys
import threading
import time

from ..conf import Configuration
from ..journal.system import NoopJournalSystem, UfsJournalSystem
from ..rpc import RpcServer
from ..utils import heartbeat as hb
from .block_master import BlockMaster
from .file_system_master import FileSystemMaster
from .meta_master import MetaMaster, MetaServices, MetricsMaster, restore_backup
from .services import (SVC_BLOCK_CLIENT, SVC_BLOCK_WORKER, SVC_FS_CLIENT, SVC_FS_JOB, SVC_FS_WORKER,
                       SVC_JOURNAL, SVC_META_CLIENT, SVC_META_CONFIG, SVC_META_MASTER, SVC_METRICS,
                       SVC_SASL, SVC_VERSION, BlockMasterClientServiceHandler,
                       BlockMasterWorkerServiceHandler, FileSystemMasterClientServiceHandler,
                       FileSystemMasterWorkerServiceHandler, SaslHandler, ServiceVersionHandler)

LOG = logging.getLogger(__name__)


class StateLockManager:
    """Shared lock held by every mutating RPC; exclusive during backups (StateLockManager.java)."""

    def __init__(self):
        from ..utils.locks import RWLock
        self._lock = RWLock()

    def acquire_shared(self):
        self._lock.acquire_read()

    def release_shared(self):
        self._lock.release_read()

    def exclusive(self):
        return self._lock.write()


class SafeModeManager:
    def __init__(self, wait_ms: int):
        self.wait_ms = wait_ms
        self._until = 0.0

    def notify_primary(self):
        self._until = time.time() + self.wait_ms / 1000.0

    def in_safe_mode(self) -> bool:
        return time.time() < self._until


def build_journal_system(conf: Configuration, host: str | None = None, enable_grpc: bool = True,
                         ephemeral: bool = False):
    """UFS / EMBEDDED (Raft among the masters) / NOOP (JournalSystem factory)."""
    jtype = conf.get("alluxio.master.journal.type", "UFS").upper()
    if jtype in ("NOOP", "NONE"):
        return NoopJournalSystem()
    folder = conf.get("alluxio.master.journal.folder")
    if folder.startswith("file://"):
        folder = folder[len("file://"):]
    if jtype == "EMBEDDED":
        from ..journal.raft_system import RaftJournalSystem
        return RaftJournalSystem.from_conf(conf, folder, host=host, enable_grpc=enable_grpc,
                                           ephemeral_port=ephemeral)
    return UfsJournalSystem(folder, max_log_bytes=conf.get_bytes("alluxio.master.journal.log.size.bytes.max"),
                            flush_batch_ms=conf.get_ms("alluxio.master.journal.flush.batch.time"),
                            checkpoint_period_entries=conf.get_int("alluxio.master.journal.checkpoint.period.entries"),
                            native_writer=conf.get_bool("alluxio.master.journal.native.writer.enabled"))


class AlluxioMasterProcess:
    def __init__(self, conf: Configuration | None = None, host: str = "127.0.0.1", port: int | None = None,
                 enable_grpc: bool = True, root_ufs: str | None = None, journal_system=None):
        self.conf = conf or Configuration(load_site=True)
        self.host = host
        self.port = self.conf.get_int("alluxio.master.rpc.port") if port is None else port
        from .. import metrics as msys
        self.metrics = msys.metrics("Master")
        self.journal = journal_system or build_journal_system(self.conf, host=host, enable_grpc=enable_grpc,
                                                              ephemeral=self.port == 0)
        self.block_master = BlockMaster(self.conf, self.journal,
                                        worker_timeout_ms=self.conf.get_ms("alluxio.master.worker.timeout"))
        # alluxio.master.mount.table.root.option.<key> = root mount properties (PropertyKey
        # MASTER_MOUNT_TABLE_ROOT_OPTION_PROPERTY)
        pfx = "alluxio.master.mount.table.root.option."
        root_opts = {k[len(pfx):]: v for k, v in self.conf.to_map().items() if k.startswith(pfx)}
        self.fs_master = FileSystemMaster(self.conf, self.block_master, self.journal, metrics=self.metrics,
                                          root_ufs=root_ufs, root_ufs_properties=root_opts)
        self.meta_master = MetaMaster(self.conf, self.journal)
        self.meta_master.block_master = self.block_master
        self.metrics_master = MetricsMaster()
        from .time_series import TimeSeriesRecorder
        self.time_series = TimeSeriesRecorder(self.block_master, self.metrics_master, self._root_ufs_space)
        self.block_master.metrics = lambda w, ms: self.metrics_master.worker_heartbeat(w.id, ms)
        self.state_lock = StateLockManager()
        self.fs_master.state_lock = self.state_lock
        self.safe_mode = SafeModeManager(self.conf.get_ms("alluxio.master.worker.connect.wait.time"))
        self._register_gauges()
        self.table_master = None
        if self.conf.get_bool("alluxio.table.enabled", "true"):
            from ..table.master import TableMaster
            self.table_master = TableMaster(self.conf, self.journal, fs_factory=lambda: self._job_fs())
        for j in (self.block_master, self.fs_master, self.meta_master, self.table_master):
            if j is not None:
                self.journal.register(j)
        self.meta_master.masters_for_backup = [m for m in (self.block_master, self.fs_master, self.meta_master,
                                                            self.table_master) if m is not None]
        self.meta_master.journal_system_for_checkpoint = self   # checkpoint() under the state lock
        from .backup import BackupLeaderRole, BackupWorkerRole, DailyMetadataBackup, MetaMasterSync
        self.backup_leader = BackupLeaderRole(self)
        self.backup_worker = BackupWorkerRole(self)
        self.meta_master.backup_role = self.backup_leader
        self.daily_backup = (DailyMetadataBackup(self.backup_leader, self.conf)
                             if self.conf.get_bool("alluxio.master.daily.backup.enabled", "false") else None)
        self.meta_sync = MetaMasterSync(self, self._primary_candidates)
        self._peer_channels = None
        self.server = RpcServer(host, self.port, max_workers=self.conf.get_int("alluxio.master.rpc.executor.max.pool.size", 500)
                                if False else 64, metrics=self.metrics, enable_grpc=enable_grpc,
                                conf=self.conf)
        self._threads: list[hb.HeartbeatThread] = []
        self.job_master = None
        if self.conf.get_bool("alluxio.job.master.embedded.enabled", "true"):
            from ..job.master import JobMaster
            self.job_master = JobMaster(self._job_fs, self.conf.get_ms("alluxio.job.master.worker.timeout") / 1000.0,
                                        self.conf.get_int("alluxio.job.master.job.capacity"))
        self._job_client_fs = None
        self.replication_checker = None
        if self.table_master is not None:
            self.table_master.job_master = self.job_master
        if self.job_master is not None:
            from .replication import ReplicationChecker
            self.replication_checker = ReplicationChecker(self.fs_master, self.job_master, safe_mode=self.safe_mode)
        self.web = None
        self.selector = None
        self._standby_hb = None
        self.web_port = 0
        self.start_time = time.time()
        self.started = False
        self.primary = False

    @property
    def address(self) -> str:
        return self.server.address

    def _register_gauges(self) -> None:
        """Master/Cluster gauges (DefaultFileSystemMaster.java:4321 registerGauges,
        DefaultBlockMaster.java:1209 registerGauges)."""
        reg, bm, tree = self.metrics.registry, self.block_master, self.fs_master.tree
        reg.gauge("Master.FilesPinned", lambda: len(tree.pinned_ids))
        reg.gauge("Master.TotalPaths", lambda: len(tree.inodes))
        reg.gauge("Cluster.CapacityTotal", bm.capacity_bytes)
        reg.gauge("Cluster.CapacityUsed", bm.used_bytes)
        reg.gauge("Cluster.CapacityFree", lambda: bm.capacity_bytes() - bm.used_bytes())
        reg.gauge("Cluster.Workers", bm.worker_count)

    def _root_ufs_space(self):
        """(total, used) bytes of the root mount's UFS (Cluster.RootUfsCapacity*)."""
        from ..underfs.base import SpaceType
        res = self.fs_master._resolve_ufs("/")
        return (res.ufs.get_space(res.uri, SpaceType.SPACE_TOTAL), res.ufs.get_space(res.uri, SpaceType.SPACE_USED))

    def _primary_candidates(self) -> list[str]:
        return [a.strip() for a in (self.conf.get_raw("alluxio.master.rpc.addresses") or "").split(",") if a.strip()]

    def peer_stub(self, address: str, service: str):
        """Stub of another master's service over the pooled channels (delegated backups)."""
        from ..rpc import ChannelPool
        if self._peer_channels is None:
            self._peer_channels = ChannelPool(self.conf)
        return self._peer_channels.get(address).stub(service)

    def _job_fs(self):
        from ..client.file_system import FileSystem
        if self._job_client_fs is None:
            self._job_client_fs = FileSystem(conf=self.conf, master_address=self.address)
        return self._job_client_fs

    def _persist_via_job(self, file_id: int, path: str) -> int:
        from ..job import PersistConfig
        return self.job_master.run(PersistConfig(path=path))

    def persistence_checker(self) -> int:
        """PersistenceChecker: poll persist jobs; mark files persisted or reschedule failures."""
        if self.job_master is None:
            return 0
        done = 0
        for fid, info in list(self.fs_master.persist_jobs.items()):
            jid = info.get("job", -1)
            if jid is None or jid < 0:
                continue
            try:
                st = self.job_master.status(jid).status
            except Exception:  # noqa: BLE001 - job purged or unknown: retry the persist
                st = "FAILED"
            if st == "COMPLETED":
                self.fs_master.persist_done(fid, True)
                done += 1
            elif st in ("FAILED", "CANCELED"):
                self.fs_master.persist_done(fid, False)
        return done

    def _register_services(self) -> None:
        s = self.server
        s.add_servicer(SVC_FS_CLIENT, FileSystemMasterClientServiceHandler(self.fs_master))
        fsw = FileSystemMasterWorkerServiceHandler(self.fs_master)
        s.add_servicer(SVC_FS_WORKER, fsw)
        s.add_servicer(SVC_FS_JOB, fsw)
        s.add_servicer(SVC_BLOCK_CLIENT, BlockMasterClientServiceHandler(self.block_master))
        s.add_servicer(SVC_BLOCK_WORKER, BlockMasterWorkerServiceHandler(self.block_master, self.metrics_master))
        meta = MetaServices(self.meta_master, self.metrics_master, self.journal)
        for svc in (SVC_META_CLIENT, SVC_META_CONFIG, SVC_META_MASTER, SVC_METRICS, SVC_JOURNAL):
            s.add_servicer(svc, meta)
        if self.job_master is not None:
            from ..job import SVC_JOB_CLIENT, SVC_JOB_WORKER
            from ..job.master import JobMasterService
            jsvc = JobMasterService(self.job_master)
            s.add_servicer(SVC_JOB_CLIENT, jsvc)
            s.add_servicer(SVC_JOB_WORKER, jsvc)
        if self.table_master is not None:
            from ..table.master import SVC_TABLE, TableMasterService
            s.add_servicer(SVC_TABLE, TableMasterService(self.table_master))
        from .backup import SVC_BACKUP_WORKER
        s.add_servicer(SVC_BACKUP_WORKER, self.backup_worker)
        self._version_handler = ServiceVersionHandler()
        s.add_servicer(SVC_VERSION, self._version_handler)
        s.add_servicer(SVC_SASL, SaslHandler())

    def format(self) -> None:
        self.journal.format()

    def start(self, primary: bool = True, start_heartbeats: bool = True) -> str:
        """Single master: become primary now.  HA (``alluxio.master.ha.primary.selector`` =
        FILE_LOCK): start as a standby tailing the journal behind an RPC gate that answers
        UNAVAILABLE, and gain primacy when elected (FaultTolerantAlluxioMasterProcess)."""
        from .. import metrics as msys
        from ..journal.raft_system import RaftJournalSystem
        from ..utils.pause_monitor import from_conf as pause_monitor
        self._sinks = msys.load_sinks(self.conf, self.metrics)
        self.pause_monitor = pause_monitor(self.conf, "master", self.metrics)
        if self.pause_monitor is not None:
            self.pause_monitor.start()
        raft = isinstance(self.journal, RaftJournalSystem)
        if not self.journal.is_formatted() and isinstance(self.journal, (UfsJournalSystem, RaftJournalSystem)):
            self.journal.format()
        self.journal.start()
        ha = raft or self.conf.get("alluxio.master.ha.primary.selector", "NONE").upper() == "FILE_LOCK"
        if primary and not ha:
            self.gain_primacy()
        if self.job_master is not None and self.fs_master.persist_handler is None:
            self.fs_master.persist_handler = self._persist_via_job
        self._register_services()
        if ha:
            from ..utils.exceptions import UnavailableException

            from .backup import SVC_BACKUP_WORKER

            def standby_gate(spec):
                if not self.primary and spec.service != SVC_BACKUP_WORKER:
                    raise UnavailableException("master is a standby (not primary)")
            self.server.gate = standby_gate
        self.native_rpc = None
        # alluxio.master.rpc.native.grpc.enabled: the master RPC port itself is the native front
        # end, which serves gRPC (HTTP/2) connections too -- stock gRPC clients (Java) then get the
        # C++ I/O threads, lanes and reply cache instead of the grpcio server
        native_grpc = self.server.enable_grpc and \
            self.conf.get_bool("alluxio.master.rpc.native.grpc.enabled", "true") and \
            self.conf.get_bool("alluxio.master.native.rpc.enabled", "true")
        if native_grpc:
            from ..ops.native import lib
            native_grpc = lib().FrameRpcServer.grpc_available()
        if self.server.enable_grpc and self.conf.get_bool("alluxio.master.native.rpc.enabled", "true"):
            # metadata fast path next to gRPC (same servicers): see alluxio_amd/rpc/native.py.
            # Started first, so the port is advertised from the first gRPC call on.
            from ..rpc.native import NativeRpcFrontend
            if native_grpc:
                self.server.enable_grpc = False
            self.native_rpc = NativeRpcFrontend(
                self.server, self.server.host,
                self.server.port if native_grpc else self.conf.get_int("alluxio.master.native.rpc.port", "0"),
                fast_threads=self.conf.get_int("alluxio.master.native.rpc.fast.threads", "2"),
                blocking_threads=self.conf.get_int("alluxio.master.native.rpc.blocking.threads", "16"),
                mutation_threads=self.conf.get_int("alluxio.master.native.rpc.mutation.threads", "2"),
                mutation_batch=self.conf.get_int("alluxio.master.native.rpc.mutation.batch", "16"),
                reply_cache=self.conf.get_bool("alluxio.master.native.rpc.reply.cache.enabled", "true")
                and self.fs_master.audit is None,
                epoch_source=self.fs_master.add_epoch_listener)
            self._version_handler.native_port = self.native_rpc.start()
            if native_grpc:
                self.server.port = self.native_rpc.port
        addr = self.server.start()
        self.meta_master.master_address = addr
        self.start_time = time.time()
        if self.conf.get_bool("alluxio.web.server.enabled", "true"):
            from ..web import WebServer, master_routes
            self.web = WebServer(self.conf.get("alluxio.master.web.bind.host", "0.0.0.0"),
                                 self.conf.get_int("alluxio.master.web.port"), master_routes(self), "master")
            self.web_port = self.web.start()
            self.meta_master.web_port = self.web_port
        if ha:
            if raft:       # primacy follows Raft leadership (RaftPrimarySelector)
                self.selector = self.journal.selector
            else:
                from .ha import FileLockPrimarySelector
                self.selector = FileLockPrimarySelector(self.conf.get("alluxio.master.ha.lock.file"))

            def on_primary():
                self.gain_primacy()
                if start_heartbeats:
                    self._start_heartbeats()
            self.selector.start(on_primary, self.lose_primacy)
            # standbys register with and heartbeat the primary (MetaMasterSync)
            self._standby_hb = hb.HeartbeatThread(
                hb.META_MASTER_SYNC,
                self.meta_sync.heartbeat, self.conf.get_ms("alluxio.master.standby.heartbeat.interval", "2min"))
            self._standby_hb.start()
        elif start_heartbeats and primary:
            self._start_heartbeats()
        self.started = True
        LOG.info("master serving at %s", addr)
        return addr

    def gain_primacy(self) -> None:
        backup = self.conf.get_raw("alluxio.master.journal.init.from.backup")
        if backup and self.journal.is_empty():
            # become the writer first (that replays the empty journal), then load the backup and
            # checkpoint it so it is durable (BackupManager.initFromBackup journals every entry)
            self.journal.gain_primacy()
            n = restore_backup(backup, self.meta_master.masters_for_backup)
            LOG.info("restored %d entries from backup %s", n, backup)
            self.journal.checkpoint()
        else:
            self.journal.gain_primacy()
        self.fs_master.start(True)
        self.meta_master.start(True)
        self.safe_mode.notify_primary()
        self.primary = True
        if self.daily_backup is not None:
            self.daily_backup.start()

    def lose_primacy(self) -> None:
        """Step down to standby: refuse RPCs, stop primary-only heartbeats, and let the journal
        rebuild the masters' state from what was committed (FaultTolerantAlluxioMasterProcess)."""
        if not self.primary:
            return
        LOG.info("master %s lost primacy", getattr(self.server, "address", "?"))
        self.primary = False
        if getattr(self, "native_rpc", None) is not None:
            self.native_rpc.server.bump_epoch()   # cached replies were a primary's answers
        if self.daily_backup is not None:
            self.daily_backup.stop()
        threads, self._threads = self._threads, []
        for t in threads:
            t.shutdown(join=False)
        try:
            self.fs_master.access_time.stop()     # batched access times are journaled first
        except Exception:  # noqa: BLE001
            LOG.debug("access time flush at step-down failed", exc_info=True)
        with self.state_lock.exclusive():
            self.journal.lose_primacy()

    def _start_heartbeats(self) -> None:
        c = self.conf
        specs = [
            (hb.MASTER_LOST_WORKER_DETECTION, self.block_master.detect_lost_workers,
             c.get_ms("alluxio.master.lost.worker.detection.interval", "10sec")),
            (hb.MASTER_TTL_CHECK, self.fs_master.ttl_check, c.get_ms("alluxio.master.ttl.checker.interval")),
            (hb.MASTER_LOST_FILES_DETECTION, self.fs_master.lost_files_check,
             c.get_ms("alluxio.master.lost.worker.file.detection.interval", "5min")),
            (hb.MASTER_PERSISTENCE_SCHEDULER, self.fs_master.persistence_scheduler_heartbeat,
             c.get_ms("alluxio.master.persistence.scheduler.interval", "1sec")),
            (hb.MASTER_ACTIVE_UFS_SYNC, self.fs_master.active_sync_heartbeat,
             c.get_ms("alluxio.master.ufs.active.sync.interval", "30sec")),
            (hb.MASTER_LOST_MASTER_DETECTION, self.meta_master.detect_lost_masters,
             c.get_ms("alluxio.master.standby.heartbeat.interval", "2min")),
            (hb.MASTER_METRICS_TIME_SERIES, self.time_series.heartbeat,
             c.get_ms("alluxio.master.metrics.time.series.interval")),
        ]
        if self.job_master is not None:
            specs.append((hb.MASTER_PERSISTENCE_CHECKER, self.persistence_checker,
                          c.get_ms("alluxio.master.persistence.checker.interval", "1sec")))
            specs.append((hb.JOB_MASTER_LOST_WORKER_DETECTION, self.job_master.detect_lost_workers,
                          c.get_ms("alluxio.job.master.lost.worker.interval")))
            if self.table_master is not None:
                specs.append(("Master Table Transformation Monitor", self.table_master.transform_heartbeat,
                              c.get_ms("alluxio.table.transform.manager.job.monitor.interval", "10sec")))
            specs.append((hb.MASTER_REPLICATION_CHECK, self.replication_checker.heartbeat,
                          c.get_ms("alluxio.master.replication.check.interval", "1min")))
            retention = c.get_ms("alluxio.job.master.finished.job.retention.time") / 1000.0
            specs.append(("Job Master Finished Job Purge",
                          lambda: self.job_master.purge_finished(retention), 10_000))
        if c.get_bool("alluxio.underfs.cleanup.enabled"):
            specs.append((hb.MASTER_UFS_CLEANUP, self.fs_master.cleanup_ufs, c.get_ms("alluxio.underfs.cleanup.interval")))
        if c.get_ms("alluxio.master.periodic.block.integrity.check.interval", "1hr") > 0:
            specs.append((hb.MASTER_BLOCK_INTEGRITY_CHECK, self.fs_master.block_integrity_check,
                          c.get_ms("alluxio.master.periodic.block.integrity.check.interval", "1hr")))
        for name, fn, interval in specs:
            t = hb.HeartbeatThread(name, fn, interval)
            t.start()
            self._threads.append(t)

    def add_heartbeat(self, name: str, fn, interval_ms: int) -> None:
        t = hb.HeartbeatThread(name, fn, interval_ms)
        t.start()
        self._threads.append(t)

    def checkpoint(self) -> None:
        with self.state_lock.exclusive():
            self.journal.checkpoint()

    def stop(self) -> None:
        for sk in getattr(self, "_sinks", []):
            sk.stop()
        if getattr(self, "pause_monitor", None) is not None:
            self.pause_monitor.stop()
        # no new elections from here on, but keep the primary lock until the journal writers are
        # closed: releasing it first lets a standby start writing the same logs while this
        # master still completes its current log file
        if self.selector is not None and hasattr(self.selector, "halt"):
            self.selector.halt()
        if getattr(self, "_standby_hb", None) is not None:
            self._standby_hb.shutdown(join=True)
            self._standby_hb = None
        if self.daily_backup is not None:
            self.daily_backup.stop()
        if self._peer_channels is not None:
            self._peer_channels.close()
            self._peer_channels = None
        self.primary = False
        for t in self._threads:
            t.shutdown(join=False)
        for t in self._threads:
            t.shutdown(join=True)
        self._threads.clear()
        if self.web is not None:
            self.web.stop()
            self.web = None
        if getattr(self, "native_rpc", None) is not None:
            self.native_rpc.stop()
            self.native_rpc = None
        self.server.stop()
        if self._job_client_fs is not None:
            self._job_client_fs.close()
            self._job_client_fs = None
        try:
            self.fs_master.access_time.stop()     # AccessTimeUpdater.beforeShutdown
        except Exception:  # noqa: BLE001
            LOG.debug("access time flush at shutdown failed", exc_info=True)
        self.journal.stop()
        if self.selector is not None:
            self.selector.stop()
        self.started = False


def main(argv=None) -> int:  # pragma: no cover - CLI entry
    import argparse
    ap = argparse.ArgumentParser(description="alluxio_amd master")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--root-ufs", default=None)
    ap.add_argument("--format", action="store_true")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from ..utils.sampler import maybe_start_from_env
    maybe_start_from_env()
    from ..conf import Configuration as _C
    from ..web.logserver import attach
    attach("MASTER", _C(load_site=True))
    import os as _os
    if _os.environ.get("ALLUXIO_SWITCH_INTERVAL_US"):
        sys.setswitchinterval(float(_os.environ["ALLUXIO_SWITCH_INTERVAL_US"]) / 1e6)
    from ..utils import optiming
    if optiming.ENABLED:                 # the bench stops the master with SIGTERM: dump first
        import signal
        signal.signal(signal.SIGTERM, lambda *_: (optiming.dump(), os._exit(0)))
    m = AlluxioMasterProcess(host=a.host, port=a.port, root_ufs=a.root_ufs)
    if a.format:
        m.format()
    m.start()
    # The namespace is millions of long-lived tracked objects: with the default gen0 threshold (700)
    # the cyclic collector runs every few RPCs and its older-generation passes walk the whole tree.
    # Freeze what startup/replay built and collect young objects less often (cycles are rare here;
    # refcounting frees the per-RPC garbage).
    gen0 = int(_os.environ.get("ALLUXIO_MASTER_GC_GEN0", "50000"))
    if gen0 > 0:
        import gc
        gc.freeze()
        gc.set_threshold(gen0, 20, 100)
    stop = threading.Event()
    try:
        stop.wait()
    except KeyboardInterrupt:
        pass
    m.stop()
    return 0


if __name__ == "__main__":  # pragma: no cover
    raise SystemExit(main())
