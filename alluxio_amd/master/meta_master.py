"""Meta master (cluster config, path config, master registry, backups, checkpoints) and metrics
master (cluster metric aggregation).

Parity: core/server/master/src/main/java/alluxio/master/meta/DefaultMetaMaster.java (:641 —
config service, server configuration checker, master (standby) registry with heartbeats, backup
& checkpoint RPCs), PathProperties.java (journaled path-level config), DailyMetadataBackup.java,
checkconf/ServerConfigurationChecker.java (inconsistent-property report);
metrics/DefaultMetricsMaster.java + MetricsStore.java (worker/client metrics aggregated into
``Cluster.*`` values).
"""
from __future__ import annotations

import gzip
import logging
import os
import threading
import time
import uuid

from ..conf import PathConfiguration
from ..journal import format as jfmt
from ..journal.system import Journaled, NoopJournalContext
from ..proto import pb
from ..utils import ids

LOG = logging.getLogger(__name__)

VERSION = "2.5.0-amd"


class MetaMaster(Journaled):
    journal_name = "MetaMaster"

    def __init__(self, conf, journal_system=None, master_address: str = "", web_port: int = 0):
        self.conf = conf
        self.journal = journal_system
        self.path_conf = PathConfiguration()
        self.cluster_id = ""
        self.start_ms = int(time.time() * 1000)
        self.master_address = master_address
        self.web_port = web_port
        self.safe_mode = False
        self._standbys: dict[int, dict] = {}
        self._worker_configs: dict[str, dict] = {}
        self.backup_role = None          # master.backup.BackupLeaderRole
        self._lock = threading.RLock()
        self.masters_for_backup: list[Journaled] = []
        self.journal_system_for_checkpoint = None
        self.block_master = None

    # ---- Journaled ----------------------------------------------------------------------------
    def reset_state(self) -> None:
        self.path_conf = PathConfiguration()
        self.cluster_id = ""

    def process_journal_entry(self, e) -> bool:
        if e.HasField("path_properties"):
            self.path_conf.set(e.path_properties.path, dict(e.path_properties.properties))
        elif e.HasField("remove_path_properties"):
            self.path_conf.remove(e.remove_path_properties.path)
        elif e.HasField("cluster_info"):
            self.cluster_id = e.cluster_info.cluster_id
        else:
            return False
        return True

    def journal_entries(self):
        if self.cluster_id:
            yield pb.journal.JournalEntry(cluster_info=pb.journal.ClusterInfoEntry(cluster_id=self.cluster_id))
        for p, props in self.path_conf.get_all().items():
            e = pb.journal.PathPropertiesEntry(path=p)
            for k, v in props.items():
                e.properties[k] = v
            yield pb.journal.JournalEntry(path_properties=e)

    def _ctx(self):
        return NoopJournalContext() if self.journal is None else self.journal.create_context(self.journal_name)

    def start(self, primary: bool = True) -> None:
        if primary and not self.cluster_id:
            e = pb.journal.JournalEntry(cluster_info=pb.journal.ClusterInfoEntry(cluster_id=str(uuid.uuid4())))
            self.process_journal_entry(e)
            ctx = self._ctx()
            ctx.append(e)
            ctx.close()

    # ---- configuration ------------------------------------------------------------------------
    def get_configuration(self, raw: bool = False):
        props = [pb.grpc.ConfigProperty(name=k, value=v, source="CLUSTER_DEFAULT")
                 for k, v in sorted(self.conf.to_map().items())]
        r = pb.meta.GetConfigurationPResponse(clusterConfigs=props, clusterConfigHash=self.conf.hash(),
                                              pathConfigHash=self.path_conf.hash())
        for p, d in self.path_conf.get_all().items():
            r.pathConfigs[p].properties.extend(pb.grpc.ConfigProperty(name=k, value=v, source="PATH_DEFAULT")
                                               for k, v in sorted(d.items()))
        return r

    def set_path_configuration(self, path: str, props: dict) -> None:
        e = pb.journal.PathPropertiesEntry(path=path)
        merged = dict(self.path_conf.get_all().get(path, {}))
        merged.update(props)
        for k, v in merged.items():
            e.properties[k] = v
        je = pb.journal.JournalEntry(path_properties=e)
        self.process_journal_entry(je)
        ctx = self._ctx()
        ctx.append(je)
        ctx.close()

    def remove_path_configuration(self, path: str, keys=None) -> None:
        cur = dict(self.path_conf.get_all().get(path, {}))
        if keys:
            for k in keys:
                cur.pop(k, None)
        ctx = self._ctx()
        if not keys or not cur:
            je = pb.journal.JournalEntry(remove_path_properties=pb.journal.RemovePathPropertiesEntry(path=path))
        else:
            e = pb.journal.PathPropertiesEntry(path=path)
            for k, v in cur.items():
                e.properties[k] = v
            self.path_conf.remove(path)
            je = pb.journal.JournalEntry(path_properties=e)
        self.process_journal_entry(je)
        ctx.append(je)
        ctx.close()

    def record_worker_config(self, worker: str, configs: dict) -> None:
        with self._lock:
            self._worker_configs[worker] = dict(configs)

    def config_report(self):
        """Properties that differ between master and registered workers (ServerConfigurationChecker)."""
        mine = self.conf.to_map()
        errors: dict[str, dict[str, set]] = {}
        with self._lock:
            for worker, cfg in self._worker_configs.items():
                for k, v in cfg.items():
                    if k.startswith("alluxio.worker.") or k.startswith("alluxio.user."):
                        continue
                    mv = mine.get(k)
                    if mv is not None and mv != v:
                        errors.setdefault(k, {}).setdefault(v, set()).add(worker)
                        errors[k].setdefault(mv, set()).add("master")
        rep = pb.meta.ConfigCheckReport(status=3 if errors else 1)
        if errors:
            inc = rep.errors["SERVER"]
            for k, vals in errors.items():
                p = inc.properties.add(name=k)
                for v, hosts in vals.items():
                    p.values[v].values.extend(sorted(hosts))
        return rep

    # ---- masters ------------------------------------------------------------------------------
    def get_master_id(self, address) -> int:
        with self._lock:
            for mid, info in self._standbys.items():
                if info["address"].host == address.host and info["address"].rpcPort == address.rpcPort:
                    return mid
            mid = ids.get_random_non_negative_long()
            self._standbys[mid] = {"address": address, "last": time.time()}
            return mid

    def master_heartbeat(self, master_id: int) -> str:
        with self._lock:
            info = self._standbys.get(master_id)
            if info is None:
                return "MetaCommand_Register"
            info["last"] = time.time()
            return "MetaCommand_Nothing"

    def register_master(self, master_id: int, configs: dict) -> None:
        with self._lock:
            if master_id in self._standbys:
                self._standbys[master_id]["configs"] = configs

    def detect_lost_masters(self, timeout_s: float = 300.0) -> list[int]:
        now = time.time()
        with self._lock:
            lost = [m for m, i in self._standbys.items() if now - i["last"] > timeout_s]
            for m in lost:
                self._standbys.pop(m)
        return lost

    def master_info(self):
        host, _, port = self.master_address.partition(":")
        info = pb.meta.MasterInfo(leaderMasterAddress=self.master_address, rpcPort=int(port or 0),
                                  safeMode=self.safe_mode, startTimeMs=self.start_ms,
                                  upTimeMs=int(time.time() * 1000) - self.start_ms, version=VERSION,
                                  webPort=self.web_port)
        info.masterAddresses.append(pb.grpc.NetAddress(host=host, rpcPort=int(port or 0)))
        with self._lock:
            for s in self._standbys.values():
                info.masterAddresses.append(pb.grpc.NetAddress(host=s["address"].host, rpcPort=s["address"].rpcPort))
        if self.block_master is not None:
            for w in self.block_master.workers():
                info.workerAddresses.append(pb.grpc.NetAddress(host=w.address.host, rpcPort=w.address.rpcPort))
        return info

    # ---- backup (master/backup.py BackupLeaderRole) ---------------------------------------------
    def backup(self, req: pb.meta.BackupPRequest) -> pb.meta.BackupPStatus:
        if self.backup_role is None:
            raise RuntimeError("backups need a master process (no backup role attached)")
        return self.backup_role.backup(req)

    def backup_status(self, backup_id: str):
        if self.backup_role is None:
            return pb.meta.BackupPStatus(backupId=backup_id, backupState=1)
        return self.backup_role.status(backup_id)

    def standby_rpc_addresses(self) -> list[str]:
        """RPC addresses of the standby masters registered through MetaMasterSync."""
        with self._lock:
            return [f"{i['address'].host}:{i['address'].rpcPort}" for i in self._standbys.values()]

    def checkpoint(self) -> str:
        if self.journal_system_for_checkpoint is not None:
            self.journal_system_for_checkpoint.checkpoint()
        return self.master_address.split(":")[0]


def restore_backup(path: str, journaled: list[Journaled]) -> int:
    """Replay a backup file into freshly reset masters (``alluxio.master.journal.init.from.backup``)."""
    by_kind: dict[str, Journaled] = {}
    with gzip.open(path, "rb") as f:
        entries = jfmt.bytes_to_entries(f.read())
    for j in journaled:
        j.reset_state()
    n = 0
    for e in entries:
        for j in journaled:
            if j.process_journal_entry(e):
                n += 1
                break
    del by_kind
    return n


class MetricsMaster:
    """Aggregates reported worker/client metrics into cluster-level values."""

    CLUSTER_SUMS = {
        "Worker.BytesReadAlluxio": "Cluster.BytesReadAlluxio",
        "Worker.BytesReadDomain": "Cluster.BytesReadDomain",
        "Worker.BytesReadUfsAll": "Cluster.BytesReadUfsAll",
        "Worker.BytesWrittenAlluxio": "Cluster.BytesWrittenAlluxio",
        "Worker.BytesWrittenUfsAll": "Cluster.BytesWrittenUfsAll",
        "Client.BytesReadLocal": "Cluster.BytesReadLocal",
        "Worker.BytesReadDevice": "Cluster.BytesReadDevice",
        "Worker.XgmiBytesSent": "Cluster.XgmiBytesSent",
    }

    def __init__(self):
        self._lock = threading.Lock()
        self._by_source: dict[str, dict[str, float]] = {}
        self._cluster: dict[str, float] = {}

    def _ingest(self, source: str, metrics) -> None:
        with self._lock:
            d = self._by_source.setdefault(source, {})
            for m in metrics:
                name = m.name
                base = name.split(".")[0:2]
                key = ".".join(base)
                if m.metricType == 1:  # COUNTER: deltas
                    d[key] = d.get(key, 0.0) + m.value
                    target = self.CLUSTER_SUMS.get(key)
                    if target:
                        self._cluster[target] = self._cluster.get(target, 0.0) + m.value
                else:
                    d[key] = m.value

    def worker_heartbeat(self, worker_id, metrics) -> None:
        self._ingest(f"worker-{worker_id}", metrics)

    def client_heartbeat(self, client_metrics) -> None:
        for cm in client_metrics:
            self._ingest(cm.source or "client", cm.metrics)

    def clear(self) -> None:
        with self._lock:
            self._by_source.clear()
            self._cluster.clear()

    def get_metrics(self) -> dict[str, float]:
        with self._lock:
            out = dict(self._cluster)
            for src, d in self._by_source.items():
                for k, v in d.items():
                    out[f"{k}.{src}"] = v
            return out


class MetaServices:
    """Meta + metrics + journal-master service handlers."""

    def __init__(self, meta: MetaMaster, metrics_master: MetricsMaster, journal_system=None):
        self.meta = meta
        self.mm = metrics_master
        self.js = journal_system

    # MetaMasterClientService
    def Backup(self, req, ctx):
        return self.meta.backup(req)

    def GetBackupStatus(self, req, ctx):
        return self.meta.backup_status(req.backupId)

    def GetConfigReport(self, req, ctx):
        return pb.meta.GetConfigReportPResponse(report=self.meta.config_report())

    def GetMasterInfo(self, req, ctx):
        return pb.meta.GetMasterInfoPResponse(masterInfo=self.meta.master_info())

    def Checkpoint(self, req, ctx):
        return pb.meta.CheckpointPResponse(masterHostname=self.meta.checkpoint())

    # MetaMasterConfigurationService
    def GetConfiguration(self, req, ctx):
        return self.meta.get_configuration(req.rawValue)

    def SetPathConfiguration(self, req, ctx):
        self.meta.set_path_configuration(req.path, dict(req.properties))
        return pb.meta.SetPathConfigurationPResponse()

    def RemovePathConfiguration(self, req, ctx):
        self.meta.remove_path_configuration(req.path, list(req.keys) or None)
        return pb.meta.RemovePathConfigurationPResponse()

    def GetConfigHash(self, req, ctx):
        return pb.meta.GetConfigHashPResponse(clusterConfigHash=self.meta.conf.hash(),
                                              pathConfigHash=self.meta.path_conf.hash())

    # MetaMasterMasterService
    def GetMasterId(self, req, ctx):
        return pb.meta.GetMasterIdPResponse(masterId=self.meta.get_master_id(req.masterAddress))

    def RegisterMaster(self, req, ctx):
        self.meta.register_master(req.masterId, {c.name: c.value for c in req.options.configs})
        return pb.meta.RegisterMasterPResponse()

    def MasterHeartbeat(self, req, ctx):
        cmd = self.meta.master_heartbeat(req.masterId)
        return pb.meta.MasterHeartbeatPResponse(command=pb.meta.MetaCommand.values_by_name[cmd].number)

    # MetricsMasterClientService
    def ClearMetrics(self, req, ctx):
        self.mm.clear()
        return pb.metric.ClearMetricsPResponse()

    def MetricsHeartbeat(self, req, ctx):
        self.mm.client_heartbeat(req.options.clientMetrics)
        return pb.metric.MetricsHeartbeatPResponse()

    def GetMetrics(self, req, ctx):
        r = pb.metric.GetMetricsPResponse()
        for k, v in self.mm.get_metrics().items():
            r.metrics[k].doubleValue = v
        return r

    # JournalMasterClientService (RaftJournalSystem.getQuorumServerInfoList / removeQuorumServer)
    def GetQuorumInfo(self, req, ctx):
        qi = getattr(self.js, "quorum_info", None)
        if qi is None:      # UFS journal: the "quorum" is this master
            host, _, port = self.meta.master_address.partition(":")
            members = [(host, int(port or 0), True)]
        else:
            members = [(a.rsplit(":", 1)[0], int(a.rsplit(":", 1)[1]), ok) for a, ok in qi()]
        return pb.journal_master.GetQuorumInfoPResponse(domain=1, serverInfo=[
            pb.journal_master.QuorumServerInfo(serverAddress=pb.grpc.NetAddress(host=h, rpcPort=p),
                                               serverState=1 if ok else 2) for h, p, ok in members])

    def RemoveQuorumServer(self, req, ctx):
        rm = getattr(self.js, "remove_quorum_server", None)
        if rm is None:
            from ..utils.exceptions import InvalidArgumentException
            raise InvalidArgumentException("quorum membership needs the EMBEDDED journal")
        a = req.serverAddress
        rm(f"{a.host}:{a.rpcPort}")
        return pb.journal_master.RemoveQuorumServerPResponse()
