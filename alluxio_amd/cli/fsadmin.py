"""``alluxio fsadmin`` — administrative shell.

Parity: shell/src/main/java/alluxio/cli/fsadmin/FileSystemAdminShell.java and commands under
shell/src/main/java/alluxio/cli/fsadmin/command/ (Backup, Doctor, GetBlockInfo, Journal
(quorum info/remove, checkpoint), Metrics (clear), PathConf (list/show/add/remove), Report
(summary/capacity/metrics/ufs/jobservice — report/*.java), Ufs (--mode)).
"""
from __future__ import annotations

import sys
import time

from ..proto import enum_name, pb
from ..utils.exceptions import AlluxioStatusException
from ..utils.format import bytes_to_human


class FileSystemAdminShell:
    def __init__(self, fs=None, out=None, conf=None):
        if fs is None:
            from ..client.file_system import FileSystem
            fs = FileSystem(conf=conf)
        self.fs = fs
        self.ctx = fs.ctx
        self.out = out or sys.stdout

    def p(self, *a):
        print(*a, file=self.out)

    def run(self, argv) -> int:
        if not argv:
            self.p("Usage: alluxio fsadmin [backup|checkpoint|doctor|getBlockInfo|journal|metrics|pathConf|report|ufs]")
            return 1
        cmd, args = argv[0], argv[1:]
        fn = getattr(self, "cmd_" + cmd, None)
        if fn is None:
            self.p(f"{cmd} is an unknown command.")
            return 1
        try:
            return fn(args) or 0
        except AlluxioStatusException as e:
            self.p(str(e))
            return -1
        except ValueError as e:
            self.p(str(e))
            return -1

    # ---- report -------------------------------------------------------------------------------
    def cmd_report(self, args) -> int:
        sub = args[0] if args else "summary"
        if sub == "summary":
            return self._summary()
        if sub == "capacity":
            return self._capacity(args[1:])
        if sub == "metrics":
            return self._metrics()
        if sub == "ufs":
            return self._ufs()
        if sub == "jobservice":
            return self._jobservice()
        raise ValueError(f"Unknown report category {sub}")

    def _summary(self) -> int:
        mi = self.ctx.meta_master().GetMasterInfo(pb.meta.GetMasterInfoPOptions()).masterInfo
        bi = self.ctx.block_master().GetBlockMasterInfo(pb.block.GetBlockMasterInfoPOptions()).blockMasterInfo
        self.p("Alluxio cluster summary: ")
        self.p(f"    Master Address: {mi.leaderMasterAddress}")
        self.p(f"    Web Port: {mi.webPort}")
        self.p(f"    Rpc Port: {mi.rpcPort}")
        self.p(f"    Started: {time.strftime('%m-%d-%Y %H:%M:%S', time.localtime(mi.startTimeMs / 1000))}")
        self.p(f"    Uptime: {mi.upTimeMs // 1000} sec")
        self.p(f"    Version: {mi.version}")
        self.p(f"    Safe Mode: {mi.safeMode}")
        self.p(f"    Live Workers: {bi.liveWorkerNum}")
        self.p(f"    Lost Workers: {bi.lostWorkerNum}")
        self.p(f"    Total Capacity: {bytes_to_human(bi.capacityBytes)}")
        for t, v in sorted(bi.capacityBytesOnTiers.items()):
            self.p(f"        Tier: {t}  Size: {bytes_to_human(v)}")
        self.p(f"    Used Capacity: {bytes_to_human(bi.usedBytes)}")
        for t, v in sorted(bi.usedBytesOnTiers.items()):
            self.p(f"        Tier: {t}  Size: {bytes_to_human(v)}")
        self.p(f"    Free Capacity: {bytes_to_human(bi.freeBytes)}")
        return 0

    def _capacity(self, args) -> int:
        rng = "ALL"
        if "-live" in args:
            rng = "LIVE"
        elif "-lost" in args:
            rng = "LOST"
        opts = pb.block.GetWorkerReportPOptions(workerRange=pb.block.WorkerRange.values_by_name[rng].number)
        infos = list(self.ctx.block_master().GetWorkerReport(opts).workerInfos)
        cap = sum(w.capacityBytes for w in infos)
        used = sum(w.usedBytes for w in infos)
        self.p("Capacity information for all workers: ")
        self.p(f"    Total Capacity: {bytes_to_human(cap)}")
        self.p(f"    Used Capacity: {bytes_to_human(used)}")
        if cap:
            self.p(f"    Used Percentage: {used * 100 // cap}%")
            self.p(f"    Free Percentage: {100 - used * 100 // cap}%")
        self.p("")
        self.p(f"{'Worker Name':<24}{'Last Heartbeat':<16}{'Storage':<10}{'Total':<12}{'Used':<12}")
        for w in infos:
            name = f"{w.address.host}:{w.address.rpcPort}"
            self.p(f"{name:<24}{w.lastContactSec:<16}{'capacity':<10}{bytes_to_human(w.capacityBytes):<12}"
                   f"{bytes_to_human(w.usedBytes):<12}")
            for t, v in sorted(w.capacityBytesOnTiers.items()):
                self.p(f"{'':<40}{t:<10}{bytes_to_human(v):<12}{bytes_to_human(w.usedBytesOnTiers.get(t, 0)):<12}")
        return 0

    def _metrics(self) -> int:
        ms = self.ctx.metrics_master().GetMetrics(pb.metric.GetMetricsPOptions()).metrics
        for k in sorted(ms):
            v = ms[k]
            val = v.stringValue if v.stringValue else (int(v.doubleValue) if v.doubleValue == int(v.doubleValue)
                                                       else v.doubleValue)
            self.p(f"{k:<60}{val}")
        return 0

    def _ufs(self) -> int:
        for mp, info in sorted(self.fs.get_mount_table().items()):
            flags = ("readonly, " if info.readOnly else "") + ("shared" if info.shared else "not shared")
            self.p(f"{info.ufsUri} on {mp} ({info.ufsType}, capacity={info.ufsCapacityBytes}, "
                   f"used={info.ufsUsedBytes}, {flags}, properties={dict(info.properties)})")
        return 0

    def _jobservice(self) -> int:
        from ..job import JobClient
        jc = JobClient(self.ctx.master_channel())
        for h in jc.worker_health():
            self.p(f"Worker: {h.hostname:<20} Task Pool Size: {h.taskPoolSize:<6} Unfinished Tasks: "
                   f"{h.unfinishedTasks:<6} Active Tasks: {h.numActiveTasks:<6} Load Avg: "
                   f"{', '.join(f'{x:.2f}' for x in h.loadAverage)}")
        s = jc.summary()
        self.p("")
        self.p("Status: " + ", ".join(f"{enum_name(pb.job.Status, c.status)}:{c.count}" for c in s.summaryPerStatus))
        self.p("")
        self.p("10 Most Recently Modified Jobs:")
        for j in s.recentActivities:
            self.p(f"Timestamp: {j.lastUpdated:<16} Id: {j.id:<16} Name: {j.name:<12} Status: "
                   f"{enum_name(pb.job.Status, j.status)}")
        self.p("10 Most Recently Failed Jobs:")
        for j in s.recentFailures:
            self.p(f"Timestamp: {j.lastUpdated:<16} Id: {j.id:<16} Name: {j.name:<12} Status: FAILED")
        return 0

    # ---- other commands ---------------------------------------------------------------------
    def cmd_backup(self, args) -> int:
        target = next((a for a in args if not a.startswith("-")), "")
        # [directory] [--local] [--allow-leader] (BackupCommand: delegated to a standby in HA
        # clusters when alluxio.master.backup.delegation.enabled; --allow-leader permits the
        # primary to take it when no standby is available)
        req = pb.meta.BackupPRequest(options=pb.meta.BackupPOptions(localFileSystem="--local" in args,
                                                                    allowLeader="--allow-leader" in args),
                                     targetDirectory=target)
        st = self.ctx.meta_master().Backup(req)
        state = enum_name(pb.meta.BackupState, st.backupState)
        if state == "Failed":
            self.p(f"Backup failed: {st.backupError.decode(errors='replace')}")
            return -1
        self.p(f"Backup Host        : {st.backupHost}")
        self.p(f"Backup URI         : {st.backupUri}")
        self.p(f"Backup Entry Count : {st.entryCount}")
        return 0

    def cmd_checkpoint(self, args) -> int:
        host = self.ctx.meta_master().Checkpoint(pb.meta.CheckpointPOptions()).masterHostname
        self.p(f"Successfully took a checkpoint on master {host}")
        return 0

    def cmd_doctor(self, args) -> int:
        cat = args[0] if args else "all"
        rc = 0
        if cat in ("all", "configuration"):
            rep = self.ctx.meta_master().GetConfigReport(pb.meta.GetConfigReportPOptions()).report
            status = enum_name(pb.meta.ConfigStatus, rep.status) if rep.status else "PASSED"
            if not rep.errors and not rep.warns:
                self.p("No server-side configuration errors or warnings.")
            for kind, group in (("errors", rep.errors), ("warnings", rep.warns)):
                for scope, props in group.items():
                    self.p(f"Server-side configuration {kind} ({scope}): ")
                    for ip in props.properties:
                        vals = "; ".join(f"{v} ({', '.join(h.values)})" for v, h in ip.values.items())
                        self.p(f"key: {ip.name} value: {vals}")
            if status == "FAILED":
                rc = -1
        if cat in ("all", "storage"):
            lost = self.ctx.block_master().GetWorkerLostStorage(pb.block.GetWorkerLostStoragePOptions())
            if not lost.workerLostStorageInfo:
                self.p("All worker storage paths are in working state.")
            for info in lost.workerLostStorageInfo:
                self.p(f"The following storage paths are lost in worker {info.address.host}: ")
                for tier, sl in info.lostStorage.items():
                    for path in sl.storage:
                        self.p(f"{tier}: {path}")
        return rc

    def cmd_getBlockInfo(self, args) -> int:
        if len(args) != 1:
            raise ValueError("getBlockInfo requires a block id")
        bid = int(args[0])
        bi = self.ctx.block_master().GetBlockInfo(pb.block.GetBlockInfoPRequest(blockId=bid)).blockInfo
        self.p(f"BlockInfo{{id={bi.blockId}, length={bi.length}, locations="
               f"{[f'{l.workerAddress.host}:{l.workerAddress.rpcPort}/{l.tierAlias}' for l in bi.locations]}}}")
        from ..utils import ids
        fid = ids.get_file_id(bid)
        if fid:
            try:
                path = self.ctx.fs_master().GetFilePath(pb.file.GetFilePathPRequest(fileId=fid)).path
                self.p(f"This block belongs to file {{id={fid}, path={path}}}")
            except AlluxioStatusException:
                pass
        return 0

    def cmd_journal(self, args) -> int:
        if args[:2] == ["quorum", "info"]:
            r = self.ctx.master_channel().stub("alluxio.grpc.journal.JournalMasterClientService").GetQuorumInfo(
                pb.journal_master.GetQuorumInfoPRequest(options=pb.journal_master.GetQuorumInfoPOptions()))
            self.p(f"Journal domain : {enum_name(pb.journal_master.JournalDomain, r.domain) if r.domain else 'MASTER'}")
            self.p(f"Quorum size    : {len(r.serverInfo)}")
            for s in r.serverInfo:
                self.p(f"{enum_name(pb.journal_master.QuorumServerState, s.serverState):<12}"
                       f"{s.serverAddress.host}:{s.serverAddress.rpcPort}")
            return 0
        if args[:2] == ["quorum", "remove"]:
            # QuorumRemoveCommand: journal quorum remove -address <host:port> [-domain MASTER]
            if "-address" not in args:
                raise ValueError("usage: journal quorum remove -address <host:port>")
            host, _, port = args[args.index("-address") + 1].rpartition(":")
            self.ctx.master_channel().stub("alluxio.grpc.journal.JournalMasterClientService").RemoveQuorumServer(
                pb.journal_master.RemoveQuorumServerPRequest(
                    options=pb.journal_master.RemoveQuorumServerPOptions(),
                    serverAddress=pb.grpc.NetAddress(host=host, rpcPort=int(port))))
            self.p(f"Removed server at: {host}:{port} from quorum")
            return 0
        if args[:1] == ["checkpoint"]:
            return self.cmd_checkpoint([])
        raise ValueError("usage: journal [quorum info | quorum remove -address <host:port> | checkpoint]")

    def cmd_metrics(self, args) -> int:
        if args[:1] != ["clear"]:
            raise ValueError("usage: metrics clear [--master] [--workers <host:port,...>]")
        if "--master" in args or "--workers" not in args:
            self.ctx.metrics_master().ClearMetrics(pb.metric.ClearMetricsPRequest())
        targets = []
        if "--workers" in args:
            targets = args[args.index("--workers") + 1].split(",")
        elif "--master" not in args:
            from .. import client
            del client
            targets = [f"{w.address.host}:{w.address.rpcPort}" for w in self.ctx.workers(refresh=True)]
        for t in targets:
            self.ctx.worker_stub(t).ClearMetrics(pb.block.ClearMetricsRequest())
        self.p("Successfully cleared metrics.")
        return 0

    def cmd_pathConf(self, args) -> int:
        if not args:
            raise ValueError("usage: pathConf [list|show|add|remove]")
        svc = self.ctx.meta_config()
        sub = args[0]
        if sub == "list":
            r = svc.GetConfiguration(pb.meta.GetConfigurationPOptions(ignoreClusterConf=True))
            for p in sorted(r.pathConfigs):
                self.p(p)
            return 0
        if sub == "show":
            path = args[-1]
            r = svc.GetConfiguration(pb.meta.GetConfigurationPOptions(ignoreClusterConf=True))
            props = {}
            for pth, cps in r.pathConfigs.items():
                if "--all" in args and (path == pth or path.startswith(pth.rstrip("/") + "/")):
                    props.update({c.name: c.value for c in cps.properties})
                elif pth == path:
                    props.update({c.name: c.value for c in cps.properties})
            for k in sorted(props):
                self.p(f"{k}={props[k]}")
            return 0
        if sub == "add":
            path = args[-1]
            kv = {}
            i = 1
            while i < len(args) - 1:
                if args[i] == "--property":
                    k, v = args[i + 1].split("=", 1)
                    kv[k] = v
                    i += 2
                else:
                    i += 1
            svc.SetPathConfiguration(pb.meta.SetPathConfigurationPRequest(path=path, properties=kv))
            return 0
        if sub == "remove":
            path = args[-1]
            keys = []
            if "--keys" in args:
                keys = args[args.index("--keys") + 1].split(",")
            svc.RemovePathConfiguration(pb.meta.RemovePathConfigurationPRequest(path=path, keys=keys))
            return 0
        raise ValueError(f"unknown pathConf subcommand {sub}")

    def cmd_ufs(self, args) -> int:
        if len(args) != 3 or args[0] != "--mode":
            raise ValueError("usage: ufs --mode <noAccess/readOnly/readWrite> <ufsPath>")
        mode = {"noAccess": "NO_ACCESS", "readOnly": "READ_ONLY", "readWrite": "READ_WRITE"}[args[1]]
        self.fs.update_ufs_mode(args[2], mode)
        self.p(f"Ufs mode updated to {args[1]}")
        return 0


def main(argv=None, out=None) -> int:
    sh = FileSystemAdminShell(out=out)
    try:
        return sh.run(list(sys.argv[1:] if argv is None else argv))
    finally:
        sh.fs.close()
