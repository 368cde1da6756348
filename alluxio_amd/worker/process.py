"""Worker process: tiered HBM store + BlockWorker + data server + master sync threads.

Parity: core/server/worker/src/main/java/alluxio/worker/AlluxioWorkerProcess.java (:99-265),
block/BlockMasterSync.java:60-199 (getWorkerId -> register -> periodic heartbeat carrying used
bytes, added/removed blocks, metrics; executes Free / Register commands), PinListSync.java,
SessionCleaner.java, the storage checker (TieredBlockStore.checkStorage :974-1009, reported as
lost storage) and the FileSystemMaster worker heartbeat (persisted files).
"""
from __future__ import annotations

import logging
import os
import socket
import threading

from .. import metrics as msys
from ..conf import Configuration
from ..proto import pb
from ..rpc import Channel, RpcServer
from ..utils import heartbeat as hb
from ..utils import ids
from .block_worker import BlockWorker
from .services import SVC_BLOCK_WORKER, BlockWorkerService
from .store import TieredStore

LOG = logging.getLogger(__name__)


class BlockMasterSync:
    def __init__(self, worker: BlockWorker, process: "AlluxioWorkerProcess"):
        self.w = worker
        self.p = process
        self.registered = False

    def register(self) -> None:
        bm = self.w._bm()
        wid = bm.GetWorkerId(pb.block.GetWorkerIdPRequest(workerNetAddress=self.w.address)).workerId
        self.w.worker_id = wid
        store = self.w.store
        req = pb.block.RegisterWorkerPRequest(workerId=wid, storageTiers=store.tier_aliases)
        for k, v in store.capacity_by_tier().items():
            req.totalBytesOnTiers[k] = v
        for k, v in store.used_by_tier().items():
            req.usedBytesOnTiers[k] = v
        for (tier, medium), blocks in self.w.current_blocks().items():
            e = req.currentBlocks.add()
            e.key.tierAlias = tier
            e.key.mediumType = medium
            e.value.blockId.extend(blocks)
        for k, v in sorted(self.p.conf.to_map().items()):
            req.options.configs.add(name=k, value=v)
        bm.RegisterWorker(req)
        self.w.drain_report()  # everything current was just reported
        self.registered = True

    def heartbeat(self) -> None:
        if not self.registered:
            self.register()
            return
        removed, added = self.w.drain_report()
        req = pb.block.BlockHeartbeatPRequest(workerId=self.w.worker_id, removedBlockIds=removed)
        for k, v in self.w.store.used_by_tier().items():
            req.usedBytesOnTiers[k] = v
        for (tier, medium), blocks in added.items():
            e = req.addedBlocks.add()
            e.key.tierAlias = tier
            e.key.mediumType = medium
            e.value.blockId.extend(blocks)
        for name, mtype, value in self.w.metrics.report_metrics():
            req.options.metrics.add(name=name, value=value, instance="Worker", source=self.w.address.host,
                                    metricType=pb.grpc.MetricType.values_by_name[mtype].number)
        for i in range(self.w.native.num_dirs()):
            if not self.w.native.dir_healthy(i):
                spec = self.w.native.dir_spec(i)
                req.lostStorage[spec.tier_alias].storage.append(spec.path or f"{spec.medium}:{i}")
        resp = self.w._bm().BlockHeartbeat(req)
        cmd = pb.grpc.CommandType.values_by_number[resp.command.commandType].name
        if cmd == "Register":
            self.registered = False
            self.register()
        elif cmd == "Free":
            for bid in resp.command.data:
                try:
                    self.w.remove_block(ids.MASTER_COMMAND_SESSION_ID, bid)
                except Exception:  # noqa: BLE001
                    LOG.debug("free of %d failed", bid, exc_info=True)
            removed2, _ = self.w.drain_report()
            if removed2:
                self.w._bm().BlockHeartbeat(pb.block.BlockHeartbeatPRequest(
                    workerId=self.w.worker_id, removedBlockIds=removed2))


class AlluxioWorkerProcess:
    def __init__(self, conf: Configuration | None = None, master_address: str | None = None,
                 host: str = "127.0.0.1", port: int | None = None, device: int | None = None,
                 enable_grpc: bool = True, work_dir: str | None = None):
        self.conf = conf or Configuration(load_site=True)
        self.master_address = master_address or "{}:{}".format(
            self.conf.get("alluxio.master.hostname", "127.0.0.1"), self.conf.get_int("alluxio.master.rpc.port"))
        self.host = host
        self.port = self.conf.get_int("alluxio.worker.rpc.port") if port is None else port
        self.store = TieredStore(self.conf, device, work_dir)
        from ..rpc import master_channel
        self.master_channel = master_channel(self.master_address)
        self.worker = BlockWorker(self.conf, self.store, self.master_channel)
        self.domain_socket = self._domain_socket_path() if enable_grpc else None
        from .data_server import available
        # the native data server (GrpcDataServer analogue) takes the domain socket when it runs
        self._native_data = enable_grpc and self.conf.get_bool("alluxio.worker.data.server.native.enabled", "true") \
            and available()
        self.server = RpcServer(host, self.port, metrics=msys.metrics("Worker"), enable_grpc=enable_grpc,
                                conf=self.conf, domain_socket=None if self._native_data else self.domain_socket)
        self.server.add_servicer(SVC_BLOCK_WORKER, BlockWorkerService(self.worker, self.conf))

        self.sync = BlockMasterSync(self.worker, self)
        self._threads: list[hb.HeartbeatThread] = []
        self.job_worker = None
        self._job_fs = None
        self.web = None
        self.web_port = 0
        self.data_server = None

    @property
    def address(self) -> str:
        return self.server.address

    def _domain_socket_path(self) -> str | None:
        """``alluxio.worker.data.server.domain.socket.address`` (a directory when
        ``...as.uuid`` is true: one socket file per worker)."""
        a = self.conf.get_raw("alluxio.worker.data.server.domain.socket.address")
        if not a:
            if a is not None or not self.conf.get_bool("alluxio.worker.data.server.domain.socket.default.enabled",
                                                       "true"):
                return None              # explicitly empty, or the default socket is off
            # the same-node default: one socket per worker in a short per-user directory (sun_path
            # holds 108 bytes)
            import uuid
            d = f"/tmp/alluxio-uds-{os.getuid()}"
            try:
                os.makedirs(d, mode=0o700, exist_ok=True)
            except OSError:
                return None
            return os.path.join(d, uuid.uuid4().hex[:16])
        if self.conf.get_bool("alluxio.worker.data.server.domain.socket.as.uuid", "false"):
            import uuid
            return os.path.join(a, uuid.uuid4().hex)
        return a

    def _enable_peer_access(self) -> list[int]:
        """Map every other GPU of the node into this worker's device (xGMI peer access), so peer
        pulls and remote ring reads by kernels on this GPU can read their HBM; returns the peers."""
        from ..ops.native import has_gpu, lib
        if not (has_gpu() and self.store.has_device_tier):
            return []
        C = lib()
        me, peers = int(self.store.device), []
        for d in range(C.device_count()):
            if d == me:
                continue
            try:
                if C.enable_peer_access(me, d):
                    peers.append(d)
            except Exception:  # noqa: BLE001 - no P2P path to that device
                LOG.debug("peer access %d -> %d unavailable", me, d, exc_info=True)
        return peers

    def start(self, register: bool = True, start_heartbeats: bool = True) -> str:
        from .. import metrics as msys
        from ..utils.pause_monitor import from_conf as pause_monitor
        self._sinks = msys.load_sinks(self.conf, self.worker.metrics)
        self.pause_monitor = pause_monitor(self.conf, "worker", self.worker.metrics)
        if self.pause_monitor is not None:
            self.pause_monitor.start()
        addr = self.server.start()
        host, port = addr.rsplit(":", 1)
        data_port = int(port)
        if self._native_data:
            # the native gRPC data port (GrpcDataServer analogue): ReadBlock streamed from C++
            from .data_server import WorkerDataServer
            self.data_server = WorkerDataServer(self.server, self.worker, self.conf, self.host, self.domain_socket)
            data_port = self.data_server.start()
        ti = pb.grpc.TieredIdentity(tiers=[pb.grpc.LocalityTier(tierName="node", value=socket.gethostname()),
                                           pb.grpc.LocalityTier(tierName="gpu", value=str(self.store.device))])
        self.worker.address = pb.grpc.WorkerNetAddress(host=host, rpcPort=int(port), dataPort=data_port,
                                                       domainSocketPath=self.domain_socket or "",
                                                       webPort=0, tieredIdentity=ti,
                                                       containerHost=socket.gethostname())
        if self.conf.get_bool("alluxio.web.server.enabled", "true"):
            from ..web import WebServer, worker_routes
            self.web = WebServer(self.conf.get("alluxio.worker.web.bind.host", "0.0.0.0"),
                                 self.conf.get_int("alluxio.worker.web.port"), worker_routes(self), "worker")
            self.web_port = self.web.start()
            self.worker.address.webPort = self.web_port
        from ..client.context import register_local_worker
        register_local_worker(addr, self.worker)
        self.peer_devices = self._enable_peer_access()
        if register:
            self.sync.register()
        if start_heartbeats:
            c = self.conf
            for name, fn, ms in [
                (hb.WORKER_BLOCK_SYNC, self.sync.heartbeat, c.get_ms("alluxio.worker.block.heartbeat.interval")),
                (hb.WORKER_PIN_LIST_SYNC, self.pin_list_sync, c.get_ms("alluxio.worker.block.heartbeat.interval")),
                (hb.WORKER_SESSION_CLEANER, self.worker.cleanup_expired_sessions,
                 c.get_ms("alluxio.worker.session.timeout")),
                (hb.WORKER_FILESYSTEM_MASTER_SYNC, self.fs_heartbeat,
                 c.get_ms("alluxio.worker.filesystem.heartbeat.interval", "1sec")),
                (hb.WORKER_STORAGE_HEALTH, self.check_storage, c.get_ms("alluxio.worker.storage.checker.interval", "1min")
                 if False else 60_000),
            ]:
                t = hb.HeartbeatThread(name, fn, ms)
                t.start()
                self._threads.append(t)
        from .management import TierManager
        self.tier_manager = TierManager(self.worker, self.conf)
        if start_heartbeats and len(self.tier_manager.tiers()) > 1:
            self.add_heartbeat(hb.WORKER_TIER_MANAGEMENT, self.tier_manager.run_once,
                               self.conf.get_ms("alluxio.worker.management.task.interval", "1sec")
                               if self.conf.get_raw("alluxio.worker.management.task.interval") else 1000)
        if self.conf.get_bool("alluxio.job.worker.enabled", "true"):
            self._start_job_worker(start_heartbeats)
        LOG.info("worker serving at %s (device %d)", addr, self.store.device)
        return addr

    def _start_job_worker(self, start_heartbeat: bool) -> None:
        """Job worker co-located with the block worker (reference AlluxioJobWorkerProcess runs
        beside each worker; here it shares the process so tasks read/write the local HBM store
        directly)."""
        from ..client.file_system import FileSystem
        from ..job.master import JobWorker
        self._job_fs = FileSystem(conf=self.conf, master_address=self.master_address)
        self.job_worker = JobWorker(self.master_channel, self.worker.address, self._job_fs, self.worker,
                                    pool_size=self.conf.get_int("alluxio.job.worker.threadpool.size"))
        try:
            self.job_worker.register()
        except Exception:  # noqa: BLE001 - job master may be absent; heartbeat retries
            LOG.info("job master not reachable at %s; job worker will retry", self.master_address)
        if start_heartbeat:
            self.add_heartbeat(hb.JOB_WORKER_COMMAND_HANDLING, self._job_heartbeat,
                               self.conf.get_ms("alluxio.job.master.worker.heartbeat.interval"))

    def _job_heartbeat(self) -> None:
        try:
            self.job_worker.heartbeat()
        except Exception as e:  # noqa: BLE001
            if "UNIMPLEMENTED" in str(e) or "not found" in str(e).lower():
                return
            raise

    def add_heartbeat(self, name: str, fn, interval_ms: int) -> None:
        t = hb.HeartbeatThread(name, fn, interval_ms)
        t.start()
        self._threads.append(t)

    def pin_list_sync(self) -> None:
        fsm = self.worker._fsm()
        ids_ = fsm.GetPinnedFileIds(pb.file.GetPinnedFileIdsPRequest()).pinnedFileIds
        self.worker.update_pinned(list(ids_))

    def fs_heartbeat(self) -> None:
        if self.worker.worker_id == ids.INVALID_WORKER_ID:
            return
        persisted, self.worker.persisted_files = self.worker.persisted_files, []
        self.worker._fsm().FileSystemHeartbeat(pb.file.FileSystemHeartbeatPRequest(
            workerId=self.worker.worker_id, persistedFiles=persisted))

    def check_storage(self) -> None:
        """GPU health into the storage checker: a failing HIP device marks its dirs lost."""
        if not self.store.has_device_tier:
            return
        try:
            import torch
            torch.cuda.synchronize(self.store.device)
        except Exception:  # noqa: BLE001
            LOG.error("HIP device %d failed; marking HBM dirs lost", self.store.device)
            for i in range(self.worker.native.num_dirs()):
                if self.store.dirs[i].medium == "HBM":
                    self.worker.native.set_dir_healthy(i, False)

    def stop(self) -> None:
        for sk in getattr(self, "_sinks", []):
            sk.stop()
        if getattr(self, "pause_monitor", None) is not None:
            self.pause_monitor.stop()
        for t in self._threads:
            t.shutdown(join=False)
        for t in self._threads:
            t.shutdown(join=True)
        self._threads.clear()
        from ..client.context import unregister_local_worker
        if self.server.address:
            unregister_local_worker(self.server.address)
            if self.domain_socket:
                from ..rpc import unregister_domain_socket
                unregister_domain_socket(self.server.address, self.domain_socket)
        if self.data_server is not None:
            self.data_server.stop()
            self.data_server = None
        self.server.stop()
        if self.web is not None:
            self.web.stop()
            self.web = None
        if self.job_worker is not None:
            self.job_worker.close()
        if self._job_fs is not None:
            self._job_fs.close()
        self.worker.close()


def main(argv=None) -> int:  # pragma: no cover - CLI entry
    import argparse
    ap = argparse.ArgumentParser(description="alluxio_amd worker (one per MI355X)")
    ap.add_argument("--master", default=None)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--device", type=int, default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from ..conf import Configuration as _C
    from ..web.logserver import attach
    attach("WORKER", _C(load_site=True))
    w = AlluxioWorkerProcess(master_address=a.master, host=a.host, port=a.port, device=a.device)
    w.start()
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        pass
    w.stop()
    return 0


if __name__ == "__main__":  # pragma: no cover
    raise SystemExit(main())
