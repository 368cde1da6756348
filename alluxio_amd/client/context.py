"""Client context: configuration, master/worker channels, cached worker list, local workers.

Parity: core/client/fs/src/main/java/alluxio/client/file/FileSystemContext.java:120-586 (master
client pools, per-worker client pools, cached worker list, local-worker detection by tiered
identity, cluster-config reinitialisation).  A worker running in the same process registers
itself here, which lets reads and writes bypass RPC entirely (the in-process analogue of the
reference's short-circuit I/O); same-node workers in other processes are reached over gRPC or
HIP IPC (``OpenDeviceBlock``).
"""
from __future__ import annotations

import socket
import threading
import time

from .. import metrics as msys
from ..conf import Configuration
from ..proto import pb
from ..rpc import ChannelPool
from ..security import login_user

SVC_FS = "alluxio.grpc.file.FileSystemMasterClientService"
SVC_BLOCK = "alluxio.grpc.block.BlockMasterClientService"
SVC_META = "alluxio.grpc.meta.MetaMasterClientService"
SVC_META_CONF = "alluxio.grpc.meta.MetaMasterConfigurationService"
SVC_METRICS = "alluxio.grpc.metric.MetricsMasterClientService"
SVC_WORKER = "alluxio.grpc.block.BlockWorker"

_LOCAL_WORKERS: dict[str, object] = {}
_LW_LOCK = threading.Lock()


def register_local_worker(address: str, worker) -> None:
    with _LW_LOCK:
        _LOCAL_WORKERS[address] = worker


def unregister_local_worker(address: str) -> None:
    with _LW_LOCK:
        _LOCAL_WORKERS.pop(address, None)


def local_worker(address: str):
    with _LW_LOCK:
        return _LOCAL_WORKERS.get(address)


def worker_address_str(addr) -> str:
    return f"{addr.host}:{addr.rpcPort}"


class FileSystemContext:
    def __init__(self, conf: Configuration | None = None, master_address: str | None = None,
                 user: str | None = None):
        self.conf = conf or Configuration(load_site=True)
        addrs = master_address or self.conf.get_raw("alluxio.master.rpc.addresses") or "{}:{}".format(
            self.conf.get("alluxio.master.hostname", "127.0.0.1"), self.conf.get_int("alluxio.master.rpc.port"))
        self.master_addresses = [a.strip() for a in str(addrs).split(",") if a.strip()]
        self.master_address = self.master_addresses[0]
        self._master_ch = None
        self.user = user or login_user(self.conf)
        self.pool = ChannelPool(self.conf)
        self.metrics = msys.metrics("Client")
        self.hostname = socket.gethostname()
        self._workers = None
        self._workers_at = 0.0
        self._lock = threading.Lock()
        self.worker_list_ttl = self.conf.get_ms("alluxio.user.worker.list.refresh.interval", "2min") / 1000.0
        self._closed = False
        self._keeper = None
        from ..parallel.ipc import set_open_timeout
        set_open_timeout(self.conf.get_ms("alluxio.user.short.circuit.open.timeout", "30s"))
        self._metrics_hb = None
        if self.conf.get_bool("alluxio.user.metrics.collection.enabled"):
            from ..utils import heartbeat as hb
            self._metrics_hb = hb.HeartbeatThread(hb.CLIENT_METRICS_SYNC, self.sync_metrics,
                                                  self.conf.get_ms("alluxio.user.metrics.heartbeat.interval"))
            self._metrics_hb.start()

    def sync_metrics(self) -> int:
        """ClientMasterSync: send this client's metric deltas to the metrics master."""
        ms = self.metrics.report_metrics()
        if not ms:
            return 0
        cm = pb.metric.ClientMetrics(source=f"{self.hostname}:{self.user}")
        for name, mtype, value in ms:
            cm.metrics.add(instance="Client", source=cm.source, name=name, value=value,
                           metricType=pb.grpc.MetricType.values_by_name[mtype].number)
        self.metrics_master().MetricsHeartbeat(pb.metric.MetricsHeartbeatPRequest(
            options=pb.metric.MetricsHeartbeatPOptions(clientMetrics=[cm])))
        return len(ms)

    # ---- stubs --------------------------------------------------------------------------------
    def master_channel(self):
        """Channel to the (primary) master; an HA address list yields a failover channel."""
        if len(self.master_addresses) == 1:
            return self.pool.get(self.master_address, self.user)
        if self._master_ch is None:
            from ..rpc import FailoverChannel
            self._master_ch = FailoverChannel(self.master_addresses, self.user, self.pool,
                                              self.conf.get_ms("alluxio.user.rpc.retry.max.duration", "2min") / 1000)
        return self._master_ch

    def fs_master(self):
        return self.master_channel().stub(SVC_FS)

    def block_master(self):
        return self.master_channel().stub(SVC_BLOCK)

    def meta_master(self):
        return self.master_channel().stub(SVC_META)

    def meta_config(self):
        return self.master_channel().stub(SVC_META_CONF)

    def metrics_master(self):
        return self.master_channel().stub(SVC_METRICS)

    def worker_channel(self, address: str):
        return self.pool.get(address, self.user)

    def worker_stub(self, address: str):
        return self.worker_channel(address).stub(SVC_WORKER)

    # ---- workers ------------------------------------------------------------------------------
    def workers(self, refresh: bool = False) -> list:
        with self._lock:
            if refresh or self._workers is None or time.time() - self._workers_at > self.worker_list_ttl:
                self._workers = list(self.block_master().GetWorkerInfoList(
                    pb.block.GetWorkerInfoListPOptions()).workerInfos)
                self._workers_at = time.time()
                for w in self._workers:
                    self._note_domain_socket(w.address)
            return list(self._workers)

    def _note_domain_socket(self, addr) -> None:
        """Same-node worker with a domain socket: its gRPC traffic skips TCP.  As in the reference
        the socket is used whenever the worker advertises one and it is reachable from here
        (NettyUtils.isDomainSocketAccessible, core/common/.../util/network/NettyUtils.java:109-119);
        alluxio.user.short.circuit.* only decides between it and the IPC short circuit."""
        import os
        from ..rpc import register_domain_socket
        p = addr.domainSocketPath
        if p and self.is_local(addr) and os.path.exists(p):
            register_domain_socket(worker_address_str(addr), p)

    def is_local(self, addr) -> bool:
        """Same node as this client (reference: tiered identity 'node' tier match)."""
        for t in addr.tieredIdentity.tiers:
            if t.tierName == "node":
                return t.value == self.hostname
        return addr.host in ("127.0.0.1", "localhost", self.hostname)

    def in_process_worker(self, addr):
        # the in-process transport switch also turns off direct calls into a same-process worker,
        # so every byte goes through the worker's data server
        if not self.conf.get_bool("alluxio.user.network.inprocess.transport.enabled", "true"):
            return None
        return local_worker(worker_address_str(addr))

    def session_keeper(self):
        """Renewer of worker sessions held open by short-circuit handles (session_keeper.py):
        renews every quarter of ``alluxio.worker.session.timeout``, at least every 10 s."""
        with self._lock:
            if self._keeper is None:
                from .session_keeper import SessionKeeper
                timeout = self.conf.get_ms("alluxio.worker.session.timeout") / 1000.0
                self._keeper = SessionKeeper(self, min(10.0, timeout / 4))
            return self._keeper

    def close(self) -> None:
        if self._keeper is not None:
            self._keeper.close()
        if self._metrics_hb is not None:
            self._metrics_hb.shutdown(join=False)
            self._metrics_hb = None
        self._closed = True
        self.pool.close()
