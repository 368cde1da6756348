"""In-process cluster: one master + N workers in this process.

Parity: minicluster/src/main/java/alluxio/master/LocalAlluxioCluster.java:40-157 and
AbstractLocalAlluxioCluster.java (temp work dir, local UFS, 1 master + N workers, start/stop,
``getClient``); tests/.../LocalAlluxioClusterResource.java (per-test config overrides).
Workers default to the HBM tier when a HIP device is visible (one worker per device, round
robin) and to a DRAM arena otherwise.
"""
from __future__ import annotations

import os
import shutil
import tempfile

from ..conf import Configuration
from ..master.process import AlluxioMasterProcess
from ..worker.process import AlluxioWorkerProcess

DEFAULTS = {
    "alluxio.master.journal.type": "UFS",
    "alluxio.worker.tieredstore.levels": "1",
    "alluxio.worker.tieredstore.level0.alias": "MEM",
    "alluxio.worker.tieredstore.level0.dirs.path": "auto",
    "alluxio.worker.tieredstore.level0.dirs.quota": "256MB",
    "alluxio.worker.hbm.page.size": "1MB",
    "alluxio.user.block.size.bytes.default": "16MB",
    "alluxio.master.worker.connect.wait.time": "0sec",
    "alluxio.security.authorization.permission.enabled": "false",
    "alluxio.user.file.writetype.default": "CACHE_THROUGH",
    "alluxio.worker.network.async.cache.manager.threads.max": "4",
    "alluxio.master.web.port": "0",
    "alluxio.worker.web.port": "0",
    "alluxio.master.web.bind.host": "127.0.0.1",
    "alluxio.worker.web.bind.host": "127.0.0.1",
}


class LocalAlluxioCluster:
    def __init__(self, num_workers: int = 1, conf: dict | None = None, work_dir: str | None = None,
                 grpc: bool = True, heartbeats: bool = False, devices: list[int] | None = None):
        self.work_dir = work_dir or tempfile.mkdtemp(prefix="alluxio_amd_")
        self._own_dir = work_dir is None
        props = dict(DEFAULTS)
        props["alluxio.work.dir"] = self.work_dir
        props["alluxio.home"] = self.work_dir
        props["alluxio.master.journal.folder"] = os.path.join(self.work_dir, "journal")
        props["alluxio.master.mount.table.root.ufs"] = os.path.join(self.work_dir, "underFSStorage")
        props.update(conf or {})
        self.conf = Configuration(props)
        self.num_workers = num_workers
        self.grpc = grpc
        self.heartbeats = heartbeats
        self.devices = devices
        self.master: AlluxioMasterProcess | None = None
        self.workers: list[AlluxioWorkerProcess] = []

    @property
    def ufs_root(self) -> str:
        return self.conf.get("alluxio.master.mount.table.root.ufs")

    def start(self) -> "LocalAlluxioCluster":
        os.makedirs(self.ufs_root, exist_ok=True)
        self.master = AlluxioMasterProcess(self.conf, port=0, enable_grpc=self.grpc, root_ufs=self.ufs_root)
        self.master.start(start_heartbeats=self.heartbeats)
        for i in range(self.num_workers):
            self.start_worker(i)
        return self

    def start_worker(self, i: int | None = None) -> AlluxioWorkerProcess:
        i = len(self.workers) if i is None else i
        dev = None
        if self.devices:
            dev = self.devices[i % len(self.devices)]
        wconf = self.conf.copy()
        w = AlluxioWorkerProcess(wconf, master_address=self.master.address, port=0, device=dev,
                                 enable_grpc=self.grpc, work_dir=os.path.join(self.work_dir, f"worker{i}"))
        w.start(register=True, start_heartbeats=self.heartbeats)
        self.workers.append(w)
        return w

    def stop_worker(self, w: AlluxioWorkerProcess) -> None:
        w.stop()
        self.workers.remove(w)

    def client(self, **kw):
        from ..client.file_system import FileSystem
        return FileSystem(conf=self.conf.copy(), master_address=self.master.address, **kw)

    def restart_master(self) -> None:
        self.master.stop()
        self.master = AlluxioMasterProcess(self.conf, port=0, enable_grpc=self.grpc, root_ufs=self.ufs_root)
        self.master.start(start_heartbeats=self.heartbeats)
        for w in self.workers:
            from ..rpc import Channel
            w.master_channel = Channel(self.master.address)
            w.worker.master_channel = w.master_channel
            w.worker._block_master = None
            w.worker._fs_master = None
            w.sync.registered = False
            w.sync.register()

    def heartbeat_workers(self) -> None:
        for w in self.workers:
            w.sync.heartbeat()

    def drive_jobs(self) -> None:
        """One job-worker heartbeat per worker plus the master persistence checker (tests run
        without background heartbeat threads)."""
        for w in self.workers:
            if w.job_worker is not None:
                w.job_worker.heartbeat()
        self.master.persistence_checker()

    def run_job(self, cfg, timeout: float = 120.0):
        """Submit a job through the JobMasterClientService and drive it to completion."""
        from ..job import JobClient
        from ..rpc import Channel
        client = JobClient(Channel(self.master.address))
        return client.run_and_wait(cfg, timeout=timeout, on_poll=self.drive_jobs)

    def stop(self) -> None:
        for w in list(self.workers):
            w.stop()
        self.workers.clear()
        if self.master is not None:
            self.master.stop()
            self.master = None
        if self._own_dir:
            shutil.rmtree(self.work_dir, ignore_errors=True)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


class MultiMasterLocalAlluxioCluster(LocalAlluxioCluster):
    """N masters sharing one journal (FILE_LOCK election) + workers; masters can be killed and
    the standby takes over (reference minicluster/.../MultiMasterLocalAlluxioCluster.java)."""

    def __init__(self, num_masters: int = 2, num_workers: int = 1, conf: dict | None = None,
                 journal_type: str = "UFS", **kw):
        c = {"alluxio.user.rpc.retry.max.duration": "20sec"}
        if journal_type.upper() == "EMBEDDED":
            # every master keeps its own Raft log; short timeouts keep failover tests quick
            c.update({"alluxio.master.embedded.journal.election.timeout": "400ms",
                      "alluxio.master.embedded.journal.heartbeat.interval": "50ms"})
        else:
            c["alluxio.master.ha.primary.selector"] = "FILE_LOCK"
        c.update(conf or {})
        super().__init__(num_workers=num_workers, conf=c, **kw)
        self.journal_type = journal_type.upper()
        if self.journal_type == "EMBEDDED":
            self.conf.set("alluxio.master.journal.type", "EMBEDDED")
        self.num_masters = num_masters
        self.masters: list[AlluxioMasterProcess] = []
        self.master_confs: list = []

    def _embedded_confs(self) -> list:
        ports = []
        for _ in range(self.num_masters):
            if self.grpc:
                import socket
                with socket.socket() as so:
                    so.bind(("127.0.0.1", 0))
                    ports.append(so.getsockname()[1])
            else:
                from ..rpc import _alloc_local_port
                ports.append(_alloc_local_port())
        addrs = ",".join(f"127.0.0.1:{p}" for p in ports)
        confs = []
        for i, p in enumerate(ports):
            c = self.conf.copy()
            c.set("alluxio.master.journal.folder", os.path.join(self.work_dir, f"journal{i}"))
            c.set("alluxio.master.embedded.journal.port", str(p))
            c.set("alluxio.master.embedded.journal.addresses", addrs)
            confs.append(c)
        return confs

    def start_master(self, i: int) -> AlluxioMasterProcess:
        """(Re)start master ``i`` with its own configuration (embedded journal: same Raft id)."""
        m = AlluxioMasterProcess(self.master_confs[i], port=0, enable_grpc=self.grpc, root_ufs=self.ufs_root)
        m.start(start_heartbeats=self.heartbeats)
        if i < len(self.masters):
            self.masters[i] = m
        else:
            self.masters.append(m)
        return m

    @property
    def master_addresses(self) -> str:
        return ",".join(m.address for m in self.masters)

    def start(self) -> "MultiMasterLocalAlluxioCluster":
        import time
        os.makedirs(self.ufs_root, exist_ok=True)
        if self.journal_type == "EMBEDDED":
            self.master_confs = self._embedded_confs()
        else:
            self.master_confs = [self.conf] * self.num_masters
        for i in range(self.num_masters):
            self.start_master(i)
        deadline = time.time() + 30
        while self.primary() is None and time.time() < deadline:
            time.sleep(0.02)
        self.master = self.primary()
        for i in range(self.num_workers):
            self.start_worker(i)
        return self

    def primary(self):
        for m in self.masters:
            if m.primary and m.started:
                return m
        return None

    def wait_primary(self, timeout: float = 30.0):
        import time
        deadline = time.time() + timeout
        while time.time() < deadline:
            p = self.primary()
            if p is not None:
                self.master = p
                return p
            time.sleep(0.02)
        raise TimeoutError("no master gained primacy")

    def start_worker(self, i: int | None = None) -> AlluxioWorkerProcess:
        i = len(self.workers) if i is None else i
        wconf = self.conf.copy()
        w = AlluxioWorkerProcess(wconf, master_address=self.master_addresses, port=0,
                                 enable_grpc=self.grpc, work_dir=os.path.join(self.work_dir, f"worker{i}"))
        w.start(register=True, start_heartbeats=self.heartbeats)
        self.workers.append(w)
        return w

    def client(self, **kw):
        from ..client.file_system import FileSystem
        return FileSystem(conf=self.conf.copy(), master_address=self.master_addresses, **kw)

    def kill_primary(self, wait_new: float = 30.0):
        """Stop the primary; wait until a standby has been elected and is serving."""
        import time
        old = self.primary()
        old.stop()
        deadline = time.time() + wait_new
        while time.time() < deadline:
            p = self.primary()
            if p is not None and p is not old:
                self.master = p
                return p
            time.sleep(0.02)
        raise TimeoutError("no standby master gained primacy")

    def stop(self) -> None:
        for w in list(self.workers):
            w.stop()
        self.workers.clear()
        for m in self.masters:
            if m.started:
                m.stop()
        self.masters.clear()
        self.master = None
        if self._own_dir:
            shutil.rmtree(self.work_dir, ignore_errors=True)
