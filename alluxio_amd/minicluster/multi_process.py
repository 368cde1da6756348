"""Cluster of real OS processes (one per master / worker) for fault-injection tests.

Parity: minicluster/src/main/java/alluxio/multi/process/MultiProcessCluster.java (masters and
workers as separate JVMs, port coordination, per-process configuration, ``waitForAllNodesRegistered``,
``stopMaster`` / ``startMaster`` / ``stopWorker`` / ``startWorker``, ``formatJournal``, primary
discovery) and PortCoordination.  Each process here is ``python -m alluxio_amd master|worker`` with
its own ``ALLUXIO_CONF_DIR/alluxio-site.properties``; masters run the embedded (Raft) journal so a
killed primary fails over to another process.
"""
from __future__ import annotations

import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time


def _free_port() -> int:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


class MultiProcessCluster:
    def __init__(self, num_masters: int = 1, num_workers: int = 1, conf: dict | None = None,
                 work_dir: str | None = None, journal_type: str = "EMBEDDED"):
        self.num_masters, self.num_workers = num_masters, num_workers
        self._own = work_dir is None
        self.work_dir = work_dir or tempfile.mkdtemp(prefix="amd-mpc-")
        self.ufs_root = os.path.join(self.work_dir, "ufs")
        self.master_ports = [_free_port() for _ in range(num_masters)]
        self.journal_ports = [_free_port() for _ in range(num_masters)]
        self.worker_ports = [_free_port() for _ in range(num_workers)]
        self.master_addresses = ",".join(f"127.0.0.1:{p}" for p in self.master_ports)
        base = {
            "alluxio.master.hostname": "127.0.0.1",
            "alluxio.master.rpc.addresses": self.master_addresses,
            "alluxio.master.mount.table.root.ufs": self.ufs_root,
            "alluxio.master.journal.type": journal_type,
            "alluxio.master.embedded.journal.addresses": ",".join(f"127.0.0.1:{p}" for p in self.journal_ports),
            "alluxio.master.embedded.journal.election.timeout": "1s",
            "alluxio.master.embedded.journal.heartbeat.interval": "100ms",
            "alluxio.master.web.port": "0",
            "alluxio.worker.web.port": "0",
            "alluxio.worker.tieredstore.levels": "1",
            "alluxio.worker.tieredstore.level0.alias": "MEM",
            "alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": "256MB",
            "alluxio.worker.hbm.page.size": "1MB",
            "alluxio.user.block.size.bytes.default": "16MB",
            "alluxio.master.worker.connect.wait.time": "0sec",
            "alluxio.security.authorization.permission.enabled": "false",
            "alluxio.user.rpc.retry.max.duration": "30sec",
            "alluxio.worker.block.heartbeat.interval": "200ms",
            "alluxio.job.worker.enabled": "false",
        }
        base.update(conf or {})
        self.base_conf = base
        self.masters: dict[int, subprocess.Popen] = {}
        self.workers: dict[int, subprocess.Popen] = {}

    # ---- configuration -----------------------------------------------------------------------
    def _conf_dir(self, role: str, i: int, extra: dict) -> str:
        d = os.path.join(self.work_dir, f"{role}{i}")
        cdir = os.path.join(d, "conf")
        os.makedirs(cdir, exist_ok=True)
        props = dict(self.base_conf)
        props["alluxio.work.dir"] = d
        props.update(extra)
        with open(os.path.join(cdir, "alluxio-site.properties"), "w") as f:
            for k, v in sorted(props.items()):
                f.write(f"{k}={v}\n")
        return cdir

    def _spawn(self, role: str, i: int, args: list[str], extra: dict) -> subprocess.Popen:
        cdir = self._conf_dir(role, i, extra)
        env = dict(os.environ)
        env["ALLUXIO_CONF_DIR"] = cdir
        env.pop("ALLUXIO_OPTS", None)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
        log = open(os.path.join(self.work_dir, f"{role}{i}.log"), "ab")
        return subprocess.Popen([sys.executable, "-m", "alluxio_amd", role] + args, env=env, stdout=log,
                                stderr=subprocess.STDOUT, cwd=self.work_dir, start_new_session=True)

    # ---- lifecycle ---------------------------------------------------------------------------
    def start(self) -> "MultiProcessCluster":
        os.makedirs(self.ufs_root, exist_ok=True)
        for i in range(self.num_masters):
            self.start_master(i)
        self.wait_for_primary()
        for j in range(self.num_workers):
            self.start_worker(j)
        self.wait_for_workers(self.num_workers)
        return self

    def start_master(self, i: int) -> None:
        extra = {"alluxio.master.rpc.port": str(self.master_ports[i]),
                 "alluxio.master.embedded.journal.port": str(self.journal_ports[i]),
                 "alluxio.master.journal.folder": os.path.join(self.work_dir, f"master{i}", "journal")}
        self.masters[i] = self._spawn("master", i, ["--host", "127.0.0.1", "--port", str(self.master_ports[i]),
                                                    "--root-ufs", self.ufs_root], extra)

    def start_worker(self, j: int) -> None:
        extra = {"alluxio.worker.rpc.port": str(self.worker_ports[j])}
        self.workers[j] = self._spawn("worker", j, ["--master", self.master_addresses, "--host", "127.0.0.1",
                                                    "--port", str(self.worker_ports[j])], extra)

    def _kill(self, p: subprocess.Popen | None, sig=signal.SIGKILL) -> None:
        if p is None or p.poll() is not None:
            return
        try:
            os.killpg(p.pid, sig)        # the process group this cluster created for it
        except ProcessLookupError:
            return
        try:
            p.wait(timeout=15)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait(timeout=15)

    def stop_master(self, i: int) -> None:
        self._kill(self.masters.pop(i, None))

    def stop_worker(self, j: int) -> None:
        self._kill(self.workers.pop(j, None))

    def stop(self) -> None:
        for j in list(self.workers):
            self.stop_worker(j)
        for i in list(self.masters):
            self.stop_master(i)
        if self._own:
            shutil.rmtree(self.work_dir, ignore_errors=True)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # ---- discovery ---------------------------------------------------------------------------
    def client_conf(self):
        from ..conf import Configuration
        c = Configuration({"alluxio.master.rpc.addresses": self.master_addresses,
                           "alluxio.user.rpc.retry.max.duration": "30sec",
                           "alluxio.user.network.inprocess.transport.enabled": "false"})
        return c

    def client(self):
        from ..client.file_system import FileSystem
        return FileSystem(conf=self.client_conf(), master_address=self.master_addresses)

    def primary_index(self) -> int | None:
        from ..proto import pb
        from ..rpc import Channel
        for i, p in enumerate(self.master_ports):
            if i not in self.masters or self.masters[i].poll() is not None:
                continue
            ch = Channel(f"127.0.0.1:{p}", force_grpc=True)
            try:
                ch.stub("alluxio.grpc.meta.MetaMasterClientService").GetMasterInfo(
                    pb.meta.GetMasterInfoPOptions(), timeout=2)
                return i
            except Exception:  # noqa: BLE001 - standby (UNAVAILABLE) or not up yet
                continue
            finally:
                ch.close()
        return None

    def wait_for_primary(self, timeout: float = 90.0) -> int:
        end = time.time() + timeout
        while time.time() < end:
            i = self.primary_index()
            if i is not None:
                return i
            for i, p in self.masters.items():
                if p.poll() is not None:
                    raise RuntimeError(f"master{i} exited with {p.returncode}; see {self.work_dir}/master{i}.log")
            time.sleep(0.2)
        raise TimeoutError(f"no primary master within {timeout}s (logs under {self.work_dir})")

    def wait_for_workers(self, n: int, timeout: float = 90.0) -> None:
        from ..proto import pb
        end = time.time() + timeout
        while time.time() < end:
            i = self.primary_index()
            if i is not None:
                from ..rpc import Channel
                ch = Channel(f"127.0.0.1:{self.master_ports[i]}", force_grpc=True)
                try:
                    infos = ch.stub("alluxio.grpc.block.BlockMasterClientService").GetWorkerInfoList(
                        pb.block.GetWorkerInfoListPOptions(), timeout=2).workerInfos
                    if len(infos) >= n:
                        return
                except Exception:  # noqa: BLE001
                    pass
                finally:
                    ch.close()
            time.sleep(0.2)
        raise TimeoutError(f"{n} workers did not register within {timeout}s (logs under {self.work_dir})")
