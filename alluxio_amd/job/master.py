"""Job master and job worker.

Parity: job/server/src/main/java/alluxio/master/job/JobMaster.java (run/cancel/status/list,
job-worker registry + lost-worker detection), plan/PlanCoordinator.java + PlanTracker.java
(selectExecutors -> per-worker RunTaskCommands, task status aggregation, join),
workflow/WorkflowTracker.java (composite sequential/parallel jobs), command/CommandManager.java
(commands delivered on heartbeat); job/server/.../worker/JobWorker.java,
worker/job/command/CommandHandlingExecutor.java (heartbeat loop), task/TaskExecutorManager.java
(pausable task pool, task status reported back).
"""
from __future__ import annotations

import itertools
import json
import logging
import os
import threading
import time
import traceback
from concurrent.futures import ThreadPoolExecutor

from ..proto import enum_name, pb
from ..utils import exceptions as ex
from .plans import CompositeConfig, JobConfig, RunTaskContext

LOG = logging.getLogger(__name__)

CREATED, CANCELED, FAILED, RUNNING, COMPLETED = "CREATED", "CANCELED", "FAILED", "RUNNING", "COMPLETED"
_STATUS_NUM = {"UNKNOWN": 0, CREATED: 1, CANCELED: 2, FAILED: 3, RUNNING: 4, COMPLETED: 5}


class JobWorkerInfo:
    def __init__(self, wid, address, block_worker_port):
        self.id = wid
        self.address = address
        self.block_worker_port = block_worker_port
        self.last_heartbeat = time.time()
        self.health = None
        self.pending: list = []   # JobCommand protos to deliver


class TaskInfo:
    def __init__(self, job_id, task_id, worker_id, args):
        self.job_id, self.task_id, self.worker_id, self.args = job_id, task_id, worker_id, args
        self.status = CREATED
        self.result = None
        self.error = ""


class PlanInfo:
    def __init__(self, job_id, cfg: JobConfig, parent_id: int = 0):
        self.id = job_id
        self.cfg = cfg
        self.parent_id = parent_id
        self.status = CREATED
        self.error = ""
        self.result = None
        self.tasks: dict[int, TaskInfo] = {}
        self.children: list[int] = []
        self.last_updated = time.time()
        self.done = threading.Event()

    def to_proto(self, detailed: bool = False, master=None):
        j = pb.job.JobInfo(id=self.id, name=self.cfg.type_name, status=_STATUS_NUM[self.status],
                           errorMessage=self.error, lastUpdated=int(self.last_updated * 1000),
                           type=3 if isinstance(self.cfg, CompositeConfig) else 1, parentId=self.parent_id,
                           description=json.dumps(json.loads(self.cfg.to_bytes()))[:512])
        if self.result is not None:
            j.result = json.dumps(self.result, default=str).encode()
        if detailed:
            for t in self.tasks.values():
                j.children.append(pb.job.JobInfo(id=t.task_id, parentId=self.id, status=_STATUS_NUM[t.status],
                                                 errorMessage=t.error, type=2))
            if master is not None:
                for c in self.children:
                    ci = master.jobs.get(c)
                    if ci is not None:
                        j.children.append(ci.to_proto(False))
        return j


class JobMaster:
    def __init__(self, fs_factory, worker_timeout_s: float = 60.0, capacity: int = 100_000):
        self.fs_factory = fs_factory  # -> client FileSystem (for selectExecutors)
        self.jobs: dict[int, PlanInfo] = {}
        self.workers: dict[int, JobWorkerInfo] = {}
        self._ids = itertools.count(int(time.time() * 1000) % 1_000_000 * 1000)
        self._wids = itertools.count(1)
        self._lock = threading.RLock()
        self.worker_timeout = worker_timeout_s
        self.capacity = capacity
        self._fs = None

    def _client(self):
        if self._fs is None:
            self._fs = self.fs_factory()
        return self._fs

    # ---- workers ------------------------------------------------------------------------------
    def register_worker(self, address, block_worker_port: int = 0) -> int:
        with self._lock:
            for w in self.workers.values():
                if w.address.host == address.host and w.address.rpcPort == address.rpcPort:
                    w.last_heartbeat = time.time()
                    return w.id
            wid = next(self._wids)
            self.workers[wid] = JobWorkerInfo(wid, address, block_worker_port or address.rpcPort)
            return wid

    def heartbeat(self, worker_id: int, health, task_infos) -> list:
        with self._lock:
            w = self.workers.get(worker_id)
            if w is None:
                return [pb.job.JobCommand(registerCommand=pb.job.RegisterCommand())]
            w.last_heartbeat = time.time()
            w.health = health
            cmds, w.pending = w.pending, []
        for ti in task_infos:
            self._update_task(ti)
        return cmds

    def detect_lost_workers(self) -> list[int]:
        now = time.time()
        lost = []
        with self._lock:
            for wid, w in list(self.workers.items()):
                if now - w.last_heartbeat > self.worker_timeout:
                    lost.append(wid)
                    del self.workers[wid]
            for p in self.jobs.values():
                for t in p.tasks.values():
                    if t.worker_id in lost and t.status in (CREATED, RUNNING):
                        t.status = FAILED
                        t.error = "job worker lost"
        for p in list(self.jobs.values()):
            self._maybe_finish(p)
        return lost

    # ---- jobs ---------------------------------------------------------------------------------
    def run(self, cfg: JobConfig, parent_id: int = 0) -> int:
        with self._lock:
            if sum(1 for j in self.jobs.values() if j.status in (CREATED, RUNNING)) >= self.capacity:
                raise ex.ResourceExhaustedException("job master at capacity")
            jid = next(self._ids)
            info = PlanInfo(jid, cfg, parent_id)
            self.jobs[jid] = info
        if isinstance(cfg, CompositeConfig):
            threading.Thread(target=self._run_workflow, args=(info,), daemon=True).start()
            return jid
        try:
            defn = cfg.definition()
            with self._lock:
                workers = list(self.workers.values())
            assignments = defn.select_executors(cfg, workers, self._client())
        except Exception as e:  # noqa: BLE001
            info.status = FAILED
            info.error = f"{type(e).__name__}: {e}"
            info.done.set()
            return jid
        with self._lock:
            info.status = RUNNING
            for i, (w, args) in enumerate(assignments):
                ti = TaskInfo(jid, i, w.id, args)
                info.tasks[i] = ti
                w.pending.append(pb.job.JobCommand(runTaskCommand=pb.job.RunTaskCommand(
                    jobId=jid, taskId=i, jobConfig=cfg.to_bytes(), taskArgs=json.dumps(args).encode())))
        self._maybe_finish(info)
        return jid

    def _run_workflow(self, info: PlanInfo) -> None:
        info.status = RUNNING
        try:
            if info.cfg.sequential:
                for c in info.cfg.jobs:
                    cid = self.run(c, parent_id=info.id)
                    info.children.append(cid)
                    child = self.wait(cid)
                    if child.status != COMPLETED:
                        raise RuntimeError(f"child job {cid} {child.status}: {child.error}")
            else:
                ids_ = [self.run(c, parent_id=info.id) for c in info.cfg.jobs]
                info.children.extend(ids_)
                for cid in ids_:
                    child = self.wait(cid)
                    if child.status != COMPLETED:
                        raise RuntimeError(f"child job {cid} {child.status}: {child.error}")
            info.status = COMPLETED
        except Exception as e:  # noqa: BLE001
            info.status = FAILED
            info.error = str(e)
        info.last_updated = time.time()
        info.done.set()

    def _update_task(self, ti) -> None:
        with self._lock:
            p = self.jobs.get(ti.parentId)
            if p is None:
                return
            t = p.tasks.get(ti.id)
            if t is None or t.status in (COMPLETED, FAILED, CANCELED):
                return
            t.status = enum_name(pb.job.Status, ti.status)
            t.error = ti.errorMessage
            if ti.result:
                t.result = json.loads(ti.result.decode())
        self._maybe_finish(p)

    def _maybe_finish(self, p: PlanInfo) -> None:
        with self._lock:
            if p.status not in (RUNNING,) or isinstance(p.cfg, CompositeConfig):
                return
            states = [t.status for t in p.tasks.values()]
            if any(s == FAILED for s in states):
                p.status = FAILED
                p.error = next(t.error for t in p.tasks.values() if t.status == FAILED)
                for t in p.tasks.values():
                    if t.status in (CREATED, RUNNING):
                        self._cancel_task(t)
            elif all(s == COMPLETED for s in states):
                try:
                    p.result = p.cfg.definition().join(p.cfg, {t.task_id: t.result for t in p.tasks.values()})
                    p.status = COMPLETED
                except Exception as e:  # noqa: BLE001
                    p.status = FAILED
                    p.error = str(e)
            else:
                return
            p.last_updated = time.time()
            p.done.set()

    def _cancel_task(self, t: TaskInfo) -> None:
        w = self.workers.get(t.worker_id)
        if w is not None:
            w.pending.append(pb.job.JobCommand(cancelTaskCommand=pb.job.CancelTaskCommand(
                jobId=t.job_id, taskId=t.task_id)))
        t.status = CANCELED

    def cancel(self, job_id: int) -> None:
        with self._lock:
            p = self.jobs.get(job_id)
            if p is None:
                raise ex.NotFoundException(f"job {job_id} not found")
            if p.status in (COMPLETED, FAILED, CANCELED):
                return
            for t in p.tasks.values():
                if t.status in (CREATED, RUNNING):
                    self._cancel_task(t)
            for c in p.children:
                try:
                    self.cancel(c)
                except ex.NotFoundException:
                    pass
            p.status = CANCELED
            p.last_updated = time.time()
            p.done.set()

    def status(self, job_id: int) -> PlanInfo:
        with self._lock:
            p = self.jobs.get(job_id)
        if p is None:
            raise ex.NotFoundException(f"job {job_id} not found")
        return p

    def wait(self, job_id: int, timeout: float | None = None) -> PlanInfo:
        p = self.status(job_id)
        p.done.wait(timeout)
        return p

    def purge_finished(self, retention_s: float) -> int:
        """Drop finished jobs older than the retention time (JobMaster finished-job purge)."""
        cutoff = time.time() - retention_s
        with self._lock:
            old = [j for j, p in self.jobs.items()
                   if p.status in (COMPLETED, FAILED, CANCELED) and p.last_updated < cutoff]
            for j in old:
                del self.jobs[j]
        return len(old)

    def summary(self):
        with self._lock:
            jobs = list(self.jobs.values())
        s = pb.job.JobServiceSummary()
        counts = {}
        for j in jobs:
            counts[j.status] = counts.get(j.status, 0) + 1
        for st, n in counts.items():
            s.summaryPerStatus.add(status=_STATUS_NUM[st], count=n)
        recent = sorted(jobs, key=lambda j: -j.last_updated)[:10]
        s.recentActivities.extend(j.to_proto() for j in recent)
        s.recentFailures.extend(j.to_proto() for j in recent if j.status == FAILED)
        return s


class JobMasterService:
    """JobMasterClientService + JobMasterWorkerService handlers."""

    def __init__(self, jm: JobMaster):
        self.jm = jm

    def Run(self, req, ctx):
        return pb.job.RunPResponse(jobId=self.jm.run(JobConfig.from_bytes(req.jobConfig)))

    def Cancel(self, req, ctx):
        self.jm.cancel(req.jobId)
        return pb.job.CancelPResponse()

    def GetJobStatus(self, req, ctx):
        return pb.job.GetJobStatusPResponse(jobInfo=self.jm.status(req.jobId).to_proto())

    def GetJobStatusDetailed(self, req, ctx):
        return pb.job.GetJobStatusDetailedPResponse(jobInfo=self.jm.status(req.jobId).to_proto(True, self.jm))

    def ListAll(self, req, ctx):
        jobs = list(self.jm.jobs.values())
        return pb.job.ListAllPResponse(jobIds=[j.id for j in jobs], jobInfos=[j.to_proto() for j in jobs])

    def GetJobServiceSummary(self, req, ctx):
        return pb.job.GetJobServiceSummaryPResponse(summary=self.jm.summary())

    def GetAllWorkerHealth(self, req, ctx):
        out = []
        for w in self.jm.workers.values():
            h = w.health or pb.job.JobWorkerHealth(workerId=w.id, hostname=w.address.host)
            out.append(h)
        return pb.job.GetAllWorkerHealthPResponse(workerHealths=out)

    def Heartbeat(self, req, ctx):
        cmds = self.jm.heartbeat(req.jobWorkerHealth.workerId, req.jobWorkerHealth, list(req.taskInfos))
        return pb.job.JobHeartbeatPResponse(commands=cmds)

    def RegisterJobWorker(self, req, ctx):
        return pb.job.RegisterJobWorkerPResponse(id=self.jm.register_worker(req.workerNetAddress))


class JobWorker:
    """Polls the job master, runs tasks in a pool, reports their status on the next heartbeat."""

    def __init__(self, channel, address, fs, block_worker=None, pool_size: int = 4):
        self.stub = channel.stub("alluxio.grpc.job.JobMasterWorkerService")
        self.address = address
        self.fs = fs
        self.block_worker = block_worker
        self.pool = ThreadPoolExecutor(max_workers=pool_size, thread_name_prefix="job-task")
        self.pool_size = pool_size
        self.id = None
        self._reports: list = []
        self._running: dict[tuple, object] = {}
        self._lock = threading.Lock()

    def register(self) -> int:
        self.id = self.stub.RegisterJobWorker(pb.job.RegisterJobWorkerPRequest(workerNetAddress=self.address)).id
        return self.id

    def heartbeat(self) -> None:
        if self.id is None:
            self.register()
        with self._lock:
            reports, self._reports = self._reports, []
            active = len(self._running)
        try:
            load = list(os.getloadavg())
        except OSError:
            load = []
        health = pb.job.JobWorkerHealth(workerId=self.id, hostname=self.address.host, loadAverage=load,
                                        lastUpdated=int(time.time() * 1000), taskPoolSize=self.pool_size,
                                        numActiveTasks=active)
        resp = self.stub.Heartbeat(pb.job.JobHeartbeatPRequest(jobWorkerHealth=health, taskInfos=reports))
        for cmd in resp.commands:
            if cmd.HasField("runTaskCommand"):
                self._submit(cmd.runTaskCommand)
            elif cmd.HasField("cancelTaskCommand"):
                c = cmd.cancelTaskCommand
                with self._lock:
                    f = self._running.pop((c.jobId, c.taskId), None)
                if f is not None:
                    f.cancel()
            elif cmd.HasField("registerCommand"):
                self.register()
            elif cmd.HasField("setTaskPoolSizeCommand"):
                self.pool_size = cmd.setTaskPoolSizeCommand.taskPoolSize

    def _submit(self, rt) -> None:
        cfg = JobConfig.from_bytes(rt.jobConfig)
        args = json.loads(rt.taskArgs.decode()) if rt.taskArgs else None

        def run():
            info = pb.job.JobInfo(id=rt.taskId, parentId=rt.jobId, type=2, workerHost=self.address.host)
            try:
                ctx = RunTaskContext(self.fs, self.block_worker, self.address, rt.jobId, rt.taskId)
                res = cfg.definition().run_task(cfg, args, ctx)
                info.status = _STATUS_NUM[COMPLETED]
                info.result = json.dumps(res, default=str).encode()
            except Exception as e:  # noqa: BLE001
                LOG.debug("task %d/%d failed: %s", rt.jobId, rt.taskId, traceback.format_exc())
                info.status = _STATUS_NUM[FAILED]
                info.errorMessage = f"{type(e).__name__}: {e}"
            with self._lock:
                self._running.pop((rt.jobId, rt.taskId), None)
                self._reports.append(info)
        with self._lock:
            self._running[(rt.jobId, rt.taskId)] = self.pool.submit(run)

    def drain(self, timeout: float = 60.0) -> None:
        """Run heartbeats until no task is running (tests / synchronous drivers)."""
        deadline = time.time() + timeout
        while time.time() < deadline:
            self.heartbeat()
            with self._lock:
                idle = not self._running and not self._reports
            if idle:
                return
            time.sleep(0.01)

    def close(self) -> None:
        self.pool.shutdown(wait=False, cancel_futures=True)
