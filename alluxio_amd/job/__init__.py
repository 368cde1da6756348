"""Job service: distributed load / persist / replicate / evict / move / migrate / stress plans.

``JobClient`` wraps JobMasterClientService (reference job/client/.../JobGrpcClientUtils.run:
submit + poll until done)."""
from __future__ import annotations

import json
import time

from ..proto import enum_name, pb
from .plans import (CompositeConfig, EvictConfig, JobConfig, LoadConfig, MigrateConfig, MoveConfig,  # noqa: F401
                    PersistConfig, ReplicateConfig, StressBenchConfig, TransformConfig)

SVC_JOB_CLIENT = "alluxio.grpc.job.JobMasterClientService"
SVC_JOB_WORKER = "alluxio.grpc.job.JobMasterWorkerService"


class JobClient:
    def __init__(self, channel):
        self.stub = channel.stub(SVC_JOB_CLIENT)

    def run(self, cfg: JobConfig) -> int:
        return self.stub.Run(pb.job.RunPRequest(jobConfig=cfg.to_bytes())).jobId

    def status(self, job_id: int, detailed: bool = False):
        if detailed:
            return self.stub.GetJobStatusDetailed(pb.job.GetJobStatusDetailedPRequest(jobId=job_id)).jobInfo
        return self.stub.GetJobStatus(pb.job.GetJobStatusPRequest(jobId=job_id)).jobInfo

    def cancel(self, job_id: int) -> None:
        self.stub.Cancel(pb.job.CancelPRequest(jobId=job_id))

    def list(self):
        return list(self.stub.ListAll(pb.job.ListAllPRequest()).jobInfos)

    def summary(self):
        return self.stub.GetJobServiceSummary(pb.job.GetJobServiceSummaryPRequest()).summary

    def worker_health(self):
        return list(self.stub.GetAllWorkerHealth(pb.job.GetAllWorkerHealthPRequest()).workerHealths)

    def wait(self, job_id: int, timeout: float = 600.0, poll: float = 0.05, on_poll=None):
        deadline = time.time() + timeout
        while True:
            info = self.status(job_id)
            st = enum_name(pb.job.Status, info.status)
            if st in ("COMPLETED", "FAILED", "CANCELED"):
                return info
            if time.time() > deadline:
                raise TimeoutError(f"job {job_id} still {st}")
            if on_poll is not None:
                on_poll()
            time.sleep(poll)

    def run_and_wait(self, cfg: JobConfig, timeout: float = 600.0, on_poll=None):
        info = self.wait(self.run(cfg), timeout, on_poll=on_poll)
        result = json.loads(info.result.decode()) if info.result else None
        return enum_name(pb.job.Status, info.status), result, info.errorMessage
