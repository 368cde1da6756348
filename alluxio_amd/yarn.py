"""Run an Alluxio cluster on YARN: ``alluxio yarn submit|status|stop``.

Parity: integration/yarn/src/main/java/alluxio/yarn/{Client,ApplicationMaster,ContainerAllocator,
CommandBuilder}.java -- the client submits an application; the master runs in one container, the
workers in one container per node (``alluxio.integration.yarn.workers.per.host.max``), each with
memory / vcores from ``alluxio.integration.{master,worker}.resource.{mem,cpu}``; the application is
killed to stop the cluster.

The reference drives YARN through its Java client libraries and a custom ApplicationMaster speaking
the AMRM protocol.  No JVM is involved here: this client uses the ResourceManager REST API
(``/ws/v1/cluster/apps/new-application``, ``/ws/v1/cluster/apps``, ``/apps/{id}/state``) and
submits one YARN application per Alluxio process -- its AM container *is* the process
(``python -m alluxio_amd master|worker``) -- which gives the same placement controls (node label
expression, resource vector incl. ``yarn.io/gpu`` so an MI355X worker container owns exactly one
GPU) without a long-lived custom AM.  All applications of one cluster share an application tag
``alluxio-cluster:<name>`` so ``status`` / ``stop`` find them again.
"""
from __future__ import annotations

import argparse
import json
import shlex
import sys
import time

APP_TYPE = "ALLUXIO"


class YarnRestClient:
    def __init__(self, rm: str, user: str = "", timeout: float = 30.0):
        import requests
        self.rm = rm.rstrip("/")
        if "://" not in self.rm:
            self.rm = "http://" + self.rm
        self.user = user
        self.session = requests.Session()
        self.timeout = timeout

    def _req(self, method: str, path: str, body=None):
        params = {"user.name": self.user} if self.user else None
        r = self.session.request(method, self.rm + path, params=params, timeout=self.timeout,
                                 data=None if body is None else json.dumps(body),
                                 headers={"Content-Type": "application/json", "Accept": "application/json"})
        if r.status_code >= 300:
            raise RuntimeError(f"YARN RM {method} {path}: {r.status_code} {r.text[:300]}")
        return r.json() if r.content else {}

    def new_application(self) -> dict:
        return self._req("POST", "/ws/v1/cluster/apps/new-application")

    def submit(self, spec: dict) -> None:
        self._req("POST", "/ws/v1/cluster/apps", spec)

    def app(self, app_id: str) -> dict:
        return self._req("GET", f"/ws/v1/cluster/apps/{app_id}").get("app", {})

    def kill(self, app_id: str) -> None:
        self._req("PUT", f"/ws/v1/cluster/apps/{app_id}/state", {"state": "KILLED"})

    def apps(self, tag: str) -> list[dict]:
        r = self._req("GET", f"/ws/v1/cluster/apps?applicationTypes={APP_TYPE}&applicationTags={tag}")
        return ((r.get("apps") or {}).get("app")) or []


def _command(role: str, home: str, args: list[str], log_dir: str = "<LOG_DIR>") -> str:
    """The container's launch command (reference CommandBuilder): run the role in the
    foreground from the distribution, stdout/stderr into YARN's container log dir."""
    py = f"{home}/bin/alluxio" if home else "python3 -m alluxio_amd"
    argv = " ".join(shlex.quote(a) for a in args)
    return f"{py} {role} {argv} 1>{log_dir}/{role}.out 2>{log_dir}/{role}.err".replace("  ", " ")


def build_specs(name: str, num_workers: int, master_host: str, home: str = "", queue: str = "default",
                master_mem_mb: int = 4096, master_vcores: int = 2, worker_mem_mb: int = 16384,
                worker_vcores: int = 8, gpus_per_worker: int = 1, node_label: str = "",
                env: dict | None = None, conf: dict | None = None) -> list[dict]:
    """Application submission bodies for the master and ``num_workers`` workers (without ids)."""
    tag = f"alluxio-cluster:{name}"
    base_env = {"ALLUXIO_MASTER_HOSTNAME": master_host, "PYTHONUNBUFFERED": "1"}
    base_env.update(env or {})
    conf = dict(conf or {})
    conf.setdefault("alluxio.master.hostname", master_host)
    props = " ".join(f"-D{k}={v}" for k, v in sorted(conf.items()))

    def entry(role: str, idx: int, mem: int, vcores: int, gpus: int) -> dict:
        res = {"memory": mem, "vCores": vcores}
        if gpus:
            res["resourceInformations"] = {"resourceInformation": [
                {"name": "yarn.io/gpu", "value": gpus, "units": "", "resourceType": "COUNTABLE"}]}
        envs = dict(base_env, ALLUXIO_YARN_ROLE=role, ALLUXIO_YARN_INDEX=str(idx))
        envs["ALLUXIO_OPTS"] = props              # -Dkey=value overrides read by conf._load_env
        spec = {
            "application-name": f"{name}-{role}" + (f"-{idx}" if role == "worker" else ""),
            "application-type": APP_TYPE,
            "queue": queue,
            "application-tags": {"tag": [tag, f"alluxio-role:{role}"]},
            "max-app-attempts": 2 if role == "master" else 3,
            "keep-containers-across-application-attempts": False,
            "unmanaged-AM": False,
            "resource": res,
            "am-container-spec": {
                "commands": {"command": _command(role, home, [])},
                "environment": {"entry": [{"key": k, "value": v} for k, v in sorted(envs.items())]},
            },
        }
        if node_label:
            spec["am-container-node-label-expression"] = node_label
        return spec
    specs = [entry("master", 0, master_mem_mb, master_vcores, 0)]
    specs += [entry("worker", i, worker_mem_mb, worker_vcores, gpus_per_worker) for i in range(num_workers)]
    return specs


def submit(rm: YarnRestClient, specs: list[dict]) -> list[str]:
    ids = []
    for spec in specs:
        app_id = rm.new_application()["application-id"]
        rm.submit(dict(spec, **{"application-id": app_id}))
        ids.append(app_id)
    return ids


def wait_running(rm: YarnRestClient, ids: list[str], timeout: float = 300.0, poll: float = 1.0) -> dict:
    deadline = time.time() + timeout
    while True:
        states = {i: rm.app(i).get("state", "UNKNOWN") for i in ids}
        if all(s == "RUNNING" for s in states.values()):
            return states
        bad = {i: s for i, s in states.items() if s in ("FAILED", "KILLED", "FINISHED")}
        if bad or time.time() > deadline:
            return states
        time.sleep(poll)


def status(rm: YarnRestClient, name: str) -> list[dict]:
    return [{"id": a.get("id"), "name": a.get("name"), "state": a.get("state"),
             "host": a.get("amHostHttpAddress", "")} for a in rm.apps(f"alluxio-cluster:{name}")]


def stop(rm: YarnRestClient, name: str) -> int:
    n = 0
    for a in rm.apps(f"alluxio-cluster:{name}"):
        if a.get("state") not in ("FINISHED", "FAILED", "KILLED"):
            rm.kill(a["id"])
            n += 1
    return n


def main(argv=None, out=None) -> int:
    out = out or sys.stdout
    ap = argparse.ArgumentParser(prog="alluxio yarn")
    ap.add_argument("action", choices=["submit", "status", "stop"])
    ap.add_argument("--rm", required=True, help="ResourceManager web address, e.g. http://rm:8088")
    ap.add_argument("--name", default="alluxio")
    ap.add_argument("--user", default="")
    ap.add_argument("--num-workers", type=int, default=1)
    ap.add_argument("--master-host", default="")
    ap.add_argument("--home", default="", help="distribution directory on the nodes (tools/release.py)")
    ap.add_argument("--queue", default="default")
    ap.add_argument("--gpus-per-worker", type=int, default=1)
    ap.add_argument("--worker-mem-mb", type=int, default=16384)
    ap.add_argument("--node-label", default="")
    ap.add_argument("--wait", type=float, default=0.0, help="seconds to wait for RUNNING")
    ap.add_argument("-D", dest="props", action="append", default=[])
    a = ap.parse_args(argv)
    rm = YarnRestClient(a.rm, a.user)
    if a.action == "submit":
        if not a.master_host:
            ap.error("--master-host is required for submit")
        specs = build_specs(a.name, a.num_workers, a.master_host, a.home, a.queue, worker_mem_mb=a.worker_mem_mb,
                            gpus_per_worker=a.gpus_per_worker, node_label=a.node_label,
                            conf=dict(p.split("=", 1) for p in a.props))
        ids = submit(rm, specs)
        print(json.dumps({"applications": ids}), file=out)
        if a.wait:
            states = wait_running(rm, ids, a.wait)
            print(json.dumps({"states": states}), file=out)
            return 0 if all(s == "RUNNING" for s in states.values()) else 1
        return 0
    if a.action == "status":
        print(json.dumps(status(rm, a.name)), file=out)
        return 0
    print(json.dumps({"killed": stop(rm, a.name)}), file=out)
    return 0
