"""HTTP endpoints of the master and worker processes.

Parity: core/server/common/src/main/java/alluxio/metrics/sink/MetricsServlet.java:35
(``/metrics/json``), PrometheusMetricsServlet.java:30 (``/metrics/prometheus``),
core/server/master/.../meta/AlluxioMasterRestServiceHandler.java (``/api/v1/master/*``:
get_info, get_configuration, get_metrics, get_capacity_bytes, get_used_bytes, get_ufs_*,
get_worker_count, get_block_master_info) and core/server/worker/.../AlluxioWorkerRestServiceHandler.java
(``/api/v1/worker/*``), plus ``/api/v1/*/log_level`` used by ``alluxio logLevel``.  Served by a
small threaded stdlib HTTP server so the processes carry no web-framework dependency.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

LOG = logging.getLogger(__name__)


class WebServer:
    """Routes: {(method, path): fn(query: dict, body: bytes) -> (status, content_type, body)}."""

    def __init__(self, host: str, port: int, routes: dict, name: str = "web"):
        self.routes = dict(routes)
        self.name = name
        outer = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, fmt, *args):  # noqa: D401 - silence default stderr logging
                LOG.debug("%s %s", outer.name, fmt % args)

            def _serve(self, method):
                u = urlparse(self.path)
                fn = outer.routes.get((method, u.path.rstrip("/") or "/"))
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else b""
                if fn is None:
                    status, ctype, out = 404, "application/json", json.dumps({"error": f"no route {u.path}"})
                else:
                    try:
                        status, ctype, out = fn({k: v[-1] for k, v in parse_qs(u.query).items()}, body)
                    except Exception as e:  # noqa: BLE001
                        LOG.exception("web handler failed")
                        status, ctype, out = 500, "application/json", json.dumps({"error": str(e)})
                data = out.encode() if isinstance(out, str) else out
                self.send_response(status)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                self._serve("GET")

            def do_POST(self):
                self._serve("POST")

        try:
            self.httpd = ThreadingHTTPServer((host, port), Handler)
        except OSError as e:  # port taken (e.g. several workers on one node): use an ephemeral one
            LOG.warning("%s web port %d unavailable (%s); binding an ephemeral port", name, port, e)
            self.httpd = ThreadingHTTPServer((host, 0), Handler)
        self.httpd.daemon_threads = True
        self._t = None

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    def start(self) -> int:
        self._t = threading.Thread(target=self.httpd.serve_forever, kwargs={"poll_interval": 0.05},
                                   name=f"{self.name}-http", daemon=True)
        self._t.start()
        return self.port

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()


def _json(obj, status=200):
    return status, "application/json", json.dumps(obj, default=str, sort_keys=True)


def log_level_route(query, body):
    name = query.get("logName", "")
    lg = logging.getLogger(name or None)
    if query.get("level"):
        lg.setLevel(query["level"].upper())
    return _json({"logName": name, "level": logging.getLevelName(lg.getEffectiveLevel())})


def metrics_routes(metrics_system) -> dict:
    return {
        ("GET", "/metrics/json"): lambda q, b: (200, "application/json", metrics_system.to_json()),
        ("GET", "/metrics/prometheus"): lambda q, b: (200, "text/plain; version=0.0.4",
                                                      metrics_system.to_prometheus()),
    }


def master_routes(master) -> dict:
    from ..proto import pb
    from ..utils.format import bytes_to_human

    def info(q, b):
        bm = master.block_master
        cap, used = bm.capacity_bytes(), bm.used_bytes()
        mounts = {mp: {"ufsUri": i.ufsUri, "readOnly": i.readOnly, "shared": i.shared}
                  for mp, i in master.fs_master.get_mount_table().items()}
        workers = [{"id": w.id, "address": f"{w.address.host}:{w.address.rpcPort}", "capacityBytes": w.capacityBytes,
                    "usedBytes": w.usedBytes, "state": w.state} for w in bm.worker_info_list()]
        from .. import __version__
        return _json({"version": __version__, "startTimeMs": int(master.start_time * 1000),
                      "uptimeMs": int((time.time() - master.start_time) * 1000),
                      "rpcAddress": master.address, "safeMode": master.safe_mode.in_safe_mode(),
                      "capacity": {"total": cap, "used": used, "totalHuman": bytes_to_human(cap)},
                      "workers": workers, "mountPoints": mounts, "primary": master.primary,
                      "journalSequenceNumbers": master.journal.sequence_numbers()})

    def conf(q, b):
        return _json({k: v for k, v in master.conf.to_map(include_defaults=q.get("all") == "true").items()})

    def metrics(q, b):
        return _json(master.metrics_master.get_metrics())

    def jobs(q, b):
        jm = master.job_master
        if jm is None:
            return _json({"jobs": []})
        return _json({"jobs": [{"id": j.id, "name": j.cfg.type_name, "status": j.status, "error": j.error}
                               for j in list(jm.jobs.values())]})

    r = metrics_routes(master.metrics)
    r.update({
        ("GET", "/api/v1/master/get_info"): info,
        ("GET", "/api/v1/master/get_configuration"): conf,
        ("GET", "/api/v1/master/get_metrics"): metrics,
        ("GET", "/api/v1/master/get_jobs"): jobs,
        ("GET", "/api/v1/master/log_level"): log_level_route,
        ("POST", "/api/v1/master/log_level"): log_level_route,
        ("POST", "/api/v1/logLevel"): log_level_route,
        ("GET", "/api/v1/master/ping"): lambda q, b: _json({"ok": True}),
    })
    from .ui import master_ui_routes
    from .webui_api import master_webui_routes, static_routes
    r.update(master_ui_routes(master))
    r.update(master_webui_routes(master))
    r.update(static_routes("master"))
    del pb
    return r


def worker_routes(wp) -> dict:
    def info(q, b):
        w = wp.worker
        store = wp.store
        dirs = []
        for i, d in enumerate(store.dirs):
            dirs.append({"tier": d.tier, "alias": d.alias, "medium": d.medium, "path": d.path,
                         "capacity": w.native.dir_capacity(i), "available": w.native.dir_available(i),
                         "healthy": w.native.dir_healthy(i)})
        plane = w.transfer_plane
        return _json({"address": wp.address, "workerId": w.worker_id, "device": store.device,
                      "capacityByTier": store.capacity_by_tier(), "usedByTier": store.used_by_tier(),
                      "blocks": len(w.native.block_ids(-1)), "dirs": dirs,
                      "transferPlane": None if plane is None else {"rank": plane.rank, "world": plane.world,
                                                                   "bytesPulled": plane.bytes_pulled,
                                                                   "bytesGathered": plane.bytes_gathered}})

    r = metrics_routes(wp.worker.metrics)
    r.update({
        ("GET", "/api/v1/worker/get_info"): info,
        ("GET", "/api/v1/worker/log_level"): log_level_route,
        ("POST", "/api/v1/worker/log_level"): log_level_route,
        ("POST", "/api/v1/logLevel"): log_level_route,
    })
    from .ui import worker_ui_routes
    from .webui_api import static_routes, worker_webui_routes
    r.update(worker_ui_routes(wp))
    r.update(worker_webui_routes(wp))
    r.update(static_routes("worker"))
    return r
