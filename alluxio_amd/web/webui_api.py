"""JSON endpoints behind the single-page web UI (``/webui``), shaped like the reference's.

Reference: core/server/master/src/main/java/alluxio/master/meta/AlluxioMasterRestServiceHandler.java
(``webui_init``, ``webui_overview``, ``webui_browse``, ``webui_data``, ``webui_logs``,
``webui_config``, ``webui_workers``, ``webui_metrics``, ``webui_mounttable``; response classes
core/common/src/main/java/alluxio/wire/MasterWebUI*.java, WorkerWebUI*.java, and
core/common/.../util/webui/UIFileInfo.java) and AlluxioWorkerRestServiceHandler.java.  The React app
of the reference (webui/master, webui/worker) renders these; here a dependency-free script
(``web/static/webui/app.js``) does, served by the same process.  Field names follow the
reference's JSON (camelCase of the Java fields) so that either front end can read them.
"""
from __future__ import annotations

import json
import os
import time

from ..utils.format import bytes_to_human


def _json(obj, status=200):
    return status, "application/json", json.dumps(obj, default=str, sort_keys=True)


def _date(ms) -> str:
    return time.strftime("%m-%d-%Y %H:%M:%S:000", time.localtime(ms / 1000)) if ms else ""


def _uptime(ms) -> str:
    s = int(ms // 1000)
    d, s = divmod(s, 86400)
    h, s = divmod(s, 3600)
    m, s = divmod(s, 60)
    return f"{d} day(s), {h} hour(s), {m} minute(s), and {s} second(s)"


def _pct(used, total) -> int:
    return int(round(100.0 * used / total)) if total else 0


def ui_file_info(i) -> dict:
    """UIFileInfo fields of one FileInfo message."""
    from ..utils.format import mode_to_string
    return {"id": i.fileId, "name": i.name, "absolutePath": i.path, "isDirectory": i.folder,
            "size": "" if i.folder else bytes_to_human(i.length),
            "blockSizeBytes": "" if i.folder else bytes_to_human(i.blockSizeBytes),
            "inAlluxio": i.inAlluxioPercentage == 100, "inAlluxioPercentage": i.inAlluxioPercentage,
            "pinned": i.pinned, "owner": i.owner, "group": i.group, "mode": mode_to_string(i.mode, i.folder),
            "persistenceState": i.persistenceState, "creationTime": _date(i.creationTimeMs),
            "modificationTime": _date(i.lastModificationTimeMs)}


def _node_info(w, state: str) -> dict:
    return {"host": w.address.host, "rpcPort": w.address.rpcPort, "workerId": w.id, "state": state,
            "lastContactSec": int(w.lastContactSec), "capacity": bytes_to_human(w.capacityBytes),
            "usedMemory": bytes_to_human(w.usedBytes), "freeSpacePercent": 100 - _pct(w.usedBytes, w.capacityBytes),
            "usedSpacePercent": _pct(w.usedBytes, w.capacityBytes),
            "uptimeClockTime": _uptime(max(0, time.time() * 1000 - getattr(w, "startTimeMs", 0)))
            if getattr(w, "startTimeMs", 0) else ""}


def master_webui_routes(master) -> dict:
    from .. import __version__
    from ..security import as_user

    conf = master.conf

    def superuser():
        return as_user(master.fs_master.permission.superuser)

    def init(q, b):
        return _json({"debug": conf.get_bool("alluxio.debug", "false"), "newerVersionAvailable": False,
                      "webFileInfoEnabled": conf.get_bool("alluxio.web.file.info.enabled", "true"),
                      "securityAuthorizationPermissionEnabled":
                          conf.get_bool("alluxio.security.authorization.permission.enabled", "true"),
                      "workerPort": conf.get_int("alluxio.worker.web.port", "30000"),
                      "refreshInterval": conf.get_int("alluxio.web.refresh.interval.ms", "15000")
                      if conf.get_raw("alluxio.web.refresh.interval.ms") else 15000})

    def overview(q, b):
        bm = master.block_master
        cap, used = bm.capacity_bytes(), bm.used_bytes()
        tiers: dict = {}
        for w in bm.worker_info_list():
            for t, c in w.capacityBytesOnTiers.items():
                tiers.setdefault(t, [0, 0])[0] += c
            for t, u in w.usedBytesOnTiers.items():
                tiers.setdefault(t, [0, 0])[1] += u
        infos = [{"storageTierAlias": t, "capacity": bytes_to_human(c), "usedCapacity": bytes_to_human(u),
                  "freeCapacity": bytes_to_human(max(0, c - u)), "usedSpacePercent": _pct(u, c),
                  "freeSpacePercent": 100 - _pct(u, c)} for t, (c, u) in sorted(tiers.items())]
        st = os.statvfs(conf.get("alluxio.master.journal.folder", "/") if os.path.isdir(
            conf.get("alluxio.master.journal.folder", "/")) else "/")
        disk_total, disk_free = st.f_blocks * st.f_frsize, st.f_bavail * st.f_frsize
        return _json({"debug": False, "masterNodeAddress": master.address, "version": __version__,
                      "startTime": _date(master.start_time * 1000),
                      "uptime": _uptime((time.time() - master.start_time) * 1000),
                      "liveWorkerNodes": str(len(bm.worker_info_list())), "capacity": bytes_to_human(cap),
                      "usedCapacity": bytes_to_human(used), "freeCapacity": bytes_to_human(max(0, cap - used)),
                      "diskCapacity": bytes_to_human(disk_total), "diskUsedCapacity": bytes_to_human(disk_total - disk_free),
                      "diskFreeCapacity": bytes_to_human(disk_free), "storageTierInfos": infos,
                      "configCheckStatus": "PASSED", "configCheckErrors": {}, "configCheckWarns": {},
                      "configCheckErrorNum": 0, "configCheckWarnNum": 0,
                      "primary": master.primary, "safeMode": master.safe_mode.in_safe_mode()})

    def browse(q, b):
        path = q.get("path", "/") or "/"
        offset, limit = int(q.get("offset", 0) or 0), int(q.get("limit", 1000) or 1000)
        out = {"currentPath": path, "debug": False, "masterNodeAddress": master.address,
               "showPermissions": conf.get_bool("alluxio.security.authorization.permission.enabled", "true"),
               "fatalError": "", "fileDoesNotExistException": "", "invalidPathError": "", "fileInfos": [],
               "nTotalFile": 0, "pathInfos": [], "fileData": "", "viewingOffset": 0}
        try:
            with superuser():
                st = master.fs_master.get_status(path)
                infos = master.fs_master.list_status(path) if st.folder else []
        except Exception as e:  # noqa: BLE001 - reported in the page like the reference
            out["fileDoesNotExistException"] = str(e)
            return _json(out)
        acc, crumbs = "", []
        for part in [p for p in path.split("/") if p]:
            acc += "/" + part
            crumbs.append({"name": part, "absolutePath": acc})
        out["pathInfos"] = crumbs
        out["currentDirectory"] = ui_file_info(st)
        if st.folder:
            rows = sorted(infos, key=lambda x: (not x.folder, x.name))
            out["nTotalFile"] = len(rows)
            out["fileInfos"] = [ui_file_info(i) for i in rows[offset:offset + limit]]
        else:
            out["blockSizeBytes"] = bytes_to_human(st.blockSizeBytes)
            out["fileBlocks"] = [{"id": f.blockInfo.blockId, "blockLength": f.blockInfo.length,
                                  "locations": [f"{loc.workerAddress.host}:{loc.workerAddress.rpcPort}"
                                                for loc in f.blockInfo.locations]} for f in st.fileBlockInfos]
        return _json(out)

    def data(q, b):
        files = []
        with superuser():
            stack = ["/"]
            while stack and len(files) < 10000:
                p = stack.pop()
                for i in master.fs_master.list_status(p):
                    if i.folder:
                        stack.append(i.path)
                    elif i.inAlluxioPercentage == 100:
                        files.append(ui_file_info(i))
        files.sort(key=lambda f: f["absolutePath"])
        return _json({"showPermissions": True, "inAlluxioFileNum": len(files), "fileInfos": files[:1000],
                      "fatalError": "", "masterNodeAddress": master.address, "permissionError": ""})

    def workers(q, b):
        bm = master.block_master
        return _json({"debug": False, "normalNodeInfos": [_node_info(w, "In Service") for w in bm.worker_info_list()],
                      "failedNodeInfos": [_node_info(w, "Out of Service") for w in bm.lost_workers_info_list()]})

    def config(q, b):
        m = conf.to_map(include_defaults=True)
        src = getattr(conf, "source", None)
        rows = [[k, str(v), src(k) if src else ""] for k, v in sorted(m.items())]
        return _json({"configuration": rows, "whitelist": conf.get("alluxio.master.whitelist", "/").split(",")})

    def metrics(q, b):
        cluster = master.metrics_master.get_metrics()
        cap, used = master.block_master.capacity_bytes(), master.block_master.used_bytes()

        def pick(*names):
            return {n: cluster.get(n, 0) for n in names}
        return _json({"masterCapacityUsedPercentage": _pct(used, cap),
                      "masterCapacityFreePercentage": 100 - _pct(used, cap),
                      "operationMetrics": {k: v for k, v in sorted(cluster.items()) if k.startswith("Master.")},
                      "rpcInvocationMetrics": {k: v for k, v in sorted(master.metrics.registry.snapshot().items())},
                      "ufsOps": {k: v for k, v in sorted(cluster.items()) if "Ufs" in k},
                      "timeSeriesMetrics": master.time_series.store.series() if hasattr(master, "time_series") else [],
                      **pick("Cluster.BytesReadLocal", "Cluster.BytesReadRemote", "Cluster.BytesReadUfsAll",
                             "Cluster.BytesWrittenLocal", "Cluster.BytesWrittenUfsAll")})

    def mounttable(q, b):
        mt = master.fs_master.get_mount_table()
        return _json({"debug": False, "mountPointInfos": {
            mp: {"ufsUri": i.ufsUri, "ufsType": getattr(i, "ufsType", "") or i.ufsUri.split("://")[0],
                 "readOnly": i.readOnly, "shared": i.shared, "properties": dict(i.properties)}
            for mp, i in sorted(mt.items())}})

    def logs(q, b):
        d = conf.get("alluxio.logs.dir", "")
        files = sorted(os.listdir(d)) if d and os.path.isdir(d) else []
        name = q.get("path", "")
        out = {"currentPath": name, "fileInfos": [{"name": f, "absolutePath": f} for f in files], "fileData": "",
               "nTotalFile": len(files), "fatalError": "", "invalidPathError": ""}
        if name:
            p = os.path.join(d, os.path.basename(name))
            if os.path.isfile(p):
                off = int(q.get("offset", 0) or 0)
                with open(p, "rb") as f:
                    f.seek(max(0, off))
                    out["fileData"] = f.read(1 << 20).decode(errors="replace")
                out["viewingOffset"] = off
            else:
                out["invalidPathError"] = f"no log file {name}"
        return _json(out)

    pre = "/api/v1/master/"
    return {("GET", pre + "webui_init"): init, ("GET", pre + "webui_overview"): overview,
            ("GET", pre + "webui_browse"): browse, ("GET", pre + "webui_data"): data,
            ("GET", pre + "webui_workers"): workers, ("GET", pre + "webui_config"): config,
            ("GET", pre + "webui_metrics"): metrics, ("GET", pre + "webui_mounttable"): mounttable,
            ("GET", pre + "webui_logs"): logs}


def worker_webui_routes(wp) -> dict:
    from .. import __version__

    def init(q, b):
        return _json({"debug": False, "refreshInterval": 15000, "webFileInfoEnabled": True})

    def overview(q, b):
        w, store = wp.worker, wp.store
        cap, used = store.capacity_by_tier(), store.used_by_tier()
        dirs = [{"tierAlias": d.alias, "dirPath": d.path, "medium": d.medium,
                 "capacity": bytes_to_human(w.native.dir_capacity(i)),
                 "usedCapacity": bytes_to_human(w.native.dir_capacity(i) - w.native.dir_available(i)),
                 "healthy": bool(w.native.dir_healthy(i))} for i, d in enumerate(store.dirs)]
        return _json({"version": __version__, "workerInfo": {"workerAddress": wp.address, "workerId": w.worker_id,
                                                             "device": store.device},
                      "capacityBytes": bytes_to_human(sum(cap.values())), "usedBytes": bytes_to_human(sum(used.values())),
                      "usageOnTiers": [{"tierAlias": t, "capacity": bytes_to_human(c),
                                        "usedCapacity": bytes_to_human(used.get(t, 0)),
                                        "usedSpacePercent": _pct(used.get(t, 0), c)} for t, c in sorted(cap.items())],
                      "storageDirs": dirs})

    def blockinfo(q, b):
        w = wp.worker
        limit = int(q.get("limit", 1000) or 1000)
        rows = []
        ids = sorted(w.native.block_ids(-1))
        for bid in ids[:limit]:
            try:
                info = w.block_info(bid)
            except Exception:  # noqa: BLE001 - evicted meanwhile
                continue
            rows.append({"id": bid, "blockLength": info.length, "tierAlias": getattr(info, "tier_alias", "") or "",
                         "medium": getattr(info, "medium", "") or ""})
        return _json({"nTotalFile": len(ids), "fileBlocksOnTier": rows, "fatalError": "", "invalidPathError": "",
                      "orderedTierAliases": sorted({d.alias for d in wp.store.dirs})})

    def metrics(q, b):
        return _json({"operationMetrics": wp.worker.metrics.registry.snapshot()})

    pre = "/api/v1/worker/"
    return {("GET", pre + "webui_init"): init, ("GET", pre + "webui_overview"): overview,
            ("GET", pre + "webui_blockinfo"): blockinfo, ("GET", pre + "webui_metrics"): metrics}


_STATIC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "static", "webui")


def static_routes(role: str) -> dict:
    """The single-page app: /webui (index, with the role) and its script and style sheet."""
    def page(q, b):
        with open(os.path.join(_STATIC, "index.html"), encoding="utf-8") as f:
            return 200, "text/html; charset=utf-8", f.read().replace("{{ROLE}}", role)

    def asset(name, ctype):
        def fn(q, b):
            with open(os.path.join(_STATIC, name), "rb") as f:
                return 200, ctype, f.read()
        return fn
    return {("GET", "/webui"): page, ("GET", "/webui/app.js"): asset("app.js", "application/javascript"),
            ("GET", "/webui/app.css"): asset("app.css", "text/css")}
