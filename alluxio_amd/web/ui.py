"""Server-rendered web UI for masters and workers.

Parity: webui/master/src (React pages Overview, Browse, Configuration, Workers, Metrics, Mount
Table, Logs) and webui/worker/src (Overview, BlockInfo, Metrics), which render the JSON of
AlluxioMasterRestServiceHandler / AlluxioWorkerRestServiceHandler.  The same pages are rendered
here as plain HTML from the same data (no JS toolchain in the image, and none needed): every page
is one GET, linkable, and readable with curl.
"""
from __future__ import annotations

import html
import time

from ..utils.format import bytes_to_human, mode_to_string

_CSS = """
body{font-family:-apple-system,Segoe UI,Helvetica,Arial,sans-serif;margin:0;color:#222;background:#fafafa}
nav{background:#1d2b3a;padding:.6em 1.2em}nav a{color:#dde;margin-right:1.4em;text-decoration:none;font-weight:600}
nav a.on{color:#fff;border-bottom:2px solid #f5a623}main{padding:1.2em 1.6em}
h1{font-size:1.35em;margin:.2em 0 .8em}h2{font-size:1.1em;margin:1.4em 0 .5em}
table{border-collapse:collapse;background:#fff;min-width:40%}td,th{border:1px solid #ddd;padding:.3em .7em;
text-align:left;font-size:.92em}th{background:#eef1f5}.num{text-align:right;font-variant-numeric:tabular-nums}
.bar{background:#e3e8ee;width:160px;height:.8em;display:inline-block}.bar>span{background:#3c8dbc;height:100%;
display:block}pre{background:#fff;border:1px solid #ddd;padding:.8em;overflow:auto;max-height:30em}
"""


def _e(x) -> str:
    return html.escape(str(x))


def _page(title: str, nav: list[tuple[str, str]], active: str, body: str) -> tuple[int, str, str]:
    links = "".join(f'<a href="{h}" class="{"on" if h == active else ""}">{_e(t)}</a>' for t, h in nav)
    doc = (f"<!doctype html><html><head><meta charset='utf-8'><title>{_e(title)}</title>"
           f"<style>{_CSS}</style></head><body><nav>{links}</nav><main><h1>{_e(title)}</h1>{body}</main>"
           f"</body></html>")
    return 200, "text/html; charset=utf-8", doc


def _table(headers, rows, num_cols=()) -> str:
    th = "".join(f"<th>{_e(h)}</th>" for h in headers)
    trs = []
    for r in rows:
        tds = "".join(f'<td class="{"num" if i in num_cols else ""}">{c}</td>' for i, c in enumerate(r))
        trs.append(f"<tr>{tds}</tr>")
    return f"<table><tr>{th}</tr>{''.join(trs)}</table>"


def _kv(pairs) -> str:
    return _table(["Property", "Value"], [(_e(k), _e(v)) for k, v in pairs])


def _bar(used: int, total: int) -> str:
    pct = 0 if not total else min(100, int(100 * used / total))
    return f'<span class="bar"><span style="width:{pct}%"></span></span> {pct}%'


def _ts(ms) -> str:
    return time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(ms / 1000)) if ms else "-"


def _dur(ms: int) -> str:
    s = int(ms // 1000)
    d, s = divmod(s, 86400)
    h, s = divmod(s, 3600)
    m, s = divmod(s, 60)
    return f"{d}d {h:02d}:{m:02d}:{s:02d}"


MASTER_NAV = [("Overview", "/"), ("Browse", "/browse"), ("Workers", "/workers"), ("Configuration", "/config"),
              ("Metrics", "/metrics"), ("Mount Table", "/mounttable"), ("Jobs", "/jobs")]
WORKER_NAV = [("Overview", "/"), ("Block Info", "/blockinfo"), ("Metrics", "/metrics")]


def master_ui_routes(master) -> dict:
    from .. import __version__
    from ..security import as_user

    def superuser():
        return as_user(master.fs_master.permission.superuser)

    def overview(q, b):
        bm = master.block_master
        cap, used = bm.capacity_bytes(), bm.used_bytes()
        live, lost = bm.worker_info_list(), bm.lost_workers_info_list()
        tree = master.fs_master.tree
        journal = type(master.journal).__name__
        rows = [("Master Address", master.address), ("Started", _ts(master.start_time * 1000)),
                ("Uptime", _dur((time.time() - master.start_time) * 1000)), ("Version", __version__),
                ("Primary", master.primary), ("Safe Mode", master.safe_mode.in_safe_mode()),
                ("Cluster Id", master.meta_master.cluster_id or "-"),
                ("Live Workers", len(live)), ("Lost Workers", len(lost)),
                ("Total Paths", len(tree.inodes)), ("Pinned Files", len(tree.pinned_ids)),
                ("Journal", journal), ("Metastore", getattr(tree.inodes, "kind", "HEAP"))]
        body = _kv(rows)
        body += "<h2>Cluster Usage</h2>" + _table(
            ["Capacity", "Used", "Usage"], [(bytes_to_human(cap), bytes_to_human(used), _bar(used, cap))])
        tiers = {}
        for w in live:
            for t, c in w.capacityBytesOnTiers.items():
                tiers.setdefault(t, [0, 0])[0] += c
            for t, u in w.usedBytesOnTiers.items():
                tiers.setdefault(t, [0, 0])[1] += u
        if tiers:
            body += "<h2>Storage Tiers</h2>" + _table(
                ["Tier", "Capacity", "Used", "Usage"],
                [(_e(t), bytes_to_human(c), bytes_to_human(u), _bar(u, c)) for t, (c, u) in sorted(tiers.items())])
        qi = getattr(master.journal, "quorum_info", None)
        if qi is not None:
            body += "<h2>Embedded Journal Quorum</h2>" + _table(
                ["Server", "State"], [(_e(a), "AVAILABLE" if ok else "UNAVAILABLE") for a, ok in qi()])
        return _page("Alluxio Master", MASTER_NAV, "/", body)

    def browse(q, b):
        path = q.get("path", "/") or "/"
        with superuser():
            st = master.fs_master.get_status(path)
            if st.folder:
                infos = master.fs_master.list_status(path)
            else:
                infos = None
        crumbs, acc = ['<a href="/browse?path=/">/</a>'], ""
        for part in [p for p in path.split("/") if p]:
            acc += "/" + part
            crumbs.append(f'<a href="/browse?path={_e(acc)}">{_e(part)}</a>')
        body = "<p>" + " / ".join(crumbs) + "</p>"
        if infos is None:
            body += _kv([("Path", st.path), ("Size", bytes_to_human(st.length)),
                         ("Block Size", bytes_to_human(st.blockSizeBytes)), ("In Alluxio", f"{st.inAlluxioPercentage}%"),
                         ("Persistence", st.persistenceState), ("Pinned", st.pinned), ("Owner", st.owner),
                         ("Group", st.group), ("Mode", mode_to_string(st.mode, False)),
                         ("Modified", _ts(st.lastModificationTimeMs)), ("Blocks", len(st.blockIds)),
                         ("UFS Path", st.ufsPath)])
            return _page(f"File {path}", MASTER_NAV, "/browse", body)
        rows = []
        for i in sorted(infos, key=lambda x: (not x.folder, x.name)):
            link = f'<a href="/browse?path={_e(i.path)}">{_e(i.name)}{"/" if i.folder else ""}</a>'
            rows.append((link, "" if i.folder else bytes_to_human(i.length),
                         "" if i.folder else bytes_to_human(i.blockSizeBytes),
                         "" if i.folder else f"{i.inAlluxioPercentage}%", _e(i.persistenceState),
                         "yes" if i.pinned else "", _e(mode_to_string(i.mode, i.folder)), _e(i.owner), _e(i.group),
                         _ts(i.lastModificationTimeMs)))
        body += _table(["Name", "Size", "Block Size", "In Alluxio", "Persistence", "Pinned", "Mode", "Owner",
                        "Group", "Modified"], rows, num_cols=(1, 2, 3))
        return _page(f"Browse {path}", MASTER_NAV, "/browse", body)

    def workers(q, b):
        bm = master.block_master

        def rows(ws, state):
            return [(_e(f"{w.address.host}:{w.address.rpcPort}"), _e(state), _e(w.id),
                     bytes_to_human(w.capacityBytes), bytes_to_human(w.usedBytes), _bar(w.usedBytes, w.capacityBytes),
                     _e(int(w.lastContactSec))) for w in ws]
        body = _table(["Worker", "State", "Id", "Capacity", "Used", "Usage", "Last Heartbeat (s)"],
                      rows(bm.worker_info_list(), "In Service") + rows(bm.lost_workers_info_list(), "Lost"),
                      num_cols=(3, 4, 6))
        return _page("Workers", MASTER_NAV, "/workers", body)

    def config(q, b):
        m = master.conf.to_map(include_defaults=True)
        return _page("Configuration", MASTER_NAV, "/config",
                     _table(["Property", "Value", "Source"],
                            [(_e(k), _e(v), _e(master.conf.source(k) if hasattr(master.conf, "source") else ""))
                             for k, v in sorted(m.items())]))

    def metrics(q, b):
        cluster = master.metrics_master.get_metrics()
        local = master.metrics.registry.snapshot()
        body = "<h2>Cluster</h2>" + _table(["Metric", "Value"], [(_e(k), _e(v)) for k, v in sorted(cluster.items())],
                                           num_cols=(1,))
        body += "<h2>Master</h2>" + _table(["Metric", "Value"], [(_e(k), _e(v)) for k, v in sorted(local.items())],
                                           num_cols=(1,))
        return _page("Metrics", MASTER_NAV, "/metrics", body)

    def mounttable(q, b):
        mt = master.fs_master.get_mount_table()
        return _page("Mount Table", MASTER_NAV, "/mounttable", _table(
            ["Alluxio Path", "UFS URI", "Read Only", "Shared"],
            [(_e(mp), _e(i.ufsUri), _e(i.readOnly), _e(i.shared)) for mp, i in sorted(mt.items())]))

    def jobs(q, b):
        jm = master.job_master
        rows = [] if jm is None else [(_e(j.id), _e(j.cfg.type_name), _e(j.status), _e(j.error or ""))
                                       for j in sorted(jm.jobs.values(), key=lambda j: j.id)]
        return _page("Jobs", MASTER_NAV, "/jobs", _table(["Id", "Type", "Status", "Error"], rows))

    return {("GET", "/"): overview, ("GET", "/browse"): browse, ("GET", "/workers"): workers,
            ("GET", "/config"): config, ("GET", "/metrics"): metrics, ("GET", "/mounttable"): mounttable,
            ("GET", "/jobs"): jobs}


def worker_ui_routes(wp) -> dict:
    def overview(q, b):
        w, store = wp.worker, wp.store
        cap, used = store.capacity_by_tier(), store.used_by_tier()
        body = _kv([("Worker Address", wp.address), ("Worker Id", w.worker_id), ("Device", store.device),
                    ("Blocks", len(w.native.block_ids(-1)))])
        body += "<h2>Tiers</h2>" + _table(
            ["Tier", "Capacity", "Used", "Usage"],
            [(_e(t), bytes_to_human(c), bytes_to_human(used.get(t, 0)), _bar(used.get(t, 0), c))
             for t, c in sorted(cap.items())])
        dirs = [(_e(d.alias), _e(d.medium), _e(d.path), bytes_to_human(w.native.dir_capacity(i)),
                 bytes_to_human(w.native.dir_available(i)), _e(w.native.dir_healthy(i)))
                for i, d in enumerate(store.dirs)]
        body += "<h2>Storage Directories</h2>" + _table(["Tier", "Medium", "Path", "Capacity", "Available", "Healthy"],
                                                       dirs)
        return _page("Alluxio Worker", WORKER_NAV, "/", body)

    def blockinfo(q, b):
        w = wp.worker
        rows = []
        for bid in sorted(w.native.block_ids(-1))[:int(q.get("limit", 1000))]:
            try:
                info = w.block_info(bid)
                rows.append((_e(bid), bytes_to_human(info.length), _e(getattr(info, "tier_alias", "")) or ""))
            except Exception:  # noqa: BLE001
                continue
        return _page("Block Info", WORKER_NAV, "/blockinfo", _table(["Block Id", "Length", "Tier"], rows))

    def metrics(q, b):
        snap = wp.worker.metrics.registry.snapshot()
        return _page("Metrics", WORKER_NAV, "/metrics",
                     _table(["Metric", "Value"], [(_e(k), _e(v)) for k, v in sorted(snap.items())], num_cols=(1,)))

    return {("GET", "/"): overview, ("GET", "/blockinfo"): blockinfo, ("GET", "/metrics"): metrics}
