// Single-page web UI for the master and worker processes (reference: webui/master/src and
// webui/worker/src, React).  Pages are client-side routes over the webui_* JSON endpoints
// (alluxio_amd/web/webui_api.py); no build step, no dependencies.
(function () {
  "use strict";
  const role = document.body.dataset.role === "worker" ? "worker" : "master";
  const api = "/api/v1/" + role + "/";
  const PAGES = role === "master"
    ? [["overview", "Overview"], ["browse", "Browse"], ["data", "In-Alluxio Data"], ["logs", "Logs"],
       ["config", "Configuration"], ["workers", "Workers"], ["metrics", "Metrics"], ["mounttable", "Mount Table"]]
    : [["overview", "Overview"], ["blockinfo", "BlockInfo"], ["metrics", "Metrics"]];
  let refreshMs = 15000, timer = null;

  const esc = (s) => String(s === undefined || s === null ? "" : s).replace(/[&<>"']/g,
    (c) => ({"&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;", "'": "&#39;"}[c]));
  const kv = (pairs) => "<table>" + pairs.map(([k, v]) => `<tr><th>${esc(k)}</th><td>${esc(v)}</td></tr>`).join("") +
    "</table>";
  const bar = (pct) => `<span class="bar"><span style="width:${Math.max(0, Math.min(100, pct | 0))}%"></span></span> ${pct | 0}%`;

  // tables sort by a clicked header (numbers numerically)
  function table(headers, rows, raw) {
    const id = "t" + Math.random().toString(36).slice(2);
    const body = rows.map((r) => "<tr>" + r.map((c, i) => `<td>${raw && raw.includes(i) ? c : esc(c)}</td>`).join("") + "</tr>");
    setTimeout(() => {
      const t = document.getElementById(id);
      if (!t) return;
      t.querySelectorAll("th").forEach((th, col) => th.addEventListener("click", () => {
        const tb = t.tBodies[0], trs = Array.from(tb.rows), dir = th.dataset.dir === "a" ? -1 : 1;
        th.dataset.dir = dir === 1 ? "a" : "d";
        trs.sort((x, y) => {
          const a = x.cells[col].textContent, b = y.cells[col].textContent, na = parseFloat(a), nb = parseFloat(b);
          return dir * (!isNaN(na) && !isNaN(nb) ? na - nb : a.localeCompare(b));
        });
        trs.forEach((tr) => tb.appendChild(tr));
      }));
    });
    return `<table id="${id}"><thead><tr>${headers.map((h) => `<th>${esc(h)}</th>`).join("")}</tr></thead><tbody>` +
      body.join("") + "</tbody></table>";
  }

  async function get(name, params) {
    const q = params ? "?" + new URLSearchParams(params).toString() : "";
    const r = await fetch(api + name + q, {headers: {Accept: "application/json"}});
    if (!r.ok) throw new Error(`${name}: HTTP ${r.status}`);
    return r.json();
  }

  const render = {
    async overview() {
      const o = await get("webui_overview");
      if (role === "worker") {
        return "<h1>Worker Overview</h1>" + kv([["Worker Address", o.workerInfo.workerAddress],
          ["Worker Id", o.workerInfo.workerId], ["Device", o.workerInfo.device], ["Version", o.version],
          ["Capacity", o.capacityBytes], ["Used", o.usedBytes]]) +
          "<h2>Tiers</h2>" + table(["Tier", "Capacity", "Used", "Usage"],
            o.usageOnTiers.map((t) => [t.tierAlias, t.capacity, t.usedCapacity, bar(t.usedSpacePercent)]), [3]) +
          "<h2>Storage Directories</h2>" + table(["Tier", "Medium", "Path", "Capacity", "Used", "Healthy"],
            o.storageDirs.map((d) => [d.tierAlias, d.medium, d.dirPath, d.capacity, d.usedCapacity, d.healthy]));
      }
      return "<h1>Master Overview</h1>" + kv([["Master Address", o.masterNodeAddress], ["Started", o.startTime],
        ["Uptime", o.uptime], ["Version", o.version], ["Primary", o.primary], ["Safe Mode", o.safeMode],
        ["Live Workers", o.liveWorkerNodes], ["Config Check", o.configCheckStatus]]) +
        "<h2>Cluster Usage</h2>" + kv([["Capacity", o.capacity], ["Used", o.usedCapacity], ["Free", o.freeCapacity]]) +
        "<h2>Storage Tiers</h2>" + table(["Tier", "Capacity", "Used", "Free", "Usage"],
          o.storageTierInfos.map((t) => [t.storageTierAlias, t.capacity, t.usedCapacity, t.freeCapacity,
            bar(t.usedSpacePercent)]), [4]) +
        "<h2>Master Disk</h2>" + kv([["Capacity", o.diskCapacity], ["Used", o.diskUsedCapacity], ["Free", o.diskFreeCapacity]]);
    },
    async browse(params) {
      const path = params.get("path") || "/";
      const b = await get("webui_browse", {path: path, offset: params.get("offset") || 0, limit: 1000});
      if (b.fileDoesNotExistException) return `<h1>Browse</h1><p class="err">${esc(b.fileDoesNotExistException)}</p>`;
      const crumbs = ['<a href="#/browse?path=/">/</a>'].concat(b.pathInfos.map((p) =>
        `<a href="#/browse?path=${encodeURIComponent(p.absolutePath)}">${esc(p.name)}</a>`)).join(" / ");
      let h = `<h1>Browse</h1><p>${crumbs}</p>`;
      if (b.currentDirectory && !b.currentDirectory.isDirectory) {
        const f = b.currentDirectory;
        return h + kv([["Path", f.absolutePath], ["Size", f.size], ["Block Size", f.blockSizeBytes],
          ["In Alluxio", f.inAlluxioPercentage + "%"], ["Persistence", f.persistenceState], ["Owner", f.owner],
          ["Group", f.group], ["Mode", f.mode], ["Modified", f.modificationTime]]) +
          "<h2>Blocks</h2>" + table(["Block Id", "Length", "Locations"],
            (b.fileBlocks || []).map((x) => [x.id, x.blockLength, x.locations.join(", ")]));
      }
      h += `<p>${b.nTotalFile} entries</p>`;
      return h + table(["Name", "Size", "Block Size", "In Alluxio", "Persistence", "Pinned", "Mode", "Owner", "Group",
        "Modified"], b.fileInfos.map((f) => [
        `<a href="#/browse?path=${encodeURIComponent(f.absolutePath)}">${esc(f.name)}${f.isDirectory ? "/" : ""}</a>`,
        f.size, f.blockSizeBytes, f.isDirectory ? "" : f.inAlluxioPercentage + "%", f.persistenceState,
        f.pinned ? "yes" : "", f.mode, f.owner, f.group, f.modificationTime]), [0]);
    },
    async data() {
      const d = await get("webui_data");
      return `<h1>In-Alluxio Data</h1><p>${d.inAlluxioFileNum} files fully in Alluxio</p>` +
        table(["Path", "Size", "Block Size", "Pinned", "Owner", "Modified"],
          d.fileInfos.map((f) => [f.absolutePath, f.size, f.blockSizeBytes, f.pinned ? "yes" : "", f.owner,
            f.modificationTime]));
    },
    async logs(params) {
      const name = params.get("path") || "";
      const l = await get("webui_logs", name ? {path: name} : null);
      if (name) return `<h1>Log ${esc(name)}</h1>` + (l.invalidPathError ? `<p class="err">${esc(l.invalidPathError)}</p>`
        : `<pre>${esc(l.fileData)}</pre>`);
      return "<h1>Logs</h1>" + (l.fileInfos.length ? table(["File"], l.fileInfos.map((f) =>
        [`<a href="#/logs?path=${encodeURIComponent(f.name)}">${esc(f.name)}</a>`]), [0]) : "<p>No log directory.</p>");
    },
    async config() {
      const c = await get("webui_config");
      return '<h1>Configuration</h1><input id="flt" placeholder="filter properties">' +
        table(["Property", "Value", "Source"], c.configuration);
    },
    async workers() {
      const w = await get("webui_workers");
      const rows = (xs) => xs.map((n) => [`${n.host}:${n.rpcPort}`, n.state, n.workerId, n.capacity, n.usedMemory,
        bar(n.usedSpacePercent), n.lastContactSec]);
      return "<h1>Workers</h1>" + table(["Worker", "State", "Id", "Capacity", "Used", "Usage", "Last Heartbeat (s)"],
        rows(w.normalNodeInfos).concat(rows(w.failedNodeInfos)), [5]);
    },
    async metrics() {
      const m = await get("webui_metrics");
      let h = "<h1>Metrics</h1>";
      if (role === "master") h += kv([["Capacity Used", m.masterCapacityUsedPercentage + "%"],
        ["Bytes Read Local", m["Cluster.BytesReadLocal"]], ["Bytes Read Remote", m["Cluster.BytesReadRemote"]],
        ["Bytes Read UFS", m["Cluster.BytesReadUfsAll"]], ["Bytes Written Local", m["Cluster.BytesWrittenLocal"]],
        ["Bytes Written UFS", m["Cluster.BytesWrittenUfsAll"]]]);
      const ops = m.operationMetrics || {};
      h += "<h2>Operations</h2>" + table(["Metric", "Value"], Object.keys(ops).sort().map((k) => [k, ops[k]]));
      if (m.rpcInvocationMetrics) h += "<h2>Process</h2>" + table(["Metric", "Value"],
        Object.keys(m.rpcInvocationMetrics).sort().map((k) => [k, m.rpcInvocationMetrics[k]]));
      return h;
    },
    async mounttable() {
      const t = await get("webui_mounttable");
      return "<h1>Mount Table</h1>" + table(["Alluxio Path", "UFS URI", "Type", "Read Only", "Shared"],
        Object.keys(t.mountPointInfos).sort().map((p) => {
          const i = t.mountPointInfos[p];
          return [p, i.ufsUri, i.ufsType, i.readOnly, i.shared];
        }));
    },
    async blockinfo() {
      const b = await get("webui_blockinfo", {limit: 1000});
      return `<h1>Block Info</h1><p>${b.nTotalFile} blocks</p>` +
        table(["Block Id", "Length", "Tier", "Medium"], b.fileBlocksOnTier.map((x) => [x.id, x.blockLength, x.tierAlias,
          x.medium]));
    },
  };

  async function route() {
    const hash = location.hash.replace(/^#\/?/, "") || "overview";
    const [page, qs] = hash.split("?");
    const name = render[page] ? page : "overview";
    document.getElementById("nav").innerHTML = PAGES.map(([p, t]) =>
      `<a href="#/${p}"${p === name ? ' class="on"' : ""}>${esc(t)}</a>`).join("");
    const main = document.getElementById("main");
    try {
      main.innerHTML = await render[name](new URLSearchParams(qs || ""));
      const flt = document.getElementById("flt");
      if (flt) flt.addEventListener("input", () => {
        const v = flt.value.toLowerCase();
        main.querySelectorAll("tbody tr").forEach((tr) => {
          tr.style.display = tr.textContent.toLowerCase().includes(v) ? "" : "none";
        });
      });
    } catch (e) {
      main.innerHTML = `<p class="err">${esc(e.message)}</p>`;
    }
    document.getElementById("foot").textContent = `Alluxio ${role} - refreshed ${new Date().toLocaleTimeString()}`;
    clearTimeout(timer);
    if (name === "overview" || name === "workers" || name === "metrics") timer = setTimeout(route, refreshMs);
  }

  window.addEventListener("hashchange", route);
  get("webui_init").then((i) => { refreshMs = i.refreshInterval || refreshMs; }).catch(() => {}).then(route);
})();
