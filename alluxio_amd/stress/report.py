"""``alluxio stress report --input a.json --input b.json --output report.html``.

Parity: stress/shell/src/main/java/alluxio/stress/cli/report/GenerateReport.java (several JSON
summaries of one benchmark type in, one HTML page of comparison graphs out, each graph followed by
the per-series error lists in ``<details>``; mismatched summary types are refused) and the
summaries' GraphGenerators (master: throughput and latency percentiles per input; worker /
client IO: throughput per input and per thread count; max throughput: achieved vs target rate).

The reference page pulls vega-lite from a CDN; this one draws inline SVG so a report opens on an
offline cluster host.  Inputs are this project's stress JSON (``python -m alluxio_amd.stress``,
``run_local``/``merge_results``) and, for convenience, the driver's ``bench.py`` JSON lines.
"""
from __future__ import annotations

import argparse
import html
import json
import os
import sys

PALETTE = ["#c0392b", "#2471a3", "#229954", "#b7950b", "#7d3c98", "#ca6f1e", "#17a589", "#5d6d7e"]


class Graph:
    """One chart: ``kind`` "bar" (categories x series) or "line" (x/y points per series)."""

    def __init__(self, title: str, x_label: str, y_label: str, kind: str = "bar"):
        self.title, self.x_label, self.y_label, self.kind = title, x_label, y_label, kind
        self.series: dict[str, list[tuple]] = {}
        self.errors: dict[str, list[str]] = {}

    def add(self, series: str, x, y: float) -> None:
        self.series.setdefault(series, []).append((x, float(y)))

    def add_errors(self, series: str, errors) -> None:
        if errors:
            self.errors.setdefault(series, []).extend(str(e) for e in errors)

    def to_dict(self) -> dict:
        return {"title": self.title, "x": self.x_label, "y": self.y_label, "kind": self.kind,
                "series": {k: [list(p) for p in v] for k, v in self.series.items()}, "errors": self.errors}

    # ---- SVG ---------------------------------------------------------------------------------
    def svg(self, width: int = 760, height: int = 360) -> str:
        ml, mr, mt, mb = 70, 170, 30, 50
        pw, ph = width - ml - mr, height - mt - mb
        ys = [y for pts in self.series.values() for _, y in pts] or [0.0]
        ymax = max(ys) * 1.1 or 1.0
        out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{width}" height="{height}" '
               f'font-family="sans-serif" font-size="11">',
               f'<text x="{width / 2}" y="16" text-anchor="middle" font-size="14">{html.escape(self.title)}</text>']
        for i in range(6):                     # y grid + ticks
            v = ymax * i / 5
            y = mt + ph - ph * i / 5
            out.append(f'<line x1="{ml}" x2="{ml + pw}" y1="{y:.1f}" y2="{y:.1f}" stroke="#ddd"/>')
            out.append(f'<text x="{ml - 6}" y="{y + 4:.1f}" text-anchor="end">{_fmt(v)}</text>')
        out.append(f'<text x="16" y="{mt + ph / 2}" transform="rotate(-90 16 {mt + ph / 2})" '
                   f'text-anchor="middle">{html.escape(self.y_label)}</text>')
        out.append(f'<text x="{ml + pw / 2}" y="{height - 8}" text-anchor="middle">{html.escape(self.x_label)}</text>')
        names = list(self.series)
        if self.kind == "bar":
            cats = []
            for pts in self.series.values():
                for x, _ in pts:
                    if x not in cats:
                        cats.append(x)
            cw = pw / max(1, len(cats))
            bw = cw * 0.8 / max(1, len(names))
            for si, name in enumerate(names):
                vals = dict(self.series[name])
                for ci, c in enumerate(cats):
                    if c not in vals:
                        continue
                    h = ph * vals[c] / ymax
                    x = ml + ci * cw + cw * 0.1 + si * bw
                    out.append(f'<rect x="{x:.1f}" y="{mt + ph - h:.1f}" width="{bw:.1f}" height="{h:.1f}" '
                               f'fill="{PALETTE[si % len(PALETTE)]}"><title>{html.escape(name)} {html.escape(str(c))}: '
                               f'{_fmt(vals[c])}</title></rect>')
            for ci, c in enumerate(cats):
                out.append(f'<text x="{ml + ci * cw + cw / 2:.1f}" y="{mt + ph + 16}" text-anchor="middle">'
                           f'{html.escape(str(c))}</text>')
        else:
            xs = [float(x) for pts in self.series.values() for x, _ in pts] or [0.0]
            xmin, xmax = min(xs), max(xs)
            span = (xmax - xmin) or 1.0
            for xv in sorted(set(xs)):
                x = ml + pw * (xv - xmin) / span
                out.append(f'<text x="{x:.1f}" y="{mt + ph + 16}" text-anchor="middle">{_fmt(xv)}</text>')
            for si, name in enumerate(names):
                pts = sorted((float(x), y) for x, y in self.series[name])
                coords = [(ml + pw * (x - xmin) / span, mt + ph - ph * y / ymax) for x, y in pts]
                col = PALETTE[si % len(PALETTE)]
                out.append('<polyline fill="none" stroke="{}" stroke-width="2" points="{}"/>'.format(
                    col, " ".join(f"{x:.1f},{y:.1f}" for x, y in coords)))
                for (x, y), (xv, yv) in zip(coords, pts):
                    out.append(f'<circle cx="{x:.1f}" cy="{y:.1f}" r="3" fill="{col}"><title>{html.escape(name)} '
                               f'{_fmt(xv)}: {_fmt(yv)}</title></circle>')
        out.append(f'<line x1="{ml}" x2="{ml}" y1="{mt}" y2="{mt + ph}" stroke="#333"/>')
        out.append(f'<line x1="{ml}" x2="{ml + pw}" y1="{mt + ph}" y2="{mt + ph}" stroke="#333"/>')
        for si, name in enumerate(names):       # legend
            y = mt + 14 * si
            out.append(f'<rect x="{ml + pw + 12}" y="{y}" width="10" height="10" fill="{PALETTE[si % len(PALETTE)]}"/>')
            out.append(f'<text x="{ml + pw + 26}" y="{y + 9}">{html.escape(_short(name))}</text>')
        out.append("</svg>")
        return "\n".join(out)


def _fmt(v: float) -> str:
    a = abs(v)
    if a >= 1e9:
        return f"{v / 1e9:.2f}G"
    if a >= 1e6:
        return f"{v / 1e6:.2f}M"
    if a >= 1e4:
        return f"{v / 1e3:.1f}k"
    if a >= 100 or v == int(v):
        return f"{v:.0f}"
    return f"{v:.2f}"


def _short(s: str, n: int = 24) -> str:
    return s if len(s) <= n else "…" + s[-(n - 1):]


# ---- summary type -> graphs (the reference GraphGenerator per Summary class) ---------------------
def summary_type(s: dict) -> str:
    if "bench" in s:
        return s["bench"]
    if "metric" in s and "value" in s:
        return "bench.py"
    raise ValueError("not a stress summary (no 'bench' field)")


def _nodes(s: dict) -> list[dict]:
    """A job-service merged summary keeps per-worker rows; a local run is its own row."""
    return s.get("nodes") or [s]


def _master_graphs(inputs) -> list[Graph]:
    thr = Graph("Master throughput", "operation", "ops/s")
    lat = Graph("Master latency percentiles", "percentile", "ms")
    for name, s in inputs:
        for n in _nodes(s):
            op = n.get("operation", "?")
            thr.add(name, op, n.get("throughput_ops", 0.0))
            for p, v in (n.get("latency_ms") or {}).items():
                lat.add(f"{name}:{op}", p, v)
        thr.add_errors(name, s.get("errors"))
    return [thr, lat]


def _io_graphs(inputs, title: str) -> list[Graph]:
    thr = Graph(f"{title} throughput", "input", "MB/s")
    by_threads = Graph(f"{title} throughput by thread count", "threads", "MB/s", kind="line")
    for name, s in inputs:
        thr.add(name, s.get("operation") or s.get("mode") or "run", s.get("throughput_MBps", 0.0))
        for n in _nodes(s):
            for r in n.get("rows", []):
                by_threads.add(name, r["threads"], r["throughput_MBps"])
            if "rows" not in n and "threads" in n:
                by_threads.add(name, n["threads"], n.get("throughput_MBps", 0.0))
        thr.add_errors(name, s.get("errors"))
    graphs = [thr]
    if any(len(v) > 1 for v in by_threads.series.values()) or len(by_threads.series) > 1:
        graphs.append(by_threads)
    return graphs


def _ufs_graphs(inputs) -> list[Graph]:
    g = Graph("UFS IO throughput", "phase", "MB/s")
    for name, s in inputs:
        for n in _nodes(s):
            for phase in ("write", "read"):
                if isinstance(n.get(phase), dict):
                    g.add(name, phase, n[phase].get("MBps", 0.0))
        g.add_errors(name, s.get("errors"))
    return [g]


def _max_graphs(inputs) -> list[Graph]:
    best = Graph("Max throughput", "input", "ops/s")
    trace = Graph("Max throughput search (achieved vs target)", "target ops/s", "achieved ops/s", kind="line")
    for name, s in inputs:
        best.add(name, s.get("operation", "run"), s.get("max_ops", 0.0))
        for t in s.get("trace", []):
            if "target" in t:
                trace.add(name, t["target"], t.get("achieved", t.get("throughput_ops", 0.0)))
    return [best, trace] if trace.series else [best]


def _benchpy_graphs(inputs) -> list[Graph]:
    g = Graph("bench.py headline", "n_gpus", "value", kind="line")
    ph = Graph("bench.py phases", "phase", "GB/s")
    for name, s in inputs:
        g.add(s.get("metric", name)[:40], s.get("n_gpus", 1), s.get("value", 0.0))
        for k, v in (s.get("config", {}).get("phases") or {}).items():
            if isinstance(v, dict) and "GBps" in v:
                ph.add(name, k, v["GBps"])
    g.y_label = inputs[0][1].get("unit", "value")
    return [g, ph] if ph.series else [g]


GENERATORS = {"master": _master_graphs, "worker": lambda i: _io_graphs(i, "Worker"),
              "client-io": lambda i: _io_graphs(i, "Client IO"), "ufs-io": _ufs_graphs,
              "max-throughput": _max_graphs, "bench.py": _benchpy_graphs}


def load(path: str) -> dict:
    with open(path) as f:
        text = f.read().strip()
    try:
        return json.loads(text)
    except json.JSONDecodeError:
        # JSON-lines output (bench.py / tools): the last JSON object line is the summary
        for line in reversed(text.splitlines()):
            line = line.strip()
            if line.startswith("{"):
                return json.loads(line)
        raise


def generate(paths: list[str], output: str) -> list[Graph]:
    inputs = [(os.path.splitext(os.path.basename(p))[0], load(p)) for p in paths]
    types = {summary_type(s) for _, s in inputs}
    if len(types) != 1:
        raise ValueError(f"Mismatched input result types: {sorted(types)}")
    kind = types.pop()
    graphs = GENERATORS[kind](inputs)
    with open(output, "w") as w:
        w.write("<!DOCTYPE html>\n<html><head><meta charset=\"utf-8\">"
                f"<title>{html.escape(kind)} stress report</title></head><body>\n")
        w.write(f"<h2>{html.escape(kind)} stress report</h2>\n<p>inputs: "
                + ", ".join(html.escape(p) for p in paths) + "</p>\n")
        for i, g in enumerate(graphs):
            w.write(f'<div id="graph{i}">\n{g.svg()}\n</div>\n')
            for series, errs in g.errors.items():
                w.write(f"<details><summary>ERRORS[{len(errs)}]: {html.escape(series)}</summary><ul>\n")
                w.write("".join(f"<li>{html.escape(e)}</li>\n" for e in errs))
                w.write("</ul></details>\n")
        w.write('<script type="application/json" id="graph-data">'
                + html.escape(json.dumps([g.to_dict() for g in graphs])) + "</script>\n</body></html>\n")
    return graphs


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="alluxio stress report",
                                 description="Generate an HTML report from stress benchmark JSON results")
    ap.add_argument("--input", action="append", required=True, help="result JSON file (repeatable)")
    ap.add_argument("--output", required=True, help="output HTML file")
    a = ap.parse_args(argv)
    graphs = generate(a.input, a.output)
    print(f"wrote {a.output} ({len(graphs)} graphs)", file=sys.stdout)
    return 0
