"""Stress report generator (stress/shell/.../cli/report/GenerateReport.java analogue)."""
import json

import pytest

from alluxio_amd.stress import report
from alluxio_amd.stress.__main__ import main as stress_main


def _w(p, obj, lines=False):
    p.write_text(("noise line\n" + json.dumps(obj) + "\n") if lines else json.dumps(obj))
    return str(p)


def test_master_report(tmp_path):
    a = _w(tmp_path / "run1.json", {"bench": "master", "operation": "CreateFile", "threads": 8,
                                    "throughput_ops": 2100.0, "latency_ms": {"p50": 3.1, "p99": 9.0},
                                    "errors": ["x: timeout"]})
    b = _w(tmp_path / "run2.json", {"bench": "master", "operation": "CreateFile", "threads": 32,
                                    "throughput_ops": 3100.0, "latency_ms": {"p50": 8.0, "p99": 20.0}, "errors": []})
    out = tmp_path / "r.html"
    assert stress_main(["report", "--input", a, "--input", b, "--output", str(out)]) == 0
    page = out.read_text()
    assert page.count("<svg") == 2 and "Master throughput" in page
    assert "ERRORS[1]: run1" in page and "x: timeout" in page
    data = json.loads(__import__("html").unescape(page.split('id="graph-data">')[1].split("</script>")[0]))
    assert data[0]["series"]["run2"] == [["CreateFile", 3100.0]]


def test_client_io_and_benchpy_lines(tmp_path):
    rows = [{"threads": t, "throughput_MBps": 100.0 * t, "bytes": 1, "errors": []} for t in (1, 2, 4)]
    a = _w(tmp_path / "cio.json", {"bench": "client-io", "operation": "ReadByteBuffer", "rows": rows,
                                   "throughput_MBps": 400.0, "errors": []})
    graphs = report.generate([a], str(tmp_path / "c.html"))
    assert [g.kind for g in graphs] == ["bar", "line"]
    assert graphs[1].series["cio"] == [(1, 100.0), (2, 200.0), (4, 400.0)]
    line = {"metric": "GB/s", "value": 5954.6, "unit": "GB/s", "n_gpus": 1,
            "config": {"phases": {"local": {"GBps": 5954.6}, "stagger": {"GBps": 2776.3}}}}
    b = _w(tmp_path / "bench.jsonl", line, lines=True)
    graphs = report.generate([b], str(tmp_path / "b.html"))
    assert graphs[1].series["bench"] == [("local", 5954.6), ("stagger", 2776.3)]


def test_mismatched_types_refused(tmp_path):
    a = _w(tmp_path / "m.json", {"bench": "master", "throughput_ops": 1})
    b = _w(tmp_path / "w.json", {"bench": "worker", "throughput_MBps": 1})
    with pytest.raises(ValueError, match="Mismatched"):
        report.generate([a, b], str(tmp_path / "x.html"))
