"""Smoke runs of the round-5 write-path benches on CPU (DRAM tier), so their output rows keep the
fields the profiles cite: worker_write_bench (CACHE_THROUGH tee bytes, sustained --min-seconds
mode) and persist_bench (worker append vs client copy, both verified)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rows(args, timeout=300):
    env = dict(os.environ)
    r = subprocess.run([sys.executable, *args], capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


def test_worker_write_bench_tee_rows():
    rows = _rows(["tools/worker_write_bench.py", "--threads", "2", "--files", "2", "--file-size", "8m",
                  "--block-size", "4m", "--write-type", "CACHE_THROUGH", "--min-seconds", "1"])
    (r,) = rows
    assert r["threads"] == 2 and not r["errors"] and r["seconds"] >= 1.0
    assert r["ufs_tee_bytes"] >= r["bytes"] and r["GBps"] > 0       # every byte reached the UFS by the tee


def test_persist_bench_rows():
    rows = _rows(["tools/persist_bench.py", "--threads", "1", "--files", "2", "--file-size", "8m",
                  "--block-size", "4m"])
    by = {r["mode"]: r for r in rows}
    assert set(by) == {"append", "client"}
    assert all(r["verified"] and not r["errors"] for r in rows)
    assert by["append"]["ufs_tee_bytes"] == by["append"]["bytes"] == 2 * (8 << 20)
    assert by["client"]["ufs_tee_bytes"] == 0
