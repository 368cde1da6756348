"""bench.py contract: --gpus N launches N ranks itself, every phase verifies its bytes.

Runs on CPU with the gloo backend and shared-memory DRAM arenas: the ``remote`` phase maps the
peer worker's arena (memfd) exactly as the GPU path maps a peer's HBM (HIP IPC), and the
``replicate`` phase's replicas pull blocks out of the primary's arena (PeerTransfer).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, tmp_path, expect_rc=0, extra_env=None):
    env = dict(os.environ)
    env.update(extra_env or {})
    env.pop("WORLD_SIZE", None)
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args, "--work-dir", str(tmp_path)],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == expect_rc, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


SMALL = ["--steps", "3", "--warmup", "1", "--file-size", "8m", "--block-size", "4m", "--page-size", "1m",
         "--threads", "8", "--duration", "0.2"]


def test_bench_single_rank(tmp_path):
    out = _run([*SMALL, "--large-size", "24m"], tmp_path)
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["warmup"] == 1
    c = out["config"]
    assert c["verified"] and c["stagger_GBps"] > 0 and c["duration_GBps"] > 0
    large = c["phases"]["large"]
    assert large["verified"] and large["file_size"] == 24 << 20 and c["large_GBps"] > 0
    # every call moves 4 KiB except the EOF (reopen) calls
    assert large["steps"] >= 32 and 0.99 * large["steps"] * 8 * (1 << 20) < large["bytes"] <= large["steps"] * 8 * (1 << 20)
    assert c["remote_GBps"] is None and c["replication"] is None
    assert out["value"] == c["phases"]["local"]["GBps"]


def test_bench_two_ranks_remote_and_replicate(tmp_path):
    out = _run(["--gpus", "2", *SMALL], tmp_path)
    assert out["n_gpus"] == 2
    c = out["config"]
    assert c["verified"] and c["parallelism"] == "workers2"
    assert c["phases"]["remote"]["verified"] and c["remote_GBps"] > 0
    rep = c["replication"]
    assert rep["replicas"] == 2 and rep["verified"]
    # each rank's 8 MiB file got one extra copy, pulled out of the primary's arena
    assert rep["shared_bytes_received"] + rep["xgmi_bytes_received"] == 2 * (8 << 20)
    assert rep["stream_fallback_bytes_received"] == 0 and rep["peer_pull_failures"] == 0
    assert rep["data_plane_ok"]
    assert c["process_group"] == {"backend": "gloo", "world_size": 2}
    assert c["devices"] == [-1, -1] and len(c["peer_devices"]) == 2


def test_bench_fails_when_replicas_fall_back_to_grpc(tmp_path):
    """A mapped-pull failure makes the replicas come through the gRPC block stream: the bytes
    still arrive (the write succeeds), but the bench must not report that as the peer data plane.
    The JSON line says so (``verified`` false); the exit status follows the headline phase, whose
    bytes were verified, so a failing secondary phase never costs the headline number."""
    out = _run(["--gpus", "2", *SMALL, "--phases", "local,replicate",
                "--prop", "alluxio.test.peer.mapped.pull.fail=true"], tmp_path, expect_rc=0)
    rep = out["config"]["replication"]
    assert not rep["data_plane_ok"] and not out["config"]["verified"]
    assert out["config"]["headline_verified"]
    # the failures themselves land in the untimed warmup write; the peer is then in its cooldown,
    # so the timed write's replicas all come through the stream
    assert rep["stream_fallback_bytes_received"] == 2 * (8 << 20)


def test_bench_remote_failure_on_one_rank_keeps_the_headline(tmp_path):
    """The remote phase's reader fails on rank 1 only: both ranks agree to skip the phase (no rank
    is left waiting in a collective), the failure is reported, and the headline line is printed."""
    out = _run(["--gpus", "2", *SMALL, "--phases", "local,remote,stagger"], tmp_path,
               extra_env={"ALLUXIO_BENCH_TEST_REMOTE_FAIL_RANK": "1"})
    c = out["config"]
    assert c["remote_GBps"] is None and "injected" in c["phase_errors"]["remote"]
    assert c["headline_verified"] and not c["verified"] and out["value"] > 0
    assert c["stagger_GBps"] > 0                    # later phases still ran on both ranks


def test_bench_hung_cross_rank_phase_ends_with_the_headline(tmp_path):
    """Rank 1 hangs inside the remote phase: past --phase-timeout every rank stops, and rank 0
    prints the JSON line first (headline measured, the phase reported as timed out)."""
    import time
    t = time.time()
    out = _run(["--gpus", "2", *SMALL, "--phases", "local,remote", "--phase-timeout", "8"], tmp_path,
               extra_env={"ALLUXIO_BENCH_TEST_REMOTE_HANG_RANK": "1"})
    c = out["config"]
    assert "timed out" in c["phase_errors"]["remote"] and c["remote_GBps"] is None
    assert c["headline_verified"] and out["value"] > 0
    assert time.time() - t < 200
