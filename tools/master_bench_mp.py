#!/usr/bin/env python3
"""StressMasterBench against a standalone master process over gRPC, with the client threads spread
over several client processes -- the setup of the reference's published master numbers
(docs/en/operation/Scalability-Tuning.md:142-148: one master, 32 clients on other hosts).

    python tools/master_bench_mp.py --ops CreateFile,GetFileStatus,ListDir,DeleteFile \
        --procs 4 --threads 8 --duration 5s --out profiles/master_bench.json

Each client process runs ``alluxio_amd.stress.master_bench`` with ``--threads`` threads; the
result is the sum of the processes' throughputs (they run the same timed window).  Operations run
in the order given on one base directory per client process, as the reference's runs do: DeleteFile
and RenameFile act on the files the preceding CreateFile run made (and stop when they run out).
CPU only: no GPU is touched.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CLIENT = r"""
import json, sys
sys.path.insert(0, {root!r})
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.conf import Configuration
from alluxio_amd.stress import master_bench
import os
if os.environ.get("ALLUXIO_PYSAMPLE_CLIENT"):
    from alluxio_amd.utils.sampler import StackSampler
    _smp = StackSampler().start()
fs = FileSystem(conf=Configuration({cprops!r}), master_address={addr!r})
r = master_bench.main({args!r}, fs=fs, print_result=False)
r["native"] = str(fs.ctx.pool.get({addr!r}, fs.ctx.user)._native)
print("RESULT " + json.dumps(r))
if os.environ.get("ALLUXIO_PYSAMPLE_CLIENT"):
    _smp.stop()
    open(os.environ["ALLUXIO_PYSAMPLE_CLIENT"] + "." + str(os.getpid()), "w").write(_smp.report())
fs.close()
"""


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(ops, procs, threads, duration, warmup, journal_dir=None, props=(), client_props=None, op_args=(),
        ufs_sleep_ms: float = 0.0) -> list[dict]:
    work = tempfile.mkdtemp(prefix="mbench_")
    port, web = _free_port(), _free_port()
    conf_dir = os.path.join(work, "conf")
    os.makedirs(conf_dir)
    with open(os.path.join(conf_dir, "alluxio-site.properties"), "w") as f:
        f.write(f"alluxio.master.journal.folder={journal_dir or os.path.join(work, 'journal')}\n")
        root = os.path.join(work, "ufs")
        os.makedirs(root, exist_ok=True)
        if ufs_sleep_ms:
            # every UFS call of the master sleeps (SleepingUnderFileSystem via the sleepfs:// scheme)
            f.write(f"alluxio.master.mount.table.root.ufs=sleepfs://{root}\n")
            f.write(f"alluxio.underfs.sleep.ms={ufs_sleep_ms}\n")
        else:
            f.write(f"alluxio.master.mount.table.root.ufs={root}\n")
        f.write(f"alluxio.master.web.port={web}\n")
        f.write("alluxio.master.journal.type=UFS\n")
        for kv in props:
            f.write(kv + "\n")
    env = dict(os.environ, ALLUXIO_CONF_DIR=conf_dir, PYTHONPATH=ROOT)
    master = subprocess.Popen([sys.executable, "-m", "alluxio_amd.master.process", "--host", "127.0.0.1",
                               "--port", str(port), "--format"], env=env, cwd=work,
                              stdout=subprocess.DEVNULL, stderr=open(os.path.join(work, "master.log"), "w"))
    addr = f"127.0.0.1:{port}"
    try:
        deadline = time.time() + 60
        while time.time() < deadline:
            with socket.socket() as s:
                if s.connect_ex(("127.0.0.1", port)) == 0:
                    break
            time.sleep(0.2)
        time.sleep(1.0)
        out = []
        created = {}     # per client process: files its CreateFile run made (DeleteFile/RenameFile input)
        def master_cpu_s(split: bool = False):
            # utime + stime of the master process (the GIL bound shows as ~1 core busy)
            with open(f"/proc/{master.pid}/stat") as f:
                fields = f.read().rsplit(")", 1)[1].split()
            tck = os.sysconf("SC_CLK_TCK")
            if split:
                return int(fields[11]) / tck, int(fields[12]) / tck
            return (int(fields[11]) + int(fields[12])) / tck

        for op in ops:
            args = ["--operation", op, "--threads", str(threads), "--duration", duration, "--warmup", warmup,
                    *op_args]
            (u0, s0), wall0 = master_cpu_s(True), time.time()
            cpu0 = u0 + s0
            samples = []            # (wall, user, sys) every 50 ms: the master's CPU inside the window
            stop_smp = threading.Event()

            def sampler():
                while not stop_smp.is_set():
                    try:
                        samples.append((time.time(), *master_cpu_s(True)))
                    except OSError:
                        return
                    stop_smp.wait(0.05)
            smp = threading.Thread(target=sampler, daemon=True)
            smp.start()
            ps = []
            for i in range(procs):
                a = args + ["--base", f"/stress-master-{i}"]
                if op in ("DeleteFile", "RenameFile") and i in created:
                    a += ["--stop-count", str(created[i])]
                ps.append(subprocess.Popen([sys.executable, "-c", CLIENT.format(root=ROOT, addr=addr, args=a,
                                                                                cprops=dict(client_props or {}))],
                                           env=env, cwd=work, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                           text=True))
            res = []
            for i, p in enumerate(ps):
                so, _ = p.communicate(timeout=600)
                line = next((ln for ln in so.splitlines() if ln.startswith("RESULT ")), None)
                if line:
                    res.append(json.loads(line[7:]))
                    if op == "CreateFile":
                        created[i] = res[-1]["completed"]
            u1, s1 = master_cpu_s(True)
            cpu = u1 + s1 - cpu0
            stop_smp.set()
            smp.join()
            win = None
            ws = [r["window_wall"] for r in res if "window_wall" in r]
            if ws:
                w0, w1 = max(w[0] for w in ws), min(w[1] for w in ws)
                inside = [x for x in samples if w0 <= x[0] <= w1]
                if len(inside) >= 2 and inside[-1][0] > inside[0][0]:
                    dt = inside[-1][0] - inside[0][0]
                    du, ds = inside[-1][1] - inside[0][1], inside[-1][2] - inside[0][2]
                    tot = sum(r["throughput_ops"] for r in res)
                    win = {"cores": round((du + ds) / dt, 2), "user_cores": round(du / dt, 2),
                           "us_per_op": round((du + ds) * 1e6 / (tot * dt), 1) if tot else None}
            wall = time.time() - wall0
            total = sum(r["throughput_ops"] for r in res)
            p50 = sorted(r["latency_ms"]["p50"] for r in res)[len(res) // 2] if res else None
            p99 = sorted(r["latency_ms"].get("p99", 0) for r in res)[len(res) // 2] if res else None
            errs = sum(len(r["errors"]) for r in res)
            done = sum(r.get("completed", 0) for r in res)
            row = {"operation": op, "procs": procs, "threads_per_proc": threads, "ops_per_s": round(total, 1),
                   "p50_ms": p50, "p99_ms": p99, "errors": errs,
                   # master process CPU over the whole client run (setup + warmup + window)
                   "master_cpu_cores": round(cpu / max(wall, 1e-9), 2),
                   "master_cpu_us_per_op": round(cpu * 1e6 / done, 1) if done else None,
                   "master_sys_fraction": round((s1 - s0) / cpu, 2) if cpu > 0 else None,
                   # the same, sampled inside the timed window only (all clients running)
                   "master_cpu_window": win}
            print(json.dumps(row), flush=True)
            out.append(row)
        return out
    finally:
        master.terminate()
        try:
            master.wait(10)
        except subprocess.TimeoutExpired:
            master.kill()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="CreateFile,GetFileStatus,ListDir,DeleteFile")
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--duration", default="5s")
    ap.add_argument("--warmup", default="1s")
    ap.add_argument("--out", default=None)
    ap.add_argument("--master-prop", action="append", default=[], help="k=v master property (repeatable)")
    ap.add_argument("--client-prop", action="append", default=[], help="k=v client property (repeatable)")
    ap.add_argument("--write-type", default="MUST_CACHE", help="CreateFile/CreateDir write type")
    ap.add_argument("--ufs-sleep-ms", type=float, default=0.0, help="root UFS = sleepfs:// with this latency")
    a = ap.parse_args(argv)
    cprops = dict(kv.split("=", 1) for kv in a.client_prop)
    rows = run(a.ops.split(","), a.procs, a.threads, a.duration, a.warmup, props=a.master_prop,
               client_props=cprops, op_args=["--write-type", a.write_type], ufs_sleep_ms=a.ufs_sleep_ms)
    native = cprops.get("alluxio.user.network.native.rpc.enabled", "true").lower() != "false"
    transport = ("native framed RPC (alluxio_amd/rpc/native.py, C++ I/O threads + reply cache)" if native
                 else "gRPC (grpcio, the transport a Java client uses)")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"setup": f"1 master process + {a.procs} client processes x {a.threads} threads, "
                                f"UFS journal on local disk, {os.cpu_count()} CPUs visible",
                       "transport": transport, "write_type": a.write_type, "ufs_sleep_ms": a.ufs_sleep_ms,
                       "results": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
