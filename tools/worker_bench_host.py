#!/usr/bin/env python3
"""Literal StressWorkerBench host readers against an HBM-tier worker (reference shape).

The reference's StressWorkerBench runs T Java threads, each looping ``read(buf)`` through
``FileInStream`` (stress/shell/.../StressWorkerBench.java:251-276, WorkerBenchParameters.java:40-70).
This harness starts a master + one worker whose MEM tier is HBM (``hbm:0``) in this process, then
runs ``alluxio_amd.stress.worker_bench --mode threads`` in a SEPARATE client process -- so every
byte crosses a process boundary the way a Java client's does -- once per transport:

* ``grpc``: short-circuit off; blocks stream over gRPC ``ReadBlock`` from the worker's native data
  port (csrc/data_server.cpp: HBM chunks DMA'd into pinned staging on the C++ I/O threads,
  ``offset_received`` flow control) into the client's native reader (csrc/block_source.cpp:
  HTTP/2 frames parsed into a chunk buffer; each ``read(buf)`` is a memcpy out of it);
* ``ipc``: short-circuit on; the client maps the worker's HBM arena through HIP IPC
  (``OpenDeviceBlock``), DMAs chunks D2H into a pinned buffer and serves each ``read(buf)`` from it;
* ``grpcio``: the pre-native path for comparison -- the grpcio client's ``ReadBlock`` against the
  worker's Python grpcio servicer (``alluxio.user.native.reader.enabled=false``).

    python tools/worker_bench_host.py --threads 32 --duration 10s --warmup 3s --out gpurun_out/wb.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CLIENT = r"""
import json, os, sys, faulthandler
faulthandler.enable()
if {cpus!r}:
    os.sched_setaffinity(0, {cpus!r})     # before anything touches the GPU
sys.path.insert(0, {root!r})
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.conf import Configuration
from alluxio_amd.stress import worker_bench
conf = Configuration({props!r})
fs = FileSystem(conf=conf, master_address={addr!r}, metadata_cache=True)
r = worker_bench.main({args!r}, fs=fs, print_result=False)
from alluxio_amd.ops.native import lib
r["placement"] = lib().process_placement()
print("RESULT " + json.dumps(r), flush=True)
fs.close()
"""

# Same-run D2H roof: N processes, started together, each copying a 64 MiB device buffer into a
# pinned host buffer (hipMemcpyAsync D2H + sync) for 2 s -- the platform ceiling the short-circuit
# readers' D2H refills share.
ROOF = r"""
import json, os, sys, time
if {cpus!r}:
    os.sched_setaffinity(0, {cpus!r})
sys.path.insert(0, {root!r})
import torch
from alluxio_amd.ops.native import lib
start = {start!r}
src = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
dst = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
dst.copy_(src, non_blocking=True); torch.cuda.synchronize()
while time.time() < start:
    time.sleep(0.001)
n, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < 2.0:
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    n += 1
el = time.perf_counter() - t0
print("ROOF " + json.dumps({{"GBps": n * (64 << 20) / el / 1e9, "placement": lib().process_placement(),
                            "gpu_numa_node": lib().gpu_numa_node(0)}}), flush=True)
"""


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="256", help="comma list of thread counts")
    ap.add_argument("--file-size", default="128m")
    ap.add_argument("--buffer-size", default="4k")
    ap.add_argument("--block-size", default="64m")
    ap.add_argument("--duration", default="10s")
    ap.add_argument("--warmup", default="3s")
    ap.add_argument("--transports", default="grpc,ipc")
    ap.add_argument("--mode", default="threads", choices=("threads", "native-threads"),
                    help="Python reader threads (FileInStream) or the native C++ reader threads")
    ap.add_argument("--tier", default="hbm:0", help="worker MEM tier dir (hbm:N or dram)")
    ap.add_argument("--reader-buffer", default="4MB", help="alluxio.user.native.reader.buffer.size")
    ap.add_argument("--client-prop", action="append", default=[], help="extra client property k=v")
    ap.add_argument("--client-procs", type=int, default=1,
                    help="spread the threads over this many client processes (the reference's --clients "
                         "makes N FileSystem instances in one JVM; Python instances in one interpreter "
                         "share one lock, so they go to separate processes); throughput is summed")
    ap.add_argument("--bind-gpu-node", action="store_true",
                    help="run the client (and roof) processes on the CPUs of the GPU's NUMA node")
    ap.add_argument("--d2h-roof", action="store_true",
                    help="after each run, the same number of processes measure the D2H copy roof together")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    cpus = []
    if a.bind_gpu_node:
        from alluxio_amd.ops.native import lib
        node = lib().gpu_numa_node(0)
        if node >= 0:
            with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
                for part in f.read().strip().split(","):
                    lo, _, hi = part.partition("-")
                    cpus.extend(range(int(lo), int(hi or lo) + 1))
            cpus = sorted(set(cpus) & os.sched_getaffinity(0))

    from alluxio_amd.minicluster import LocalAlluxioCluster
    import numpy as np
    from alluxio_amd.utils.format import parse_space_size
    work = tempfile.mkdtemp(prefix="wbench_")
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": a.tier,
            "alluxio.worker.tieredstore.level0.dirs.quota": "4GB",
            "alluxio.worker.hbm.page.size": "2MB",
            "alluxio.user.block.size.bytes.default": a.block_size,
            "alluxio.security.authorization.permission.enabled": "false"}
    rows = []
    with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=work) as c:
        fs = c.client()
        size = parse_space_size(a.file_size)
        fs.create_directory("/stress-worker-base", recursive=True, allow_exists=True)
        fs.write_file("/stress-worker-base/data", np.full(size, ord("A"), dtype=np.uint8),
                      write_type="CACHE_THROUGH", block_size=parse_space_size(a.block_size))
        st = fs.get_status("/stress-worker-base/data")
        assert st.in_alluxio_percentage == 100
        stats = c.workers[0].data_server.stats if c.workers[0].data_server is not None else None
        for transport in a.transports.split(","):
            props = {"alluxio.user.network.inprocess.transport.enabled": "false",
                     "alluxio.user.short.circuit.enabled": "true" if transport == "ipc" else "false",
                     "alluxio.user.native.reader.enabled": "false" if transport == "grpcio" else "true",
                     "alluxio.user.native.reader.buffer.size": a.reader_buffer,
                     "alluxio.user.file.passive.cache.enabled": "false"}
            props.update(dict(kv.split("=", 1) for kv in a.client_prop))
            for t in a.threads.split(","):
                nproc = max(1, a.client_procs)
                per = max(1, int(t) // nproc)
                args = ["--threads", str(per), "--file-size", a.file_size, "--buffer-size", a.buffer_size,
                        "--block-size", a.block_size, "--duration", a.duration, "--warmup", a.warmup,
                        "--mode", a.mode]
                t0 = time.time()
                sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
                from _threadcpu import busy, thread_cpu
                tc0 = thread_cpu()
                s0 = (stats.streams, stats.bytes, stats.declined) if stats is not None else (0, 0, 0)
                procs = [subprocess.Popen([sys.executable, "-c", CLIENT.format(root=ROOT, addr=c.master.address,
                                                                              args=args, props=props, cpus=cpus)],
                                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                         for _ in range(nproc)]
                results = []
                for p in procs:
                    out, err = p.communicate(timeout=600)
                    line = next((ln for ln in out.splitlines() if ln.startswith("RESULT ")), None)
                    if line is None:
                        print(f"client process ({transport}, {t} threads) exited rc={p.returncode} without a result",
                              file=sys.stderr)
                        print(out[-2000:], file=sys.stderr)
                        print(err[-3000:], file=sys.stderr)
                        return 1
                    results.append(json.loads(line[7:]))
                # the worker's threads (this process) over the clients' lifetime, by name group
                worker_cores = busy(tc0, thread_cpu(), time.time() - t0)
                r = {"throughput_MBps": sum(x["throughput_MBps"] for x in results),
                     "bytes": sum(x["bytes"] for x in results), "duration_s": results[0]["duration_s"],
                     "errors": [e for x in results for e in x["errors"]]}
                row = {"bench": f"StressWorkerBench --mode {a.mode} (host readers, separate client process)",
                       "transport": transport, "tier": a.tier, "threads": per * nproc, "buffer": a.buffer_size,
                       "file_size": a.file_size, "block_size": a.block_size,
                       "throughput_MBps": round(r["throughput_MBps"], 1), "bytes": r["bytes"],
                       "duration_s": r["duration_s"], "errors": r["errors"], "wall_s": round(time.time() - t0, 1),
                       "reader_buffer": a.reader_buffer, "client_props": a.client_prop,
                       "client_procs": nproc}
                row["client_placement"] = [x.get("placement", "") for x in results]
                row["worker_thread_cores"] = worker_cores
                if results[0].get("native"):
                    row["native"] = [x.get("native") for x in results]
                row["bound_to_gpu_node"] = bool(cpus)
                row["reader_buffer"] = a.reader_buffer
                if a.d2h_roof:
                    start = time.time() + 8.0       # all roof processes start copying together
                    rp = [subprocess.Popen([sys.executable, "-c", ROOF.format(root=ROOT, start=start, cpus=cpus)],
                                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                          for _ in range(nproc)]
                    roofs = []
                    for p in rp:
                        out, err = p.communicate(timeout=120)
                        line = next((ln for ln in out.splitlines() if ln.startswith("ROOF ")), None)
                        if line:
                            roofs.append(json.loads(line[5:]))
                    row["d2h_roof_GBps"] = round(sum(x["GBps"] for x in roofs), 2)
                    row["d2h_roof_per_proc"] = [round(x["GBps"], 2) for x in roofs]
                    row["roof_placement"] = [x["placement"] for x in roofs]
                    row["gpu_numa_node"] = roofs[0]["gpu_numa_node"] if roofs else None
                    row["fraction_of_roof"] = round(r["throughput_MBps"] / 1e3 / row["d2h_roof_GBps"], 3) \
                        if row["d2h_roof_GBps"] else None
                if stats is not None:
                    row["data_server"] = {"native_streams": stats.streams - s0[0],
                                          "native_bytes": stats.bytes - s0[1],
                                          "bridged_streams": stats.declined - s0[2]}
                print(json.dumps(row), flush=True)
                rows.append(row)
                if a.out:
                    with open(a.out, "a") as f:
                        f.write(json.dumps(row) + "\n")
        fs.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
