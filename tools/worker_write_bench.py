#!/usr/bin/env python3
"""Host writers into a worker's cache tier from a SEPARATE client process (StressWorkerBench's
write counterpart; reference ``GrpcDataWriter`` -> ``BlockWriteHandler``).

A master + one worker (HBM tier when a GPU is visible, else DRAM) run in this process; a client
process runs T threads, each writing ``--files`` files of ``--file-size`` with MUST_CACHE from host
memory, ``--write-size`` bytes per ``write()``.  With in-process transport and short-circuit off,
every block streams to the worker's data port as gRPC ``WriteBlock``.  Reports GB/s per thread count.

    python tools/worker_write_bench.py --threads 1,4,16 --file-size 256m --out gpurun_out/ww.jsonl
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
import faulthandler, json, os, sys, threading, time
if {cpus!r}:
    os.sched_setaffinity(0, {cpus!r})     # before anything touches the GPU
sys.path.insert(0, {root!r})
if os.environ.get("WW_DUMP_AFTER"):     # debugging a stuck writer: dump every thread's stack, exit
    faulthandler.dump_traceback_later(float(os.environ["WW_DUMP_AFTER"]), exit=True)
import numpy as np
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.conf import Configuration
conf = Configuration({props!r})
fs = FileSystem(conf=conf, master_address={addr!r})
size, nfiles, threads, wsize, tag, wtype = {size}, {nfiles}, {threads}, {wsize}, {tag!r}, {wtype!r}
min_s = {min_s}
data = np.random.default_rng(1).integers(0, 256, wsize, dtype=np.uint8)
fs.create_directory("/ww", recursive=True, allow_exists=True)
with fs.create_file(f"/ww/{{tag}}-warm", write_type=wtype) as f:
    f.write(data)
done = [0] * threads
errs = []
from alluxio_amd.utils import optiming
clk = time.perf_counter
def run(t):
    try:
        k = 0
        # at least nfiles files; with min_s, keep going (reusing the nfiles names: the previous
        # file of a name is deleted first, so the cache never holds more) until min_s has passed
        while k < nfiles or time.perf_counter() - t0 < min_s:
            name = f"/ww/{{tag}}-{{t}}-{{k % nfiles}}"
            c0 = clk()
            if k >= nfiles:
                fs.delete(name)
            k += 1
            c1 = clk()
            f = fs.create_file(name, write_type=wtype)
            c2 = clk()
            left = size
            while left > 0:
                n = min(wsize, left)
                w0 = clk()
                f.write(data[:n])
                optiming.add("bench.write_call", clk() - w0)
                left -= n
                done[t] += n
            c3 = clk()
            f.close()
            c4 = clk()
            # where one file's time goes (with --client-timing)
            optiming.add("bench.delete", c1 - c0)
            optiming.add("bench.create", c2 - c1)
            optiming.add("bench.writes", c3 - c2)
            optiming.add("bench.close", c4 - c3)
    except Exception as e:
        errs.append(repr(e))
ts = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
c0 = os.times()
t0 = time.perf_counter()
for t in ts: t.start()
for t in ts: t.join()
el = time.perf_counter() - t0
c1 = os.times()
cpu = (c1.user - c0.user + c1.system - c0.system) / el
print("RESULT " + json.dumps({{"bytes": sum(done), "seconds": el, "errors": errs[:3], "client_cpu_cores": round(cpu, 2)}}), flush=True)
fs.close()
"""


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,4,16")
    ap.add_argument("--files", type=int, default=2, help="files per thread")
    ap.add_argument("--file-size", default="256m")
    ap.add_argument("--write-size", default="1m")
    ap.add_argument("--block-size", default="64m")
    ap.add_argument("--tier", default=None, help="worker MEM tier (default hbm:0 with a GPU, else dram)")
    ap.add_argument("--transports", default="grpc", help="grpc (WriteBlock on the data port) and/or ipc "
                    "(short-circuit: the worker's arena mapped into the writer, OpenDeviceWrite)")
    ap.add_argument("--write-type", default="MUST_CACHE", help="MUST_CACHE, CACHE_THROUGH or THROUGH "
                    "(the UFS is a local directory under the work dir)")
    ap.add_argument("--client-prop", action="append", default=[], help="extra client property k=v")
    ap.add_argument("--worker-prop", action="append", default=[], help="extra worker property k=v")
    ap.add_argument("--work-dir", default=None,
                    help="cluster work dir (the UFS lives under it), e.g. on /dev/shm to take the disk out")
    ap.add_argument("--client-timing", default=None,
                    help="per-phase client timing (optiming JSON, one file per run: <path>.<run>)")
    ap.add_argument("--bind-gpu-node", action="store_true",
                    help="run the worker (this process) and the client on the CPUs of the GPU's NUMA node")
    ap.add_argument("--repeat", type=int, default=1, help="runs per thread count (each row is one run)")
    ap.add_argument("--min-seconds", type=float, default=0.0,
                    help="each writer keeps writing files (deleting its oldest) for at least this long")
    ap.add_argument("--s3", action="store_true", help="/ww is an S3 mount (a native BlobServer on tmpfs, "
                    "64 MiB parts): THROUGH / CACHE_THROUGH go to object storage")
    ap.add_argument("--py-sample", action="store_true",
                    help="sample the bench process's Python stacks (attribution of its interpreter CPU)")
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
            os.sched_setaffinity(0, cpus)          # the in-process worker's threads inherit it
    if a.client_timing:
        # the master's and worker's handlers too (this process), dumped at exit
        os.environ.setdefault("ALLUXIO_MASTER_OP_TIMING", f"{a.client_timing}.server")
    import torch

    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.utils.format import parse_space_size
    tier = a.tier or ("hbm:0" if torch.cuda.is_available() else "dram")
    size = parse_space_size(a.file_size)
    total = max(int(t) for t in a.threads.split(",")) * a.files * size
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": tier,
            "alluxio.worker.tieredstore.level0.dirs.quota": str(total + (1 << 30)),
            "alluxio.worker.hbm.page.size": "2MB",
            "alluxio.user.block.size.bytes.default": a.block_size,
            "alluxio.security.authorization.permission.enabled": "false",
            "alluxio.worker.tieredstore.dram.prefault": str(a.write_type != "THROUGH").lower()}
    conf.update(dict(kv.split("=", 1) for kv in a.worker_prop))
    work = tempfile.mkdtemp(prefix="wwbench_", dir=a.work_dir)
    blob = None
    if a.s3:
        import requests

        from alluxio_amd.ops.native import lib
        blob_root = tempfile.mkdtemp(prefix="wwblob_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        blob = lib().BlobServer(blob_root, "127.0.0.1", 0)
        blob.start()
        endpoint = f"http://127.0.0.1:{blob.port}"
        requests.put(endpoint + "/bkt")
        requests.put(endpoint + "/bkt/ww/")
    with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=work) as c:
        if blob is not None:
            c.client().mount("/ww", "s3://bkt/ww", properties={
                "alluxio.underfs.s3.endpoint": endpoint,
                "alluxio.underfs.s3.streaming.upload.partition.size": "64MB",
                "alluxio.underfs.object.store.upload.buffer.size": "256MB"})
        time.sleep(min(10.0, total / 4e9))     # let the DRAM prefault finish (no-op on HBM)
        runs = [(tr, t) for tr in a.transports.split(",") for t in a.threads.split(",")
                for _ in range(max(1, a.repeat))]
        for i, (transport, t) in enumerate(runs):
            props = {"alluxio.user.network.inprocess.transport.enabled": "false",
                     "alluxio.user.short.circuit.enabled": "true" if transport == "ipc" else "false",
                     "alluxio.user.block.size.bytes.default": a.block_size}
            props.update(dict(kv.split("=", 1) for kv in a.client_prop))
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            from _threadcpu import StackSampler, busy, python_thread_cpu, python_user_sys, thread_cpu
            tc0, tw0 = thread_cpu(), time.perf_counter()
            pc0 = python_thread_cpu()
            pus0 = python_user_sys()
            sampler = StackSampler().start() if a.py_sample else None
            ds = getattr(c.workers[0], "data_server", None)
            tee0 = ds.stats.ufs_tee_bytes if ds is not None else 0
            cenv = dict(os.environ)
            if a.client_timing:
                cenv["ALLUXIO_MASTER_OP_TIMING"] = f"{a.client_timing}.{a.write_type}.t{t}"
            p = subprocess.run([sys.executable, "-c", CLIENT.format(
                root=ROOT, props=props, addr=c.master.address, size=size, nfiles=a.files, threads=int(t),
                wsize=parse_space_size(a.write_size), tag=f"r{i}", wtype=a.write_type, cpus=cpus,
                min_s=a.min_seconds)],
                capture_output=True, text=True, timeout=900, env=cenv)
            line = next((ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")), None)
            if line is None:
                print(p.stdout[-2000:], p.stderr[-3000:], file=sys.stderr)
                return 1
            r = json.loads(line[7:])
            worker_threads = busy(tc0, thread_cpu(), r["seconds"])   # over the client's timed window
            py_threads = busy(pc0, python_thread_cpu(), r["seconds"])
            pus1 = python_user_sys()
            samples = sampler.stop() if sampler is not None else None
            row = {"bench": f"host writers, separate client process ({a.write_type})", "transport": transport, "tier": tier,
                   "min_seconds": a.min_seconds,
                   "threads": int(t), "files_per_thread": a.files, "file_size": a.file_size,
                   "write_size": a.write_size, "bytes": r["bytes"], "seconds": round(r["seconds"], 3),
                   "GBps": round(r["bytes"] / r["seconds"] / 1e9, 3), "errors": r["errors"],
                   "client_props": a.client_prop, "worker_props": a.worker_prop,
                   # worker process CPU by thread group during the run (approx: whole subprocess
                   # lifetime / timed window), and the client's own CPU over its timed window
                   "worker_thread_cores": worker_threads, "client_cpu_cores": r.get("client_cpu_cores"),
                   "python_thread_cores": py_threads,
                   # the same threads split into user (interpreter) and system (syscall) time
                   "python_user_cores": round((pus1[0] - pus0[0]) / r["seconds"], 2),
                   "python_sys_cores": round((pus1[1] - pus0[1]) / r["seconds"], 2),
                   "bound_to_gpu_node": bool(cpus), "work_dir": work, "ufs": "s3" if a.s3 else "local",
                   # bytes the worker copied from its block store into UFS files (CACHE_THROUGH tee)
                   "ufs_tee_bytes": (ds.stats.ufs_tee_bytes - tee0) if ds is not None else None}
            if samples is not None:
                row["python_stack_samples"] = samples
            if ds is not None:
                row["native_commits"] = ds.stats.commits
                row["native_commit_batches"] = ds.stats.commit_batches
            print(json.dumps(row), flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(json.dumps(row) + "\n")
            # free the cache for the next thread count
            fs = c.client()
            for st in fs.list_status("/ww"):
                fs.delete(st.path)
            fs.close()
    if blob is not None:
        import shutil
        blob.stop()
        shutil.rmtree(blob_root, ignore_errors=True)
    if a.work_dir:
        import shutil
        shutil.rmtree(work, ignore_errors=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
