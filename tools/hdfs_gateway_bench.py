#!/usr/bin/env python3
"""Read throughput through the HDFS-protocol gateway (proxy/hdfs_gateway.py) with this
repository's Hadoop client, in a SEPARATE client process (as a Spark/Hive task would be).

A cluster (HBM tier when a GPU is visible, else DRAM) caches a file; the gateway serves it as
hdfs://127.0.0.1:<port>/; T client threads each read the whole file sequentially through
``HdfsUnderFileSystem.open`` in ``--read-size`` pieces.  Reports GB/s and whether the DataNode
used the native packet sender (csrc/hdfs_packets.cpp).  Reference: HdfsFileInputStream.java:103-139
(reads at block-stream speed).

    python tools/hdfs_gateway_bench.py --file-size 1g --threads 1,4 --out gpurun_out/hdfs_gateway.jsonl
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
import json, sys, threading, time
sys.path.insert(0, {root!r})
from alluxio_amd.underfs.registry import create
ufs = create("hdfs://127.0.0.1:{port}/", properties={{"dfs.blocksize": "64m"}})
size = {size}
threads = {threads}
read = {read}
done = [0] * threads
def run(i):
    buf = bytearray(read)
    with ufs.open("/bench/data") as f:
        while True:
            n = f.readinto(buf)
            if not n:
                break
            done[i] += n
from alluxio_amd.ops.native import lib as _lib
_lib()                                  # native library load + first connection outside the timing
with ufs.open("/bench/data") as f:
    f.readinto(bytearray(min(read, size)))
ts = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
t0 = time.perf_counter()
for t in ts: t.start()
for t in ts: t.join()
el = time.perf_counter() - t0
print("RESULT " + json.dumps({{"bytes": sum(done), "seconds": el}}), flush=True)
"""


WRITER = r"""
import json, sys, threading, time
sys.path.insert(0, {root!r})
import numpy as np
from alluxio_amd.underfs.registry import create
from alluxio_amd.ops.native import lib as _lib
_lib()
ufs = create("hdfs://127.0.0.1:{port}/", properties={{"dfs.blocksize": "64m"}})
size, threads, wsize = {size}, {threads}, {wsize}
data = np.random.default_rng(1).integers(0, 256, wsize, dtype=np.uint8).tobytes()
with ufs.create("/wbench/warm-{tag}") as f:
    f.write(data[:1 << 20])
done = [0] * threads
def run(i):
    with ufs.create(f"/wbench/{tag}-{{i}}") as f:
        left = size
        while left > 0:
            n = min(wsize, left)
            f.write(data[:n])
            left -= n
            done[i] += n
ts = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
t0 = time.perf_counter()
for t in ts: t.start()
for t in ts: t.join()
el = time.perf_counter() - t0
print("RESULT " + json.dumps({{"bytes": sum(done), "seconds": el}}), flush=True)
"""


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--file-size", default="1g")
    ap.add_argument("--threads", default="1,4")
    ap.add_argument("--read-size", default="4m")
    ap.add_argument("--write-threads", default="1,4", help="writer threads per run ('' = no write runs)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    import numpy as np
    import torch

    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.proxy.hdfs_gateway import HdfsGateway
    from alluxio_amd.utils.format import parse_space_size
    size = parse_space_size(a.file_size)
    gpu = torch.cuda.is_available()
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "hbm:0" if gpu else "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": str(size * 5 + (512 << 20)),
            "alluxio.worker.tieredstore.dram.prefault": "true",
            "alluxio.worker.hbm.page.size": "2MB", "alluxio.user.block.size.bytes.default": "64MB",
            "alluxio.security.authorization.permission.enabled": "false"}
    work = tempfile.mkdtemp(prefix="hdfsgw_")
    with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=work) as c:
        fs = c.client()
        fs.write_file("/bench/data", np.random.default_rng(0).integers(0, 256, size, dtype=np.uint8),
                      write_type="MUST_CACHE")
        g = HdfsGateway(fs)
        try:
            for t in a.threads.split(","):
                calls0 = dict(g.calls)
                p = subprocess.run([sys.executable, "-c", CLIENT.format(root=ROOT, port=g.port, size=size,
                                                                       threads=int(t),
                                                                       read=parse_space_size(a.read_size))],
                                   capture_output=True, text=True, timeout=900)
                line = next((ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")), None)
                if line is None:
                    print(p.stdout[-2000:], p.stderr[-3000:], file=sys.stderr)
                    return 1
                r = json.loads(line[7:])
                row = {"bench": "HDFS gateway read (separate Hadoop-client process)", "tier": conf[
                    "alluxio.worker.tieredstore.level0.dirs.path"], "file_size": a.file_size, "threads": int(t),
                       "read_size": a.read_size, "bytes": r["bytes"], "seconds": round(r["seconds"], 3),
                       "GBps": round(r["bytes"] / r["seconds"] / 1e9, 3),
                       "getBlockLocations": g.calls.get("getBlockLocations", 0) - calls0.get("getBlockLocations", 0)}
                print(json.dumps(row), flush=True)
                if a.out:
                    with open(a.out, "a") as f:
                        f.write(json.dumps(row) + "\n")
            # writes: separate Hadoop-client process, one file per thread (MUST_CACHE gateway)
            gw = HdfsGateway(fs, write_type="MUST_CACHE")
            try:
                for i, t in enumerate(x for x in a.write_threads.split(",") if x):
                    p = subprocess.run([sys.executable, "-c", WRITER.format(
                        root=ROOT, port=gw.port, size=size, threads=int(t), wsize=parse_space_size(a.read_size),
                        tag=f"w{i}")], capture_output=True, text=True, timeout=900)
                    line = next((ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")), None)
                    if line is None:
                        print(p.stdout[-2000:], p.stderr[-3000:], file=sys.stderr)
                        return 1
                    r = json.loads(line[7:])
                    row = {"bench": "HDFS gateway write (separate Hadoop-client process, MUST_CACHE)",
                           "tier": conf["alluxio.worker.tieredstore.level0.dirs.path"], "file_size": a.file_size,
                           "threads": int(t), "write_size": a.read_size, "bytes": r["bytes"],
                           "seconds": round(r["seconds"], 3), "GBps": round(r["bytes"] / r["seconds"] / 1e9, 3)}
                    print(json.dumps(row), flush=True)
                    if a.out:
                        with open(a.out, "a") as f:
                            f.write(json.dumps(row) + "\n")
                    for st in fs.list_status("/wbench"):
                        fs.delete(st.path)
            finally:
                gw.stop()
        finally:
            g.stop()
            fs.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
