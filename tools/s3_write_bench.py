#!/usr/bin/env python3
"""Object-store write throughput and memory bound (THROUGH into an S3 mount).

The S3 endpoint is this build's native BlobServer (csrc/http_blob.cpp) over ``--blob-root``
(tmpfs on the GPU box by default, so the disk does not bound the number).  Two paths:

* ``ufs``: the S3 under file system's own writer (``create()`` -> bounded multipart upload of
  ``alluxio.underfs.s3.streaming.upload.partition.size`` parts, native PUT from the part buffer),
  streaming or spooled (``--spool``), in this process;
* ``through``: a client in a separate process writes the file THROUGH an Alluxio worker whose
  data server streams it to the bucket as a multipart upload (csrc/data_server.cpp
  S3UfsWriteStream); the first file registers the mount through the Python servicer.

Each row reports GB/s (bytes / wall time up to the completed object) and the growth of this
process's resident set during the write (``rss_growth_MiB``: the worker and the endpoint live in
it; sampled every 20 ms).

    python tools/s3_write_bench.py --size 8g --paths ufs,through --out gpurun_out/s3_write.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CLIENT = r"""
import json, sys, time
sys.path.insert(0, {root!r})
import numpy as np
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.conf import Configuration
fs = FileSystem(conf=Configuration({props!r}), master_address={addr!r})
chunk = np.random.default_rng(2).integers(0, 256, {wsize}, dtype=np.uint8)
fs.write_file("/s3/warm", chunk[:1 << 20], write_type="THROUGH")     # registers the mount natively
t0 = time.perf_counter()
with fs.create_file("/s3/data", write_type={wtype!r}) as f:
    left = {size}
    while left > 0:
        n = min(left, chunk.nbytes)
        f.write(chunk[:n])
        left -= n
el = time.perf_counter() - t0
print("RESULT " + json.dumps({{"seconds": el}}), flush=True)
fs.close()
"""


def rss_mib() -> float:
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024.0
    return 0.0


class RssSampler:
    def __init__(self):
        self.base = rss_mib()
        self.peak = self.base
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        while not self._stop.wait(0.02):
            self.peak = max(self.peak, rss_mib())

    def stop(self) -> float:
        self._stop.set()
        self._t.join()
        return self.peak - self.base


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="8g")
    ap.add_argument("--write-size", default="64m", help="bytes per write() call")
    ap.add_argument("--paths", default="ufs,through")
    ap.add_argument("--part", default="64MB")
    ap.add_argument("--buffer", default="256MB", help="alluxio.underfs.object.store.upload.buffer.size")
    ap.add_argument("--spool", action="store_true", help="ufs path: spooled (reference default) writer")
    ap.add_argument("--blob-root", default=None)
    ap.add_argument("--write-type", default="THROUGH", help="through path: THROUGH or CACHE_THROUGH")
    ap.add_argument("--tier", default="dram", help="through path: the worker's MEM tier (dram, hbm:0)")
    ap.add_argument("--client-prop", action="append", default=[], help="through path: client property k=v")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    import numpy as np
    import requests

    from alluxio_amd.ops.native import lib
    from alluxio_amd.utils.format import parse_space_size
    size = parse_space_size(a.size)
    wsize = parse_space_size(a.write_size)
    root = a.blob_root or tempfile.mkdtemp(prefix="s3wb_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    os.makedirs(root, exist_ok=True)
    srv = lib().BlobServer(root, "127.0.0.1", 0)
    srv.start()
    base = f"http://127.0.0.1:{srv.port}"
    requests.put(base + "/bkt")
    requests.put(base + "/bkt/out/")
    props = {"alluxio.underfs.s3.endpoint": base, "alluxio.underfs.s3.streaming.upload.partition.size": a.part,
             "alluxio.underfs.object.store.upload.buffer.size": a.buffer,
             "alluxio.underfs.s3.streaming.upload.enabled": "false" if a.spool else "true"}
    rows = []
    try:
        for path in a.paths.split(","):
            if path == "ufs":
                from alluxio_amd.underfs.registry import create as create_ufs
                ufs = create_ufs("s3://bkt/", properties=props)
                chunk = np.random.default_rng(1).integers(0, 256, wsize, dtype=np.uint8)
                samp = RssSampler()
                t0 = time.perf_counter()
                w = ufs.create("s3://bkt/out/ufs-data")
                left = size
                while left > 0:
                    n = min(left, wsize)
                    w.write(chunk[:n])
                    left -= n
                w.close()
                el = time.perf_counter() - t0
                growth = samp.stop()
                extra = {"parts": w.parts_uploaded, "part_buffers": w.buffers_allocated,
                         "writer": "spooled" if a.spool else "streaming", **w.timings}
                del chunk
            else:
                from alluxio_amd.minicluster import LocalAlluxioCluster
                conf = {"alluxio.worker.tieredstore.level0.dirs.path": a.tier,
                        "alluxio.worker.tieredstore.level0.dirs.quota": str(size + (1 << 30)),
                        "alluxio.user.block.size.bytes.default": "64MB",
                        "alluxio.security.authorization.permission.enabled": "false"}
                with LocalAlluxioCluster(num_workers=1, conf=conf,
                                         work_dir=tempfile.mkdtemp(prefix="s3wb_cluster_")) as c:
                    fs = c.client()
                    fs.mount("/s3", "s3://bkt/out", properties=props)
                    cprops = {"alluxio.user.network.inprocess.transport.enabled": "false",
                              "alluxio.user.short.circuit.enabled": "false",
                              **dict(kv.split("=", 1) for kv in a.client_prop)}
                    samp = RssSampler()
                    p = subprocess.run([sys.executable, "-c", CLIENT.format(
                        root=ROOT, props=cprops, addr=c.master.address, size=size, wsize=min(wsize, 4 << 20),
                        wtype=a.write_type)],
                        capture_output=True, text=True, timeout=900)
                    growth = samp.stop()
                    line = next((ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")), None)
                    if line is None:
                        print(p.stdout[-2000:], p.stderr[-3000:], file=sys.stderr)
                        return 1
                    el = json.loads(line[7:])["seconds"]
                    st = c.workers[0].data_server.stats
                    extra = {"native_ufs_write_streams": st.ufs_write_streams, "native_ufs_write_bytes": st.ufs_write_bytes,
                             "ufs_tee_bytes": st.ufs_tee_bytes, "write_type": a.write_type, "tier": a.tier,
                             "client_props": a.client_prop}
                    fs.close()
            got = requests.head(f"{base}/bkt/out/{'ufs-data' if path == 'ufs' else 'data'}")
            row = {"bench": "THROUGH write into an S3 mount (native BlobServer endpoint on "
                            f"{'tmpfs' if root.startswith('/dev/shm') else 'disk'})",
                   "path": path, "bytes": size, "seconds": round(el, 3), "GBps": round(size / el / 1e9, 3),
                   "rss_growth_MiB": round(growth, 1), "part": a.part, "buffer": a.buffer,
                   "object_size_ok": int(got.headers.get("Content-Length", -1)) == size, **extra}
            rows.append(row)
            print(json.dumps(row), flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(json.dumps(row) + "\n")
            for k in ("ufs-data", "data", "warm"):
                requests.delete(f"{base}/bkt/out/{k}")
    finally:
        srv.stop()
        if a.blob_root is None:
            shutil.rmtree(root, ignore_errors=True)
    return 0 if all(r["object_size_ok"] for r in rows) else 2


if __name__ == "__main__":
    raise SystemExit(main())
