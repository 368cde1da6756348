#!/usr/bin/env python3
"""Persist throughput: cached files copied to their local UFS by the persist job's task
(``job/persist.py``), the ASYNC_THROUGH path (reference PersistDefinition: read through the client,
write the UFS file).

Two ways per thread count:
* ``append``  -- the worker holding the blocks appends them from its store to the file's native UFS
                 stream (``AppendBlock``); no file bytes pass through the persisting process;
* ``client``  -- the reference shape: read the file through the client (native gRPC reader) and
                 write it to the UFS from this process.

    python tools/persist_bench.py --threads 1,4 --files 4 --file-size 1g --out gpurun_out/persist.jsonl
    python tools/persist_bench.py --ufs s3 --threads 1,4 --files 2 --file-size 1g
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,4")
    ap.add_argument("--files", type=int, default=4, help="files per thread")
    ap.add_argument("--file-size", default="1g")
    ap.add_argument("--block-size", default="64m")
    ap.add_argument("--modes", default="append,client")
    ap.add_argument("--ufs", default="local", help="local (the root mount's directory) or s3 (a native "
                    "BlobServer mounted at /p; parts of --s3-part)")
    ap.add_argument("--s3-part", default="16MB")
    ap.add_argument("--work-dir", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)

    import numpy as np
    import torch

    from alluxio_amd.client.file_system import FileSystem
    from alluxio_amd.conf import Configuration
    from alluxio_amd.job.persist import persist_file
    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.utils.format import parse_space_size

    gpu = torch.cuda.is_available()
    size = parse_space_size(a.file_size)
    threads = [int(t) for t in a.threads.split(",")]
    total = max(threads) * a.files * size
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "hbm:0" if gpu else "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": str(total + (1 << 30)),
            "alluxio.worker.hbm.page.size": "2MB",
            "alluxio.user.block.size.bytes.default": a.block_size,
            "alluxio.security.authorization.permission.enabled": "false"}
    work = tempfile.mkdtemp(prefix="persist_", dir=a.work_dir)
    src = np.random.default_rng(3).integers(0, 256, size, dtype=np.uint8)
    blob = None
    if a.ufs == "s3":
        from alluxio_amd.ops.native import lib
        blob = lib().BlobServer(os.path.join(work, "blobs"), "127.0.0.1", 0)
        blob.start()
        import requests
        endpoint = f"http://127.0.0.1:{blob.port}"
        requests.put(endpoint + "/bkt")
        requests.put(endpoint + "/bkt/p/")
    with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=work) as c:
        ds = c.workers[0].data_server
        if blob is not None:
            c.client().mount("/p", "s3://bkt/p", properties={
                "alluxio.underfs.s3.endpoint": endpoint,
                "alluxio.underfs.s3.streaming.upload.partition.size": a.s3_part,
                "alluxio.underfs.object.store.upload.buffer.size": str(4 * parse_space_size(a.s3_part))})

        def ufs_bytes(n):
            if blob is None:
                with open(fs.get_status(n).info.ufsPath.replace("file://", ""), "rb") as fh:
                    return fh.read()
            return requests.get(endpoint + "/bkt/p/" + n.split("/p/", 1)[1]).content
        for mode in a.modes.split(","):
            props = {"alluxio.user.network.inprocess.transport.enabled": "false",
                     "alluxio.user.short.circuit.enabled": "false",
                     "alluxio.user.block.size.bytes.default": a.block_size,
                     "alluxio.job.persist.worker.append.enabled": str(mode == "append").lower()}
            fs = FileSystem(conf=Configuration(props), master_address=c.master.address)
            fs.write_file(f"/p/warm-{mode}", b"w" * 100, write_type="CACHE_THROUGH")   # registers the mount natively
            for t in threads:
                names = [f"/p/{mode}-t{t}-{i}-{k}" for i in range(t) for k in range(a.files)]
                for n in names:
                    fs.write_file(n, src, write_type="MUST_CACHE")
                tee0 = ds.stats.ufs_tee_bytes if ds is not None else 0
                done, errs = [0] * t, []

                def run(i):
                    try:
                        for k in range(a.files):
                            done[i] += persist_file(fs, f"/p/{mode}-t{t}-{i}-{k}")
                    except Exception as e:  # noqa: BLE001
                        errs.append(repr(e))
                c0 = os.times()
                t0 = time.perf_counter()
                ts = [threading.Thread(target=run, args=(i,)) for i in range(t)]
                for th in ts:
                    th.start()
                for th in ts:
                    th.join()
                el = time.perf_counter() - t0
                c1 = os.times()
                ok = True
                for n in names[:2]:                  # spot-check the persisted bytes
                    ok = ok and ufs_bytes(n) == src.tobytes()
                row = {"bench": "persist (ASYNC_THROUGH job task) of cached files to a local UFS", "mode": mode,
                       "threads": t, "files": len(names), "file_size": a.file_size, "bytes": sum(done),
                       "seconds": round(el, 3), "GBps": round(sum(done) / el / 1e9, 3), "errors": errs[:3],
                       "verified": ok, "process_cpu_cores": round((c1.user - c0.user + c1.system - c0.system) / el, 2),
                       "ufs_tee_bytes": (ds.stats.ufs_tee_bytes - tee0) if ds is not None else None,
                       "tier": conf["alluxio.worker.tieredstore.level0.dirs.path"], "ufs": a.ufs}
                print(json.dumps(row), flush=True)
                if a.out:
                    with open(a.out, "a") as f:
                        f.write(json.dumps(row) + "\n")
                for n in names:
                    fs.delete(n)
            fs.close()
    if blob is not None:
        blob.stop()
    shutil.rmtree(work, ignore_errors=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
