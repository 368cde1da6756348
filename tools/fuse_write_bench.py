#!/usr/bin/env python3
"""Sequential writes through the FUSE mount (reference integration/fuse AlluxioFuseFileSystem
write/flush/release): a separate process writes ``--files`` files of ``--file-size`` in 1 MiB
``write()`` calls under the mount, with the native server's write-behind (8 MiB batches answered in
C++, one outstanding batch per handle) on and off, and the pure-Python request loop for reference.

Needs /dev/fuse and the right to mount (root / CAP_SYS_ADMIN), so it runs in a container, not on
the GPU pool's user boxes.

    python tools/fuse_write_bench.py --files 8 --file-size 64m --out profiles/r5_fuse_write.jsonl
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

WRITER = r"""
import json, os, time
m, n, size = {mnt!r}, {files}, {size}
os.makedirs(m + "/w", exist_ok=True)
chunk = os.urandom(1 << 20)
t = time.perf_counter()
for i in range(n):
    with open(f"{{m}}/w/{{i}}.bin", "wb") as f:
        left = size
        while left > 0:
            k = min(left, len(chunk))
            f.write(chunk[:k])
            left -= k
el = time.perf_counter() - t
print(json.dumps({{"seconds": el}}))
"""


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--file-size", default="64m")
    ap.add_argument("--modes", default="write_behind,native_sync,python")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    from alluxio_amd.fuse import AlluxioFuseOps
    from alluxio_amd.fuse.kernel import mount_kernel
    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.utils.format import parse_space_size
    size = parse_space_size(a.file_size)
    for mode in a.modes.split(","):
        work = tempfile.mkdtemp(prefix="fusewb_")
        mnt = os.path.join(work, "mnt")
        os.makedirs(mnt)
        conf = {"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                "alluxio.worker.tieredstore.level0.dirs.quota": str(a.files * size + (1 << 30)),
                "alluxio.user.block.size.bytes.default": "64MB",
                "alluxio.user.file.writetype.default": "MUST_CACHE",
                "alluxio.worker.tieredstore.dram.prefault": "true"}
        with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=os.path.join(work, "c")) as c:
            time.sleep(min(10.0, a.files * size / 2e9))      # let the arena prefault finish
            fs = c.client()
            srv = mount_kernel(AlluxioFuseOps(fs), mnt, threads=2, native=(mode != "python"),
                               write_behind=(mode == "write_behind"))
            try:
                p = subprocess.run([sys.executable, "-c", WRITER.format(mnt=mnt, files=a.files, size=size)],
                                   capture_output=True, text=True, timeout=600)
                if p.returncode != 0:
                    print(p.stderr[-2000:], file=sys.stderr)
                    return 1
                el = json.loads(p.stdout.strip().splitlines()[-1])["seconds"]
                ok = all(fs.get_status(f"/w/{i}.bin").length == size for i in range(a.files))
                stats = srv.op_stats() if hasattr(srv, "op_stats") else {}
                row = {"bench": "FUSE sequential writes, 1 MiB write() calls (MUST_CACHE, DRAM tier)",
                       "mode": mode, "files": a.files, "file_size": a.file_size, "seconds": round(el, 3),
                       "GBps": round(a.files * size / el / 1e9, 3), "lengths_ok": ok,
                       "python_write_ops": (stats.get("python") or {}).get("WRITE", 0),
                       "write_batches": getattr(getattr(srv, "_srv", None), "write_batches", None)}
                print(json.dumps(row), flush=True)
                if a.out:
                    with open(a.out, "a") as f:
                        f.write(json.dumps(row) + "\n")
            finally:
                srv.unmount()
                fs.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
