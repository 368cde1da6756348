"""UfsIOBench: raw UFS read/write throughput (reference stress/shell/.../UfsIOBench.java:
``--path`` UFS URI, ``--threads`` writers each writing one ``--io-size`` file, then the same
threads reading them back; reports per-phase MB/s)."""
from __future__ import annotations

import argparse
import json
import os
import threading
import time


def parse(argv):
    ap = argparse.ArgumentParser(prog="UfsIOBench")
    ap.add_argument("--path", default="/tmp/alluxio_ufs_io_bench")
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--io-size", default="64m")
    ap.add_argument("--buffer-size", default="8m")
    ap.add_argument("--conf", action="append", default=[])
    return ap.parse_args(argv)


def main(argv=None, fs=None, print_result=True) -> dict:
    from ..underfs import registry
    from ..utils.format import parse_space_size
    a = parse(argv or [])
    props = dict(kv.split("=", 1) for kv in a.conf)
    ufs = registry.create(a.path, None, props)
    size, buf = parse_space_size(a.io_size), parse_space_size(a.buffer_size)
    if not ufs.exists(a.path):
        ufs.mkdirs(a.path)
    chunk = os.urandom(min(buf, 1 << 20)) * max(1, buf // (1 << 20))
    chunk = chunk[:buf]
    res = {}
    errors = []

    def phase(name, fn):
        ts = [threading.Thread(target=fn, args=(i,), daemon=True) for i in range(a.threads)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        el = time.perf_counter() - t0
        res[name] = {"MBps": a.threads * size / el / 1e6, "seconds": el}

    def write(i):
        try:
            with ufs.create(f"{a.path.rstrip('/')}/io-{i}") as f:
                left = size
                while left > 0:
                    n = min(left, buf)
                    f.write(chunk[:n])
                    left -= n
        except Exception as e:  # noqa: BLE001
            errors.append(str(e))

    def read(i):
        try:
            with ufs.open(f"{a.path.rstrip('/')}/io-{i}") as f:
                while f.read(buf):
                    pass
        except Exception as e:  # noqa: BLE001
            errors.append(str(e))
    phase("write", write)
    phase("read", read)
    for i in range(a.threads):
        ufs.delete_file(f"{a.path.rstrip('/')}/io-{i}")
    out = {"bench": "ufs-io", "path": a.path, "threads": a.threads, "io_size": size, **res,
           "throughput_MBps": res["read"]["MBps"], "errors": errors[:10]}
    if print_result:
        print(json.dumps(out))
    return out


if __name__ == "__main__":  # pragma: no cover
    main(__import__("sys").argv[1:])
