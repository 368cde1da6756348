"""StressClientIOBench: client read/write throughput with per-thread files.

Parity: stress/shell/src/main/java/alluxio/stress/cli/client/StressClientIOBench.java
(operations Write, Read, ReadByteBuffer, ReadFully, PosRead, PosReadFully; ``--threads``
list run one after another, each thread on its own file; ClientIOTaskResult throughput per
thread count).
"""
from __future__ import annotations

import argparse
import json
import random
import threading
import time

OPS = ["Write", "Read", "ReadByteBuffer", "ReadFully", "PosRead", "PosReadFully"]


def parse(argv):
    ap = argparse.ArgumentParser(prog="StressClientIOBench")
    ap.add_argument("--operation", choices=OPS, default="Read")
    ap.add_argument("--threads", default="1,4")
    ap.add_argument("--file-size", default="16m")
    ap.add_argument("--buffer-size", default="1m")
    ap.add_argument("--block-size", default="16m")
    ap.add_argument("--duration", default="3s")
    ap.add_argument("--warmup", default="0s")
    ap.add_argument("--base", default="/stress-client-io-base")
    ap.add_argument("--write-type", default="MUST_CACHE")
    ap.add_argument("--master", default=None)
    return ap.parse_args(argv)


def main(argv=None, fs=None, print_result=True) -> dict:
    from ..utils.format import parse_space_size, parse_time_size
    a = parse(argv or [])
    own = fs is None
    if own:
        from ..client.file_system import FileSystem
        fs = FileSystem(master_address=a.master, metadata_cache=True)
    size, buf, bs = parse_space_size(a.file_size), parse_space_size(a.buffer_size), parse_space_size(a.block_size)
    dur = parse_time_size(a.duration) / 1000.0
    threads_list = [int(x) for x in a.threads.split(",")]
    payload = bytes(random.Random(0).getrandbits(8) for _ in range(min(buf, 1 << 16))) * (buf // min(buf, 1 << 16) + 1)
    payload = payload[:buf]
    fs.create_directory(a.base, recursive=True, allow_exists=True)
    rows = []
    for nthreads in threads_list:
        paths = [f"{a.base}/t{nthreads}-{i}" for i in range(nthreads)]
        if a.operation != "Write":
            for p in paths:
                if not fs.exists(p):
                    with fs.create_file(p, block_size=bs, write_type=a.write_type) as f:
                        for _ in range(size // buf):
                            f.write(payload)
        counts = [0] * nthreads
        errors = []

        def run(i):
            end = time.perf_counter() + dur
            rng = random.Random(i)
            b = bytearray(buf)
            try:
                if a.operation == "Write":
                    n = 0
                    while time.perf_counter() < end:
                        p = f"{paths[i]}.w{n}"
                        with fs.create_file(p, block_size=bs, write_type=a.write_type) as f:
                            for _ in range(max(1, size // buf)):
                                f.write(payload)
                                counts[i] += buf
                        fs.delete(p)
                        n += 1
                    return
                while time.perf_counter() < end:
                    with fs.open_file(paths[i]) as f:
                        if a.operation in ("Read", "ReadByteBuffer"):
                            while True:
                                got = f.readinto(b)
                                if not got:
                                    break
                                counts[i] += got
                        elif a.operation == "ReadFully":
                            counts[i] += len(f.read())
                        else:  # positioned reads
                            for _ in range(max(1, size // buf)):
                                pos = rng.randrange(0, max(1, size - buf))
                                counts[i] += f.pread(pos, b)
                                if a.operation == "PosRead" and time.perf_counter() > end:
                                    break
            except Exception as e:  # noqa: BLE001
                errors.append(str(e))
        ts = [threading.Thread(target=run, args=(i,), daemon=True) for i in range(nthreads)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        el = time.perf_counter() - t0
        rows.append({"threads": nthreads, "bytes": sum(counts), "throughput_MBps": sum(counts) / el / 1e6,
                     "errors": errors[:10]})
    out = {"bench": "client-io", "operation": a.operation, "rows": rows,
           "throughput_MBps": max(r["throughput_MBps"] for r in rows), "bytes": sum(r["bytes"] for r in rows),
           "errors": [e for r in rows for e in r["errors"]]}
    if print_result:
        print(json.dumps(out))
    if own:
        fs.close()
    del parse_time_size
    return out


if __name__ == "__main__":  # pragma: no cover
    main(__import__("sys").argv[1:])
