"""StressMasterBench: metadata-operation throughput against the master.

Parity: stress/shell/src/main/java/alluxio/stress/cli/StressMasterBench.java (operations
CreateFile, GetBlockLocations, GetFileStatus, OpenFile, CreateDir, ListDir, ListDirLocated,
RenameFile, DeleteFile; ``--threads`` concurrent clients, ``--target-throughput`` rate limiter,
``--stop-count`` / ``--fixed-count`` path selection as in applyOperation: op ``i`` acts on
``fixed/i`` for i < fixed-count else ``files/i``, so RenameFile / DeleteFile consume what a previous
CreateFile run made; warmup then timed window) and
MasterBenchSummary (ops/s, latency percentiles, errors).  Reference published numbers for these
operations are in docs/en/operation/Scalability-Tuning.md:142-148.
"""
from __future__ import annotations

import argparse
import itertools
import json
import threading
import time

OPS = ["CreateFile", "GetBlockLocations", "GetFileStatus", "OpenFile", "CreateDir", "ListDir",
       "ListDirLocated", "RenameFile", "DeleteFile",
       # beyond StressMasterBench: the "ListStatus, file does not exist" row of the published
       # master numbers (docs/en/operation/Scalability-Tuning.md:148)
       "GetFileStatusNonexistent"]


def parse(argv):
    ap = argparse.ArgumentParser(prog="StressMasterBench")
    ap.add_argument("--operation", required=True, choices=OPS)
    ap.add_argument("--write-type", default="MUST_CACHE",
                    help="write type of CreateFile / CreateDir (THROUGH: the master does UFS I/O)")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--target-throughput", type=int, default=0, help="ops/s cap; 0 = unthrottled")
    ap.add_argument("--base", default="/stress-master-base")
    ap.add_argument("--duration", default="5s")
    ap.add_argument("--warmup", default="1s")
    ap.add_argument("--stop-count", type=int, default=-1)
    ap.add_argument("--fixed-count", type=int, default=100)
    ap.add_argument("--create-file-size", default="0")
    ap.add_argument("--master", default=None)
    return ap.parse_args(argv)


class _Rate:
    def __init__(self, ops_per_s):
        self.period = 1.0 / ops_per_s if ops_per_s > 0 else 0.0
        self.next = time.perf_counter()
        self.lock = threading.Lock()

    def acquire(self):
        if not self.period:
            return
        with self.lock:
            now = time.perf_counter()
            self.next = max(self.next + self.period, now)
            wait = self.next - now
        if wait > 0:
            time.sleep(wait)


def main(argv=None, fs=None, print_result=True) -> dict:
    from ..utils.format import parse_space_size, parse_time_size
    a = parse(argv or [])
    own = fs is None
    if own:
        from ..client.file_system import FileSystem
        fs = FileSystem(master_address=a.master)
    clients = [fs] + ([] if own or a.clients <= 1 else [])
    base = a.base.rstrip("/")
    fixed = f"{base}/fixed"
    files = f"{base}/files"
    payload = b"x" * parse_space_size(a.create_file_size)
    # preparation: the base directories, and (a convenience beyond the reference, which expects a
    # CreateFile run first) the fixed-count files the read-type operations use
    fs.create_directory(files, recursive=True, allow_exists=True, write_type="MUST_CACHE")
    fs.create_directory(fixed, recursive=True, allow_exists=True, write_type="MUST_CACHE")
    if a.operation in ("GetBlockLocations", "GetFileStatus", "OpenFile", "ListDir", "ListDirLocated"):
        existing = {s.name for s in fs.list_status(fixed)}
        for i in range(a.fixed_count):
            if str(i) not in existing:
                fs.write_file(f"{fixed}/{i}", payload, write_type="MUST_CACHE")
    counter = [0]
    lock = threading.Lock()
    stop = threading.Event()
    rate = _Rate(a.target_throughput)
    warm_s = parse_time_size(a.warmup) / 1000.0
    dur_s = parse_time_size(a.duration) / 1000.0
    start = time.perf_counter() + 0.05
    wall_off = time.time() - time.perf_counter()
    record_from = start + warm_s
    end = record_from + dur_s
    results = []

    ids_ = itertools.count(0)

    def next_id():
        return next(ids_)        # GIL-atomic; a shared mutex here would throttle the clients

    def target(i):
        # StressMasterBench.applyOperation: the first fixed-count paths live under fixed/, the
        # rest under files/; RenameFile / DeleteFile act on the paths a CreateFile run made
        return f"{fixed}/{i}" if i < a.fixed_count else f"{files}/{i}"

    def op_once(c, tid):
        i = next_id()
        if a.stop_count >= 0 and i >= a.stop_count:
            stop.set()
            return False
        k = i % max(1, a.fixed_count)
        if a.operation == "CreateFile":
            c.write_file(target(i), payload, write_type=a.write_type)
        elif a.operation == "CreateDir":
            c.create_directory(target(i), write_type=a.write_type)
        elif a.operation == "GetFileStatus":
            c.get_status(f"{fixed}/{k}")
        elif a.operation == "GetFileStatusNonexistent":
            if c.exists(f"{base}/missing/{k}"):
                raise IOError("a missing path exists")
        elif a.operation == "GetBlockLocations":
            c.get_block_locations(f"{fixed}/{k}")
        elif a.operation == "OpenFile":
            c.open_file(f"{fixed}/{k}").close()
        elif a.operation in ("ListDir", "ListDirLocated"):
            n = len(c.list_status(fixed))
            if n != a.fixed_count:
                raise IOError(f"listing {fixed} expected {a.fixed_count} files but got {n} files")
        elif a.operation == "RenameFile":
            src = target(i)
            c.rename(src, src + "-renamed")
        elif a.operation == "DeleteFile":
            c.delete(target(i), recursive=False)
        return True

    def worker(tid):
        c = clients[tid % len(clients)]
        ops, done, lat, errs = 0, 0, [], []
        while time.perf_counter() < start:
            time.sleep(0.001)
        while not stop.is_set() and time.perf_counter() < end:
            rate.acquire()
            t0 = time.perf_counter()
            try:
                if not op_once(c, tid):
                    break
            except Exception as e:  # noqa: BLE001
                errs.append(f"{type(e).__name__}: {e}")
                if len(errs) > 100:
                    break
                continue
            t1 = time.perf_counter()
            done += 1
            if t0 >= record_from:
                ops += 1
                lat.append(t1 - t0)
        results.append((ops, lat, errs, done))

    threads = [threading.Thread(target=worker, args=(t,), daemon=True) for t in range(a.threads)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    total = sum(r[0] for r in results)
    lats = sorted(x for r in results for x in r[1])
    window = min(dur_s, max(1e-9, time.perf_counter() - record_from)) if a.stop_count < 0 else \
        max(1e-9, time.perf_counter() - record_from)

    def pct(p):
        return lats[min(len(lats) - 1, int(p * len(lats)))] * 1e3 if lats else 0.0
    out = {"bench": "master", "operation": a.operation, "threads": a.threads, "ops": total,
           "window_wall": [record_from + wall_off, record_from + window + wall_off],
           "completed": sum(r[3] for r in results),
           "throughput_ops": total / window, "latency_ms": {"p50": pct(0.5), "p90": pct(0.9), "p99": pct(0.99),
                                                             "max": lats[-1] * 1e3 if lats else 0.0},
           "errors": [e for r in results for e in r[2]][:20]}
    if print_result:
        print(json.dumps(out))
    if own:
        fs.close()
    return out


if __name__ == "__main__":  # pragma: no cover
    main(__import__("sys").argv[1:])
