"""StressWorkerBench (library form): T reader threads loop ``read(buf)`` over one file and re-open
at EOF; MB/s = bytes read after warmup / duration.

Parity: stress/shell/src/main/java/alluxio/stress/cli/worker/StressWorkerBench.java (prepare:
write the file CACHE_THROUGH to one worker; BenchThread.applyOperation :265-276) and
WorkerBenchParameters.java:40-70 (defaults: 256 threads, 128m file, 4k buffer, 32m blocks, 30s
duration + 30s warmup).  ``--mode threads`` runs literal Python threads with FileInStream (the
reference shape, for host readers); ``--mode batched`` runs the same T streams as one native
read session with one page-gather launch per round (the MI355X shape; what bench.py times).
"""
from __future__ import annotations

import argparse
import json
import threading
import time


def parse(argv):
    ap = argparse.ArgumentParser(prog="StressWorkerBench")
    ap.add_argument("--base", default="/stress-worker-base")
    ap.add_argument("--threads", type=int, default=256)
    ap.add_argument("--file-size", default="128m")
    ap.add_argument("--buffer-size", default="4k")
    ap.add_argument("--block-size", default="32m")
    ap.add_argument("--duration", default="30s")
    ap.add_argument("--warmup", default="30s")
    ap.add_argument("--free", action="store_true")
    ap.add_argument("--mode", choices=["threads", "batched"], default="threads")
    ap.add_argument("--device", choices=["host", "cuda"], default="host")
    ap.add_argument("--master", default=None)
    return ap.parse_args(argv)


def main(argv=None, fs=None, print_result=True) -> dict:
    from ..utils.format import parse_space_size, parse_time_size
    a = parse(argv or [])
    own = fs is None
    if own:
        from ..client.file_system import FileSystem
        fs = FileSystem(master_address=a.master, metadata_cache=True)
    import numpy as np
    size, buf, bs = parse_space_size(a.file_size), parse_space_size(a.buffer_size), parse_space_size(a.block_size)
    path = a.base.rstrip("/") + "/data"
    if not fs.exists(path):
        fs.create_directory(a.base, recursive=True, allow_exists=True)
        fs.write_file(path, np.full(size, ord("A"), dtype=np.uint8), write_type="CACHE_THROUGH", block_size=bs)
    if a.free:
        fs.free(path)
    warm, dur = parse_time_size(a.warmup) / 1000.0, parse_time_size(a.duration) / 1000.0
    errors: list[str] = []
    if a.mode == "batched":
        import torch
        from ..client.batch_reader import MultiStreamReader
        dev = torch.device("cuda") if a.device == "cuda" else None
        allb = torch.empty(a.threads * buf, dtype=torch.uint8, device=dev)
        r = MultiStreamReader(fs, path, [allb[i * buf:(i + 1) * buf] for i in range(a.threads)])
        t_end_warm = time.perf_counter() + warm
        while time.perf_counter() < t_end_warm:
            r.step()
        if dev is not None:
            torch.cuda.synchronize()
        b0, t0 = r.total_bytes, time.perf_counter()
        while time.perf_counter() - t0 < dur:
            r.step()
        if dev is not None:
            torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        nbytes = r.total_bytes - b0
        r.close()
    else:
        start = time.perf_counter() + 0.05
        record = start + warm
        end = record + dur
        counts = []
        st = fs.get_status(path)

        def thread():
            n = 0
            b = bytearray(buf)
            f = None
            try:
                while time.perf_counter() < start:
                    time.sleep(0.001)
                while time.perf_counter() < end:
                    if f is None:
                        f = fs.open_file(path, status=fs.get_status(path))
                    got = f.readinto(b)
                    if got == 0:
                        f.close()
                        f = None
                        continue
                    if time.perf_counter() > record:
                        n += got
            except Exception as e:  # noqa: BLE001
                errors.append(str(e))
            finally:
                if f is not None:
                    f.close()
            counts.append(n)
        del st
        ts = [threading.Thread(target=thread, daemon=True) for _ in range(a.threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        elapsed, nbytes = dur, sum(counts)
    out = {"bench": "worker", "mode": a.mode, "threads": a.threads, "bytes": nbytes,
           "throughput_MBps": nbytes / elapsed / 1e6, "duration_s": elapsed, "errors": errors[:20]}
    if print_result:
        print(json.dumps(out))
    if own:
        fs.close()
    return out


if __name__ == "__main__":  # pragma: no cover
    main(__import__("sys").argv[1:])
