"""StressWorkerBench (library form): T reader threads loop ``read(buf)`` over one file and re-open
at EOF; MB/s = bytes read after warmup / duration.

Parity: stress/shell/src/main/java/alluxio/stress/cli/worker/StressWorkerBench.java (prepare:
write the file CACHE_THROUGH to one worker; BenchThread.applyOperation :265-276) and
WorkerBenchParameters.java:40-70 (defaults: 256 threads, 128m file, 4k buffer, 32m blocks, 30s
duration + 30s warmup).  ``--mode threads`` runs literal Python threads with FileInStream (the
reference shape, for host readers); ``--mode native-threads`` runs the same T reader threads in
C++ (csrc/stress_bench.cpp: one chunk-buffered in-stream per thread, re-opened at EOF, no
interpreter lock in the loop -- the JVM shape of the reference's bench); ``--mode batched`` runs
the same T streams as one native read session with one page-gather launch per round (the MI355X
shape; what bench.py times).
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
    ap.add_argument("--mode", choices=["threads", "native-threads", "batched"], default="threads")
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
    native_extra = {}
    if a.mode == "native-threads":
        nbytes, elapsed, errs, native_extra = _native_threads(fs, path, a.threads, buf, bs, warm, dur)
        errors.extend(errs)
    elif a.mode == "batched":
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
    out.update(native_extra)
    if print_result:
        print(json.dumps(out))
    if own:
        fs.close()
    return out


def _native_threads(fs, path: str, threads: int, buf: int, block_size: int, warm: float, dur: float):
    """The reader loop in C++ threads over the file's blocks as this client would read them: the
    HIP-IPC short circuit for a same-node worker when the client's configuration picks it
    (``OpenDeviceBlock`` once per block for the run; every re-open maps the pages anew), else a
    ``ReadBlock`` call per block per pass over the worker's data port (its domain socket on the
    same node)."""
    from ..client.context import worker_address_str
    from ..client.streams import IpcBlockReader, _native_call
    from ..ops.native import lib
    from ..utils import ids
    ctx = fs.ctx
    conf = ctx.conf
    st = fs.get_status(path)
    chunk = conf.get_bytes("alluxio.user.native.reader.buffer.size", "4MB")
    rchunk = conf.get_bytes("alluxio.user.network.reader.chunk.size.bytes", "1MB")
    blocks, held, transport = [], [], None
    try:
        for fbi in st.fileBlockInfos:
            bi = fbi.blockInfo
            loc = bi.locations[0].workerAddress
            addr = worker_address_str(loc)
            spec = None
            use_ipc = ctx.is_local(loc) and conf.get_bool("alluxio.user.short.circuit.enabled", "true") and \
                conf.get_bool("alluxio.worker.ipc.enabled", "true") and \
                (not loc.domainSocketPath or conf.get_bool("alluxio.user.short.circuit.preferred", "false"))
            if use_ipc:
                try:
                    r = IpcBlockReader(ctx, addr, bi.blockId, ids.create_session_id())
                    held.append(r)
                    from ..parallel.ipc import map_handle
                    spec = {"length": bi.length, "kind": "host" if r.h.arena_kind == "dram" else "ipc",
                            "base": map_handle(r.h, r.device), "pages": list(r.h.pages),
                            "page_size": r.h.page_size, "device": r.device}
                    transport = "ipc"
                except Exception:  # noqa: BLE001 - not shareable: the data port
                    spec = None
            if spec is None:
                if ctx.is_local(loc):
                    ctx._note_domain_socket(loc)
                call = _native_call(ctx, addr, (loc.host, loc.dataPort or loc.rpcPort))
                if call is None:
                    raise RuntimeError("native-threads needs a worker in another process")
                host, port, cid, user, timeout, uds = call
                spec = {"length": bi.length, "kind": "grpc", "host": host, "port": port, "unix_path": uds,
                        "block_id": bi.blockId, "chunk": rchunk, "channel_id": cid, "user": user,
                        "timeout_ms": timeout}
                transport = transport or ("grpc-uds" if uds else "grpc")
            blocks.append(spec)
        r = lib().run_stress_reads(blocks, block_size, threads, buf, chunk, warm, dur,
                                   conf.get_bool("alluxio.user.native.reader.prefetch.enabled", "true"))
    finally:
        for h in held:
            h.close()
    extra = {"native": {"transport": transport, "reads": r["reads"], "file_opens": r["opens"],
                        "block_opens": r["block_opens"], "reader_chunk": chunk,
                        "min_thread_MBps": round(min(r["per_thread"]) / max(r["seconds"], 1e-9) / 1e6, 1)
                        if r["per_thread"] else 0.0}}
    return r["bytes"], r["seconds"], list(r["errors"]), extra


if __name__ == "__main__":  # pragma: no cover
    main(__import__("sys").argv[1:])
