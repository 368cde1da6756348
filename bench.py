#!/usr/bin/env python3
"""StressWorkerBench-equivalent cached sequential-read benchmark on MI355X workers.

Reference methodology (stress/shell/.../StressWorkerBench.java,
stress/common/.../WorkerBenchParameters.java:40-70): a file is written CACHE_THROUGH to exactly
one worker, then ``--threads`` readers loop ``read(buf)`` over it and re-open at EOF; the
result is bytes read / time.  Here every GPU rank is one worker (HBM MEM tier) with its own
in-process client; the rank writes its file through the client API (CACHE_THROUGH: local UFS +
local worker), then its ``threads`` reader streams read it with the reference's default
parameters (256 streams, 128 MiB file, 4 KiB ``read(buf)`` calls; 64 MiB blocks per BASELINE.md).

One bench *step* = every stream performs ``depth`` consecutive ``read(buf)`` calls (EOF calls
re-open the file, as the reference loop does), all executed by ONE device-cursor kernel launch:
the file's page table lives on the GPU, each call's bytes land in that stream's own ring slot
``ring[stream, call]`` (no call is skipped or merged: every call's bytes are copied to distinct
memory a consumer can use), and host work per step is O(1).  depth defaults to 1 MiB worth of
calls per stream (256 for 4 KiB) — the same amortisation the reference client gets by serving
read(4k) out of 1 MiB chunk buffers (GrpcDataReader chunks).  ``--buffer-size >= 1m`` (or
``--depth 1``) uses the per-call batched page-gather reader instead.

``value`` = total bytes read by all ranks in the K timed steps / max-over-ranks wall time (GB/s,
whole node, weak scaling: each worker serves its own file).

Run: python bench.py [--gpus N --steps K --warmup W]; N>1 is launched by torch.distributed.run.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "StressWorkerBench cached seq-read GB/s (whole node) at 1/2/4/8 MI355X workers"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--threads", type=int, default=256, help="reader streams per worker")
    ap.add_argument("--file-size", default="128m")
    ap.add_argument("--block-size", default="64m")
    ap.add_argument("--buffer-size", default="4k")
    ap.add_argument("--page-size", default="2m")
    ap.add_argument("--depth", type=int, default=0,
                    help="read calls per stream per step into a per-stream ring (device-cursor reader); "
                         "0 = auto (1 MiB of calls per stream for buffers < 1 MiB, else 1)")
    ap.add_argument("--dest", choices=["device", "host"], default="device")
    ap.add_argument("--host-check", action="store_true", help="also time a short host-reader (D2H) run")
    ap.add_argument("--work-dir", default=None)
    ap.add_argument("--profile-json", default=None, help="append per-rank timings to this file")
    return ap.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    import torch
    import torch.distributed as dist
    from alluxio_amd.utils.format import parse_space_size

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local_rank)
    distributed = world > 1
    if distributed:
        dist.init_process_group("nccl" if gpu else "gloo")

    file_size = parse_space_size(a.file_size)
    block_size = parse_space_size(a.block_size)
    buf = parse_space_size(a.buffer_size)
    page = parse_space_size(a.page_size)
    work = a.work_dir or os.path.join("/tmp", f"alluxio_amd_bench_{os.getpid() if not distributed else 'dist'}")
    os.makedirs(work, exist_ok=True)

    from alluxio_amd.client.batch_reader import MultiStreamReader, RingStreamReader
    from alluxio_amd.client.file_system import FileSystem
    from alluxio_amd.conf import Configuration
    from alluxio_amd.master.process import AlluxioMasterProcess
    from alluxio_amd.worker.process import AlluxioWorkerProcess

    quota = max(2 * file_size, 1 << 30)
    quota += (-quota) % page
    props = {
        "alluxio.work.dir": work,
        "alluxio.master.journal.type": "UFS",
        "alluxio.master.journal.folder": os.path.join(work, "journal"),
        "alluxio.master.mount.table.root.ufs": os.path.join(work, "ufs"),
        "alluxio.worker.tieredstore.levels": "1",
        "alluxio.worker.tieredstore.level0.alias": "MEM",
        "alluxio.worker.tieredstore.level0.dirs.path": "hbm" if gpu else "dram",
        "alluxio.worker.tieredstore.level0.dirs.quota": str(quota),
        "alluxio.worker.hbm.page.size": str(page),
        "alluxio.user.block.size.bytes.default": str(block_size),
        "alluxio.user.file.writetype.default": "CACHE_THROUGH",
        "alluxio.user.block.write.location.policy.class": "alluxio.client.block.policy.LocalFirstPolicy",
        "alluxio.master.web.port": "0",
        "alluxio.worker.web.port": "0",
        "alluxio.master.web.bind.host": "127.0.0.1",
        "alluxio.worker.web.bind.host": "127.0.0.1",
        "alluxio.user.metadata.cache.enabled": "true",
        "alluxio.security.authorization.permission.enabled": "false",
        "alluxio.master.worker.connect.wait.time": "0sec",
    }
    conf = Configuration(props)

    master = None
    if rank == 0:
        import shutil
        for d in ("journal", "ufs"):
            shutil.rmtree(os.path.join(work, d), ignore_errors=True)
        os.makedirs(os.path.join(work, "ufs"), exist_ok=True)
        master = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=os.path.join(work, "ufs"))
        master_addr = master.start(start_heartbeats=False)
    else:
        master_addr = None
    if distributed:
        box = [master_addr]
        dist.broadcast_object_list(box, src=0)
        master_addr = box[0]

    worker = AlluxioWorkerProcess(conf.copy(), master_address=master_addr, host="127.0.0.1", port=0,
                                  device=local_rank if gpu else 0, work_dir=os.path.join(work, f"w{rank}"))
    worker.start(register=True, start_heartbeats=False)
    fs = FileSystem(conf=conf.copy(), master_address=master_addr)

    # ---- prepare: write the file CACHE_THROUGH to this rank's worker -------------------------
    import numpy as np
    path = f"/stress-worker-base/data-{rank}"
    rng = np.random.default_rng(1234 + rank)
    data = rng.integers(0, 256, file_size, dtype=np.uint8)
    if distributed:
        dist.barrier()
    if rank == 0:
        fs.create_directory("/stress-worker-base", recursive=True, allow_exists=True)
    if distributed:
        dist.barrier()
    t0 = time.perf_counter()
    fs.write_file(path, data, write_type="CACHE_THROUGH", block_size=block_size)
    write_s = time.perf_counter() - t0
    st = fs.get_status(path)
    assert st.length == file_size and st.in_alluxio_percentage == 100, (st.length, st.in_alluxio_percentage)

    # ---- reader streams -----------------------------------------------------------------------
    dev = torch.device("cuda", local_rank) if (gpu and a.dest == "device") else None
    depth = a.depth or (max(1, (1 << 20) // buf) if buf < (1 << 20) else 1)
    if depth > 1:
        # device-cursor ring reader: each step = `depth` read(buf) calls per stream, one launch
        ring = torch.empty((a.threads, depth, buf), dtype=torch.uint8, device=dev,
                           pin_memory=(gpu and dev is None))
        reader = RingStreamReader(fs, path, ring)
        bufs = None
    else:
        if dev is not None:
            bufs_all = torch.empty(a.threads * buf, dtype=torch.uint8, device=dev)
        else:
            bufs_all = torch.empty(a.threads * buf, dtype=torch.uint8, pin_memory=gpu)
        bufs = [bufs_all[i * buf:(i + 1) * buf] for i in range(a.threads)]
        reader = MultiStreamReader(fs, path, bufs)

    def sync():
        if gpu:
            torch.cuda.synchronize()

    for _ in range(a.warmup):
        reader.step()
    sync()
    if distributed:
        dist.barrier()
    sync()
    b0 = reader.total_bytes
    t0 = time.perf_counter()
    for _ in range(a.steps):
        reader.step()
    sync()
    elapsed = time.perf_counter() - t0
    nbytes = reader.total_bytes - b0
    if distributed:
        dist.barrier()

    # ---- verify: sampled streams' last reads equal the file bytes at their offsets ------------
    ok = True
    check = [0, a.threads // 2, a.threads - 1]
    if bufs is None:
        for i in check:
            for k in (0, depth // 2, depth - 1):
                off, n = reader.last_call(i, k)
                if n and not np.array_equal(ring[i, k, :n].cpu().numpy(), data[off:off + n]):
                    ok = False
    else:
        for i in check:
            pos = reader.position(i)
            if pos == 0:
                continue
            n = min(buf, pos - ((pos - 1) // buf) * buf) if pos % buf else buf
            start = pos - n
            got = bufs[i][:n].cpu().numpy()
            if not np.array_equal(got, data[start:start + n]):
                ok = False
    reader.close()

    host_gbps = None
    if a.host_check and gpu:
        hb = torch.empty(64 * buf, dtype=torch.uint8, pin_memory=True)
        hr = MultiStreamReader(fs, path, [hb[i * buf:(i + 1) * buf] for i in range(64)])
        for _ in range(3):
            hr.step()
        hb0 = hr.total_bytes
        th = time.perf_counter()
        for _ in range(10):
            hr.step()
        host_gbps = (hr.total_bytes - hb0) / (time.perf_counter() - th) / 1e9
        hr.close()

    # ---- aggregate ----------------------------------------------------------------------------
    if distributed:
        dev_t = torch.device("cuda", local_rank) if gpu else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev_t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        b = torch.tensor([float(nbytes)], dtype=torch.float64, device=dev_t)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
        okt = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=dev_t)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        elapsed, total_bytes, ok = t.item(), b.item(), okt.item() > 0
    else:
        total_bytes = float(nbytes)

    if a.profile_json:
        with open(a.profile_json, "a") as f:
            f.write(json.dumps({"rank": rank, "elapsed_s": elapsed, "bytes": nbytes, "write_s": write_s,
                                "reopens": reader.reopens}) + "\n")
    value = total_bytes / elapsed / 1e9
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8",
            "data": "synthetic (random bytes written through the client API, CACHE_THROUGH)",
            "config": {
                "model": "StressWorkerBench cached seq-read, HBM MEM tier",
                "global_batch": a.threads * world,
                "seq_len": buf,
                "parallelism": f"workers{world}",
                "threads_per_worker": a.threads,
                "file_size": file_size,
                "block_size": block_size,
                "buffer_size": buf,
                "calls_per_stream_per_step": depth,
                "reads_per_step": a.threads * depth,
                "page_size": page,
                "reader": ("gpu-consumer (same-GPU device buffers)" if dev is not None else "host (pinned)")
                + (f", device-cursor ring x{depth}" if depth > 1 else ""),
                "verified": bool(ok),
                "host_reader_GBps": round(host_gbps, 3) if host_gbps else None,
                "write_GBps_per_worker": round(file_size / write_s / 1e9, 3),
            },
        }
        print(json.dumps(out), flush=True)

    fs.close()
    worker.stop()
    if distributed:
        dist.barrier()
    if master is not None:
        master.stop()
    if distributed:
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
