#!/usr/bin/env python3
"""StressWorkerBench-equivalent cached sequential-read benchmark on MI355X workers.

Reference methodology (stress/shell/.../StressWorkerBench.java:71-116,251-276,
stress/common/.../WorkerBenchParameters.java:40-70, WorkerBenchSummary.java:59-71): a file is
written CACHE_THROUGH to exactly one worker, then ``--threads`` readers loop ``read(buf)`` over it
and re-open at EOF; the result is bytes read / time.  Every GPU rank here is one worker (HBM MEM
tier) plus its own client, one process per GPU (``torch.distributed``; rank 0 also runs the
master).  Each rank writes its file through the client API (CACHE_THROUGH: local UFS + its own
worker), then its reader streams read it with the reference defaults (256 streams, 128 MiB file,
4 KiB ``read(buf)``; 64 MiB blocks per BASELINE.md).

One bench *step* = every stream performs ``depth`` consecutive ``read(buf)`` calls (EOF calls
re-open the file, as the reference loop does), all executed by ONE device-cursor kernel launch:
the file's page table lives on the GPU and each call's bytes land in that stream's own ring slot
``ring[stream, call]`` — no call is skipped or merged.  depth defaults to 1 MiB of calls per
stream (256 for 4 KiB), the amortisation the reference client gets from 1 MiB chunk buffers.

Phases (all timed between a barrier + ``torch.cuda.synchronize()`` on both sides; max over ranks):

* ``local``  (the headline ``value``): every stream starts at offset 0, as StressWorkerBench's
  threads do, so all 256 streams read the same window in lockstep;
* ``stagger``: stream s starts at s/threads of the file, so the streams read distinct data;
* ``host``: the ring lives in pinned host memory (a CPU-side reader; the copy crosses to DRAM);
* ``large``: a ``--large-size`` file (16 GiB by default on GPU: far larger than the 256 MB MALL)
  written MUST_CACHE from device memory and read by staggered streams, so every byte comes from
  HBM — the MEM-tier read rate a 288 GB tier serves, not an L2/MALL-resident window;
* ``remote`` (N > 1): rank r's streams read the file cached on worker (r+1) % N — the peer GPU's
  HBM mapped through HIP IPC and read over xGMI by the kernel on rank r's GPU;
* ``replicate`` (N > 1): every rank writes a new file with ``--replication`` copies; the local
  worker takes the bytes and the replica workers pull each block out of its HBM over xGMI;
* ``duration``: the local phase re-run for ``--duration`` seconds of wall time.

``value`` = total bytes read by all ranks in the K timed ``local`` steps / max-over-ranks time
(GB/s, whole node, weak scaling: each worker serves its own file).

Run: python bench.py [--gpus N --steps K --warmup W].  With N > 1 and no torchrun environment
the script launches ``torch.distributed.run`` itself as a child process (before touching the GPU).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "StressWorkerBench cached seq-read GB/s (whole node) at 1/2/4/8 MI355X workers"
PHASES = ("local", "stagger", "host", "large", "remote", "replicate", "duration")


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
                    help="read calls per stream per step (0 = 1 MiB of calls per stream)")
    ap.add_argument("--phases", default=",".join(PHASES), help="comma list of " + "/".join(PHASES))
    ap.add_argument("--duration", type=float, default=2.0, help="seconds for the duration phase")
    ap.add_argument("--phase-timeout", type=float, default=180.0,
                    help="deadline (s) of the cross-rank remote/replicate phases; past it the run "
                         "reports the phase as timed out and ends instead of hanging")
    ap.add_argument("--replication", type=int, default=3)
    ap.add_argument("--work-dir", default=None)
    ap.add_argument("--large-size", default=None,
                    help="file size of the large phase (default 16g on GPU, 0 = skip; CPU default 0)")
    ap.add_argument("--prop", action="append", default=[], metavar="KEY=VALUE",
                    help="extra alluxio property for master/worker/client (repeatable)")
    ap.add_argument("--profile-json", default=None, help="append per-rank timings to this file")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses device 0 and the process group is gloo "
                         "(RCCL refuses two ranks on one GPU); the data plane still runs on the GPU")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn_torchrun(a, argv) -> int:
    """N > 1 without a torchrun environment: run ourselves under torch.distributed.run as a CHILD
    process (never exec: nothing has touched the GPU yet, and the parent only waits)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse_args(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _spawn_torchrun(a, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    phases = [p for p in a.phases.split(",") if p]
    for p in phases:
        if p not in PHASES:
            raise SystemExit(f"unknown phase {p}")

    import numpy as np
    import torch
    import torch.distributed as dist
    from alluxio_amd.utils.format import parse_space_size

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available()
    if a.one_device:
        local_rank = 0
    if gpu:
        torch.cuda.set_device(local_rank)
    distributed = world > 1
    if distributed:
        dist.init_process_group("nccl" if gpu and not a.one_device else "gloo")
    dev_t = torch.device("cuda", local_rank) if gpu else torch.device("cpu")
    red_dev = torch.device("cpu") if a.one_device else dev_t     # gloo collectives on host tensors

    file_size = parse_space_size(a.file_size)
    block_size = parse_space_size(a.block_size)
    buf = parse_space_size(a.buffer_size)
    page = parse_space_size(a.page_size)
    work = a.work_dir or os.path.join("/tmp", f"alluxio_amd_bench_{os.getpid() if not distributed else 'dist'}")
    os.makedirs(work, exist_ok=True)

    from alluxio_amd.client.batch_reader import RemoteRingReader, RingStreamReader
    from alluxio_amd.client.context import worker_address_str
    from alluxio_amd.client.file_system import FileSystem
    from alluxio_amd.conf import Configuration
    from alluxio_amd.master.process import AlluxioMasterProcess
    from alluxio_amd.worker.process import AlluxioWorkerProcess

    replicas = max(1, min(a.replication, world))
    large_size = parse_space_size(a.large_size) if a.large_size is not None else ((16 << 30) if gpu else 0)
    if "large" not in phases:
        large_size = 0
    large_size -= large_size % buf
    # own file + one replica of each of (replicas-1) neighbours' replicated files + own replicated file
    quota = max((2 + replicas) * file_size, (4 << 30) if gpu else (1 << 30)) + large_size
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
    for kv in a.prop:
        k, _, v = kv.partition("=")
        props[k.strip()] = v.strip()
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
    phase_errors: dict = {}     # secondary phases that failed or were skipped (reported in config)
    my_addr = worker_address_str(worker.worker.address)
    addrs = [my_addr]
    devices = [local_rank if gpu else -1]
    peer_devices = [list(getattr(worker, "peer_devices", []) or [])]
    if distributed:
        addrs, devices, peer_devices = [None] * world, [None] * world, [None] * world
        dist.all_gather_object(addrs, my_addr)
        dist.all_gather_object(devices, local_rank if gpu else -1)
        dist.all_gather_object(peer_devices, list(getattr(worker, "peer_devices", []) or []))
        if gpu:
            # a remote phase over xGMI needs every rank's peer GPU mapped (hipDeviceEnablePeerAccess);
            # without it that phase is skipped and reported, the headline still runs
            for r in range(world):
                peer = devices[(r + 1) % world]
                if peer != devices[r] and peer not in peer_devices[r]:
                    phase_errors["remote"] = (f"rank {r} (device {devices[r]}) has no peer access to "
                                              f"device {peer}: peer_devices={peer_devices[r]}")
                    break

    def barrier():
        if distributed:
            dist.barrier()

    def sync():
        if gpu:
            torch.cuda.synchronize()

    def reduce(value: float, op) -> float:
        if not distributed:
            return value
        t = torch.tensor([value], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=op)
        return t.item()

    def MAX(v):
        return reduce(v, dist.ReduceOp.MAX if distributed else None)

    def SUM(v):
        return reduce(v, dist.ReduceOp.SUM if distributed else None)

    # ---- prepare: write the file CACHE_THROUGH to this rank's worker -------------------------
    path = f"/stress-worker-base/data-{rank}"
    rng = np.random.default_rng(1234 + rank)
    data = rng.integers(0, 256, file_size, dtype=np.uint8)
    barrier()
    if rank == 0:
        fs.create_directory("/stress-worker-base", recursive=True, allow_exists=True)
    barrier()
    t0 = time.perf_counter()
    fs.write_file(path, data, write_type="CACHE_THROUGH", block_size=block_size)
    write_s = time.perf_counter() - t0
    st = fs.get_status(path)
    assert st.length == file_size and st.in_alluxio_percentage == 100, (st.length, st.in_alluxio_percentage)
    barrier()

    depth = a.depth or max(1, (1 << 20) // buf)
    ring_dev = torch.empty((a.threads, depth, buf), dtype=torch.uint8, device=dev_t)
    stagger_offsets = [((s * file_size) // a.threads) // buf * buf for s in range(a.threads)]
    results: dict = {}
    ok_all = True

    def verify(reader, ring, src):
        good = True
        for s in (0, a.threads // 2, a.threads - 1):
            for k in (0, depth // 2, depth - 1):
                off, n = reader.last_call(s, k)
                if n and not np.array_equal(ring[s, k, :n].cpu().numpy(), src[off:off + n]):
                    good = False
        return good

    def timed(reader, steps, warmup):
        for _ in range(warmup):
            reader.step()
        sync()
        barrier()
        sync()
        b0 = reader.total_bytes
        t = time.perf_counter()
        for _ in range(steps):
            reader.step()
        sync()
        el = time.perf_counter() - t
        nb = reader.total_bytes - b0
        barrier()
        return el, nb

    def run_phase(name, make_reader, ring, src, steps, warmup):
        nonlocal ok_all
        reader = make_reader(ring)
        try:
            el, nb = timed(reader, steps, warmup)
            good = verify(reader, ring, src)
        finally:
            reader.close()
        el_max, total = MAX(el), SUM(float(nb))
        good = SUM(0.0 if good else 1.0) == 0
        ok_all = ok_all and good
        results[name] = {"GBps": round(total / el_max / 1e9, 3), "s": round(el_max, 5), "bytes": int(total),
                         "verified": good}
        return results[name]

    def emit():
        """Rank 0 prints the one JSON line (also called by the phase watchdog)."""
        if rank != 0:
            return
        cfg = {
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
            "reader": "gpu-consumer (same-GPU device ring), device-cursor ring x%d, streams start at offset 0" % depth,
            "verified": bool(ok_all),
            "headline_verified": bool(local["verified"]),
            "phase_errors": phase_errors or None,
            "stagger_GBps": results.get("stagger", {}).get("GBps"),
            "host_reader_GBps": results.get("host", {}).get("GBps"),
            "large_GBps": results.get("large", {}).get("GBps"),
            "large_file_size": results.get("large", {}).get("file_size"),
            "remote_GBps": results.get("remote", {}).get("GBps"),
            "replication": results.get("replicate"),
            "duration_GBps": results.get("duration", {}).get("GBps"),
            "duration_s": results.get("duration", {}).get("s"),
            "write_GBps_per_worker": round(file_size / write_s / 1e9, 3),
            "devices": devices,
            "peer_devices": peer_devices,
            "process_group": ({"backend": dist.get_backend(), "world_size": dist.get_world_size()}
                              if distributed else None),
            "phases": results,
        }
        out = {
            "metric": METRIC,
            "value": local["GBps"],
            "unit": "GB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(local["s"] / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8",
            "data": "synthetic (random bytes written through the client API, CACHE_THROUGH)",
            "config": cfg,
        }
        print(json.dumps(out), flush=True)

    class watchdog:
        """Deadline for a secondary phase that crosses ranks (remote / replicate over xGMI): if it
        has not finished in time, every rank stops there -- rank 0 first prints the JSON line with
        the results so far and the phase reported as timed out -- instead of hanging the job."""

        def __init__(self, name, seconds):
            self.name, self.seconds, self.timer = name, seconds, None

        def fire(self):
            phase_errors[self.name] = f"timed out after {self.seconds:.0f} s on rank {rank}"
            try:
                emit()
            finally:
                sys.stdout.flush()
                sys.stderr.flush()
                os._exit(0 if results.get("local", {}).get("verified") else 1)

        def __enter__(self):
            import threading
            self.timer = threading.Timer(self.seconds, self.fire)
            self.timer.daemon = True
            self.timer.start()
            return self

        def __exit__(self, *exc):
            self.timer.cancel()
            return False

    # ---- local (headline): lockstep from offset 0 --------------------------------------------
    run_phase("local", lambda r: RingStreamReader(fs, path, r), ring_dev, data, a.steps, a.warmup)
    local = results["local"]

    if "stagger" in phases:
        run_phase("stagger", lambda r: RingStreamReader(fs, path, r, start_offsets=stagger_offsets),
                  ring_dev, data, a.steps, a.warmup)

    if "host" in phases and gpu:
        ring_host = torch.empty((a.threads, depth, buf), dtype=torch.uint8, pin_memory=True)
        run_phase("host", lambda r: RingStreamReader(fs, path, r), ring_host, data,
                  max(2, min(a.steps, 20)), max(1, min(a.warmup, 3)))
        del ring_host

    if large_size:
        # 16 GiB of fresh device bytes (generated on the GPU), cached MUST_CACHE from device memory
        lpath = f"/stress-worker-base/large-{rank}"
        lsrc = torch.randint(0, 256, (large_size,), dtype=torch.uint8, device=dev_t,
                             generator=torch.Generator(device=dev_t).manual_seed(99 + rank))
        sync()
        t0 = time.perf_counter()
        fs.write_file(lpath, lsrc, write_type="MUST_CACHE", block_size=block_size)
        sync()
        lwrite_s = time.perf_counter() - t0
        loffs = [((s * large_size) // a.threads) // buf * buf for s in range(a.threads)]

        def verify_dev(reader, ring, src):
            good = True
            for s in (0, 1, a.threads // 2, a.threads - 1):
                for k in (0, depth // 2, depth - 1):
                    off, n = reader.last_call(s, k)
                    if n and not torch.equal(ring[s, k, :n], src[off:off + n].to(ring.device)):
                        good = False
            return good

        lr = RingStreamReader(fs, lpath, ring_dev, start_offsets=loffs)
        try:
            lsteps, lwarm = max(a.steps, 32), max(a.warmup, 2)
            el, nb = timed(lr, lsteps, lwarm)
            good = verify_dev(lr, ring_dev, lsrc)
        finally:
            lr.close()
        el_max, total = MAX(el), SUM(float(nb))
        good = SUM(0.0 if good else 1.0) == 0
        ok_all = ok_all and good
        results["large"] = {"GBps": round(total / el_max / 1e9, 3), "s": round(el_max, 5), "bytes": int(total),
                            "file_size": large_size, "steps": lsteps, "verified": good,
                            "write_GBps": round(SUM(float(large_size)) / MAX(lwrite_s) / 1e9, 3)}
        del lsrc
        fs.delete(lpath)
        if gpu:
            torch.cuda.empty_cache()
        barrier()

    def agree(ok: bool) -> bool:
        """True when the step succeeded on every rank (all ranks reach this same collective)."""
        return SUM(0.0 if ok else 1.0) == 0

    def all_errors(err):
        """Every rank's error text of a step that failed somewhere (collective on all ranks)."""
        errs = [err]
        if distributed:
            errs = [None] * world
            dist.all_gather_object(errs, err)
        return "; ".join(e for e in errs if e) or "failed"

    if "remote" in phases and world > 1 and "remote" not in phase_errors:
        with watchdog("remote", a.phase_timeout):
            peer = (rank + 1) % world
            peer_data = np.random.default_rng(1234 + peer).integers(0, 256, file_size, dtype=np.uint8)
            rreader, err = None, None
            try:
                if os.environ.get("ALLUXIO_BENCH_TEST_REMOTE_FAIL_RANK") == str(rank):
                    raise RuntimeError("injected remote-phase failure")          # tests/test_bench.py
                if os.environ.get("ALLUXIO_BENCH_TEST_REMOTE_HANG_RANK") == str(rank):
                    time.sleep(3600)                                             # tests/test_bench.py
                rreader = RemoteRingReader(fs, f"/stress-worker-base/data-{peer}", ring_dev, addrs[peer])
            except Exception as e:  # noqa: BLE001 - reported in the JSON; the headline stands
                err = f"rank {rank}: {e!r}"
            if agree(err is None):
                run_phase("remote", lambda r: rreader, ring_dev, peer_data, a.steps, a.warmup)
            else:
                if rreader is not None:
                    rreader.close()
                phase_errors["remote"] = all_errors(err)
                ok_all = False
            del peer_data

    if "replicate" in phases and world > 1:
        with watchdog("replicate", a.phase_timeout):
            wm = worker.worker.metrics
            names = ("XgmiBytesReceived", "PeerSharedBytesReceived", "PeerStreamBytesReceived", "PeerPullFailures")
            before = {k: wm.counter(k).count for k in names}
            from alluxio_amd.parallel.peer import pull_times
            pt0 = pull_times()
            src = torch.from_numpy(data).to(dev_t)
            sync()
            err = None

            def rep_write(name: str, copies: int) -> float:
                barrier()
                t = time.perf_counter()
                fs.write_file(name, src, write_type="MUST_CACHE", block_size=block_size, replication_min=copies)
                sync()
                el = time.perf_counter() - t
                barrier()
                return el

            el_plain = 0.0
            try:
                if a.warmup > 0:
                    # untimed: first peer-arena maps, control threads, channels
                    rep_write(f"/stress-worker-base/rep-warm-{rank}", replicas)
                    fs.delete(f"/stress-worker-base/rep-warm-{rank}")
                    pt0 = pull_times()
                    before = {k: wm.counter(k).count for k in names}
                    # the same write with one copy: what replication adds on top of it
                    el_plain = rep_write(f"/stress-worker-base/rep-plain-{rank}", 1)
                    fs.delete(f"/stress-worker-base/rep-plain-{rank}")
                el = rep_write(f"/stress-worker-base/rep-{rank}", replicas)
            except Exception as e:  # noqa: BLE001 - reported in the JSON; the headline stands
                err = f"rank {rank}: {e!r}"
                el = 0.0
                barrier()
            if not agree(err is None):
                phase_errors["replicate"] = all_errors(err)
            delta = {k: int(SUM(float(wm.counter(k).count - before[k]))) for k in names}
            el_max = max(MAX(el), 1e-9)
            plain_max = MAX(el_plain)
            # where a replica pull's time goes (ms per pull, summed over ranks / pulls)
            pt1 = pull_times()
            steps = ("open_rpc", "map", "create_and_plan", "copy", "verify_crc", "commit_and_report", "unlock_rpc",
                     "total", "handler", "pulls")
            tot = {k: SUM(float(pt1.get(k, 0.0) - pt0.get(k, 0.0))) for k in steps}
            npulls = max(tot.pop("pulls"), 1.0)
            pull_ms = {k: round(v / npulls * 1e3, 3) for k, v in tot.items()}
            pull_ms["pulls"] = int(npulls)
            # the writer's side of each block's fan-out (shared open, the replicas' PeerTransfer
            # calls, the unlock) and close()'s wait for the last block's pulls, per file
            fsteps = ("fan_open_rpc", "fan_transfers", "fan_unlock_rpc", "fan_total", "fans", "fan_close_wait",
                      "fan_call", "fan_call_start", "fan_calls")
            ftot = {k: SUM(float(pt1.get(k, 0.0) - pt0.get(k, 0.0))) for k in fsteps}
            nfans = max(ftot.pop("fans"), 1.0)
            ncalls = max(ftot.pop("fan_calls"), 1.0)
            per_call = {k: ftot.pop(k) for k in ("fan_call", "fan_call_start")}
            fan_ms = {k[4:]: round(v / nfans * 1e3, 3) for k, v in ftot.items() if k != "fan_close_wait"}
            fan_ms["fans"] = int(nfans)
            # one PeerTransfer call as the writer sees it, and how long it waited to be issued
            fan_ms["call"] = round(per_call["fan_call"] / ncalls * 1e3, 3)
            fan_ms["call_issue_delay"] = round(per_call["fan_call_start"] / ncalls * 1e3, 3)
            fan_ms["close_wait_per_file"] = round(ftot["fan_close_wait"] / world * 1e3, 3)
            try:
                rst = fs.get_status(f"/stress-worker-base/rep-{rank}")
                good = all(len(f.blockInfo.locations) >= replicas for f in rst.fileBlockInfos)
            except Exception:  # noqa: BLE001 - the write failed: already in phase_errors
                good = False
            good = SUM(0.0 if good else 1.0) == 0
            # every replica byte must have moved over the mapped plane (xGMI between distinct GPUs,
            # shared DRAM on CPU): a silent gRPC fallback or a failed pull fails the bench
            expect = world * file_size * (replicas - 1)
            distinct_gpus = gpu and len(set(devices)) == world
            plane_ok = (delta["PeerStreamBytesReceived"] == 0 and delta["PeerPullFailures"] == 0
                        and delta["XgmiBytesReceived"] + delta["PeerSharedBytesReceived"] == expect
                        and (not distinct_gpus or delta["XgmiBytesReceived"] == expect))
            if not plane_ok and rank == 0:
                print(f"replicate: data plane check failed: {delta} (expected {expect} peer bytes"
                      f"{' over xGMI' if distinct_gpus else ''})", file=sys.stderr, flush=True)
            ok_all = ok_all and good and plane_ok and "replicate" not in phase_errors
            results["replicate"] = {"replicas": replicas,
                                    "write_GBps": round(SUM(float(file_size)) / el_max / 1e9, 3),
                                    "replica_GBps": round(SUM(float(file_size * (replicas - 1))) / el_max / 1e9, 3),
                                    "xgmi_bytes_received": delta["XgmiBytesReceived"],
                                    "shared_bytes_received": delta["PeerSharedBytesReceived"],
                                    "stream_fallback_bytes_received": delta["PeerStreamBytesReceived"],
                                    "peer_pull_failures": delta["PeerPullFailures"],
                                    "s": round(el_max, 4), "verified": good, "data_plane_ok": plane_ok,
                                    "plain_write_GBps": (round(SUM(float(file_size)) / plain_max / 1e9, 3)
                                                         if plain_max > 0 else None),
                                    "pull_ms": pull_ms, "fan_ms": fan_ms}
            del src

    if "duration" in phases and a.duration > 0:
        reader = RingStreamReader(fs, path, ring_dev)
        try:
            for _ in range(a.warmup):
                reader.step()
            sync()
            barrier()
            b0, t, n = reader.total_bytes, time.perf_counter(), 0
            # every rank runs the same step count: rank 0's clock decides when to stop
            while True:
                for _ in range(64):
                    reader.step()
                n += 64
                sync()
                stop = torch.tensor([1.0 if time.perf_counter() - t >= a.duration else 0.0], device=red_dev)
                if distributed:
                    dist.broadcast(stop, src=0)
                if stop.item() > 0:
                    break
            el = time.perf_counter() - t
            nb = reader.total_bytes - b0
            barrier()
        finally:
            reader.close()
        el_max = MAX(el)
        results["duration"] = {"GBps": round(SUM(float(nb)) / el_max / 1e9, 3), "s": round(el_max, 3), "steps": n}

    if a.profile_json:
        with open(a.profile_json, "a") as f:
            f.write(json.dumps({"rank": rank, "results": results, "write_s": write_s}) + "\n")
    emit()

    fs.close()
    worker.stop()
    barrier()
    if master is not None:
        master.stop()
    if distributed:
        dist.destroy_process_group()
    # the exit status follows the headline; failures of secondary phases are in the JSON line
    return 0 if local["verified"] else 1


if __name__ == "__main__":
    sys.exit(main())
