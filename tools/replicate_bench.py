#!/usr/bin/env python3
"""Transfer-plane replication micro-bench: GB/s of ``replicate_ring`` / ``replicate_all`` per
round size (``batch_bytes``).

N worker ranks (one per GPU when the node has them, RCCL; else all on device 0 coordinated by
gloo -- the one-GPU rehearsal) each cache ``--blocks`` blocks of ``--block-size`` in their HBM tier,
then replicate them with every batch size in ``--batches`` (the received copies are removed
between runs).  Reference: job/server/.../plan/replicate/ReplicateDefinition.java (one gRPC block
stream per copy).

    python tools/replicate_bench.py --ranks 2 --blocks 8 --block-size 64m --batches 64m,256m,1g \
        --out gpurun_out/replicate_bench.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(a) -> None:
    import numpy as np
    import torch
    import torch.distributed as dist

    from alluxio_amd.conf import Configuration
    from alluxio_amd.master.process import AlluxioMasterProcess
    from alluxio_amd.parallel.transfer import TransferPlane
    from alluxio_amd.utils.format import parse_space_size
    from alluxio_amd.worker.process import AlluxioWorkerProcess
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = rank % max(ngpu, 1)
    backend = "nccl" if ngpu >= world and a.backend != "gloo" else "gloo"
    if ngpu:
        torch.cuda.set_device(dev)
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{a.port}", rank=rank, world_size=world)
    bs = parse_space_size(a.block_size)
    tier = f"hbm:{dev}" if ngpu else "dram"
    quota = bs * a.blocks * world + (256 << 20)
    conf = Configuration({"alluxio.master.journal.folder": a.work + "/journal",
                          "alluxio.worker.tieredstore.level0.dirs.path": tier,
                          "alluxio.worker.tieredstore.level0.dirs.quota": str(quota),
                          "alluxio.worker.hbm.page.size": "2MB", "alluxio.job.worker.enabled": "false",
                          "alluxio.web.server.enabled": "false"})
    box = [None]
    m = None
    if rank == 0:
        m = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=a.work + "/ufs")
        box[0] = m.start(start_heartbeats=False)
    dist.broadcast_object_list(box, src=0)
    w = AlluxioWorkerProcess(conf.copy(), master_address=box[0], port=0, device=dev if ngpu else None,
                             work_dir=a.work + f"/w{rank}")
    w.start(register=False, start_heartbeats=False)
    plane = TransferPlane.establish(w.worker, timeout_s=120.0)
    # blocks filled in place (no client write path in the measurement)
    mine = []
    host = None if ngpu else np.random.default_rng(rank).integers(0, 256, bs, dtype=np.uint8)
    for i in range(a.blocks):
        bid = (rank + 1) * 1_000_000 + i
        w.worker.native.create_block(1, bid, 0, "", bs, True, False)
        if ngpu:
            w.worker.native.fill_pattern(1, bid, bs, rank * 1000 + i)
        else:
            w.worker.write_bytes(1, bid, 0, host)
        w.worker.native.commit_block(1, bid, False)
        mine.append((bid, bs, rank))
    allb = [None] * world
    dist.all_gather_object(allb, mine)
    blocks = [x for part in allb for x in part]
    rows = []
    for method in a.methods.split(","):
        for batch in a.batches.split(","):
            plane.batch_bytes = parse_space_size(batch)
            for _rep in range(a.reps):
                dist.barrier()
                if ngpu:
                    torch.cuda.synchronize()
                r0 = plane.rounds
                t0 = time.perf_counter()
                moved = plane.replicate_ring(blocks, a.copies) if method == "ring" else plane.replicate_all(blocks)
                if ngpu:
                    torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                tmax = [None] * world
                dist.all_gather_object(tmax, (dt, moved))
                span = max(t for t, _ in tmax)
                total = sum(mv for _, mv in tmax)
                rows.append({"method": method, "batch": batch, "backend": backend, "ranks": world,
                             "block_size": a.block_size, "blocks_per_rank": a.blocks,
                             "rounds": plane.rounds - r0, "bytes_moved": total, "seconds": round(span, 4),
                             "GBps": round(total / span / 1e9, 2), "agreements": plane.agreements})
                # drop the received copies so the next run moves them again
                for bid, _n, owner in blocks:
                    if owner != rank and w.worker.has_block(bid):
                        w.worker.remove_block(1, bid)
                w.worker.drain_report()
    if rank == 0:
        for r in rows:
            print(json.dumps(r), flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(json.dumps(r) + "\n")
    dist.barrier()
    w.stop()
    if m is not None:
        m.stop()
    dist.destroy_process_group()      # a normal exit: profilers flush their traces at exit


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--block-size", default="64m")
    ap.add_argument("--batches", default="64m,256m,1g")
    ap.add_argument("--methods", default="ring,all")
    ap.add_argument("--copies", type=int, default=2)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--backend", default="auto", choices=["auto", "gloo"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--work", default=None)
    a = ap.parse_args(argv)
    if "RANK" in os.environ:
        rank_main(a)
        return 0
    import tempfile
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    work = a.work or tempfile.mkdtemp(prefix="replbench_")
    args = [sys.executable, os.path.abspath(__file__)] + (argv if argv is not None else sys.argv[1:]) + \
        ["--port", str(port), "--work", work]
    procs = [subprocess.Popen(args, env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(a.ranks)))
             for r in range(a.ranks)]
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


if __name__ == "__main__":
    raise SystemExit(main())
