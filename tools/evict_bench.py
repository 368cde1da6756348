#!/usr/bin/env python3
"""Eviction select (K4-K6) and page allocation (K7): device vs CPU on a real BlockStore.

For each candidate count N: N committed one-page blocks in an HBM dir, a random tenth re-accessed,
then the victim set for 10% of the footprint is computed `--iters` times by the device grid select
(select_victims_device: dirty-slot flush + keys/4 histogram passes/compaction + one sync) and by
the CPU sort (the pre-device path), and K7 claims (peeked, given back) are timed against the host
bitmap scan.  Prints one JSON line per N.

    python tools/evict_bench.py --counts 10000,150000 --out gpurun_out/evict_bench.jsonl
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n: int, iters: int, page: int, policy: int) -> dict:
    import numpy as np
    import torch

    from alluxio_amd.ops.native import lib
    C = lib()
    arena = torch.empty((n + 64) * page, dtype=torch.uint8, device="cuda")
    d = C.DirSpec()
    d.tier, d.tier_alias, d.medium, d.kind = 0, "MEM", "HBM", C.DirKind.DEVICE
    d.base, d.capacity, d.page_size, d.device = arena.data_ptr(), arena.numel(), page, 0
    s = C.BlockStore([d], annotator=policy, alloc_policy=0, lrfu_step=1e-4, device=0)
    s.set_use_device_alloc(True, 64)
    ids = list(range(1, n + 1))
    t = time.perf_counter()
    s.create_blocks(1, ids, 0, "", [page] * n, False)
    bulk_create_s = time.perf_counter() - t
    for b in ids:
        s.commit_block(1, b)
    hot = np.random.default_rng(0).choice(n, n // 10, replace=False) + 1
    s.access_blocks(hot.tolist())
    need = (n // 10) * page
    s.select_for_bench(0, need, True)      # first flush of all slots + warm
    out = {"candidates": n, "page": page, "policy": "LRFU" if policy else "LRU", "need_blocks": n // 10}
    for name, dev in (("device", True), ("cpu", False)):
        ts = []
        for i in range(iters):
            s.access_blocks(hot[i::iters][:64].tolist())   # a few touches between selections
            t = time.perf_counter()
            v = s.select_for_bench(0, need, dev)
            ts.append(time.perf_counter() - t)
        out[f"select_{name}_ms_p50"] = round(statistics.median(ts) * 1e3, 3)
        out[f"select_{name}_victims"] = len(v)
    for name, dev in (("device", True), ("cpu", False)):
        ts = []
        for _ in range(iters):
            t = time.perf_counter()
            p = s.peek_free_pages(0, 64, dev)
            ts.append(time.perf_counter() - t)
        out[f"alloc64_{name}_ms_p50"] = round(statistics.median(ts) * 1e3, 3)
    # bulk: claim n/2 pages after evicting half the blocks
    s.free_space(1, (n // 2) * page, 0, -1)
    for name, dev in (("device", True), ("cpu", False)):
        ts = []
        for _ in range(max(3, iters // 4)):
            t = time.perf_counter()
            p = s.peek_free_pages(0, n // 2, dev)
            ts.append(time.perf_counter() - t)
        out[f"alloc_half_{name}_ms_p50"] = round(statistics.median(ts) * 1e3, 3)
        out[f"alloc_half_{name}_pages"] = len(p)
    out["bulk_create_ms"] = round(bulk_create_s * 1e3, 2)
    out["stats"] = s.evict_stats()
    del s
    # K7 on its consumers: bulk create_blocks and ingest_files with the device magazine (claims
    # by kernels from a resident bitmap) vs the host bitmap scan, each on a fresh store
    for name, dev in (("device", True), ("host", False)):
        s = C.BlockStore([d], annotator=policy, alloc_policy=0, lrfu_step=1e-4, device=0)
        s.set_use_device_alloc(dev, 64)
        t = time.perf_counter()
        s.create_blocks(1, ids, 0, "", [page] * n, False)
        out[f"bulk_create_{name}_ms"] = round((time.perf_counter() - t) * 1e3, 2)
        del s
    nf = min(n, 20000)
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        blob = np.random.default_rng(1).integers(0, 256, page, dtype=np.uint8).tobytes()
        paths = []
        for i in range(nf):
            p = os.path.join(tmp, f"f{i}")
            with open(p, "wb") as f:
                f.write(blob)
            paths.append(p)
        staging = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
        for name, dev in (("device", True), ("host", False)):
            s = C.BlockStore([d], annotator=policy, alloc_policy=0, lrfu_step=1e-4, device=0)
            s.set_use_device_alloc(dev, 64)
            best = None
            for r in range(3):
                fids = list(range(10_000_000 * (r + 1), 10_000_000 * (r + 1) + nf))
                t = time.perf_counter()
                stt = s.ingest_files(2, fids, paths, [0] * nf, [page] * nf, staging.data_ptr(), staging.numel(), 8, 0)
                dt = time.perf_counter() - t
                assert stt == [0] * nf
                best = dt if best is None else min(best, dt)
                for b in fids:
                    s.remove_block(2, b)
            out[f"ingest_{nf}_{name}_ms"] = round(best * 1e3, 2)
            # per-phase wall time, mean of the 3 calls: setup, preads, launches, stream wait,
            # attach+commit, magazine refill
            out[f"ingest_{name}_phase_ms"] = [round(x / 3e6, 2) for x in s.evict_stats()["ingest_ns"]]
            del s
    del arena
    torch.cuda.synchronize()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counts", default="10000,150000")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--page", type=int, default=4096)
    ap.add_argument("--policy", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    for n in [int(x) for x in a.counts.split(",")]:
        r = run(n, a.iters, a.page, a.policy)
        line = json.dumps(r)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")


if __name__ == "__main__":
    main()
