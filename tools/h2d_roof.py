#!/usr/bin/env python3
"""H2D copy roof of one MI355X from pinned host memory: 1 / 4 / 8 streams, 8 MiB copies.

The write path's ceiling (host bytes into the HBM tier) is this roof: the data server stages
received chunks in pinned buffers and DMAs them H2D on one stream per I/O thread.

    python tools/h2d_roof.py --out gpurun_out/r6_h2d_roof.json
"""
import argparse
import json
import time

import torch


def run(streams: int, piece: int, total: int) -> float:
    dev = torch.device("cuda", 0)
    srcs = [torch.empty(piece, dtype=torch.uint8).pin_memory() for _ in range(streams)]
    dst = torch.empty(total, dtype=torch.uint8, device=dev)
    ss = [torch.cuda.Stream(dev) for _ in range(streams)]
    n = total // piece
    for _ in range(2):                       # warm: first touches, engine setup
        for i in range(n):
            k = i % streams
            with torch.cuda.stream(ss[k]):
                dst[i * piece:(i + 1) * piece].copy_(srcs[k], non_blocking=True)
        torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(n):
        k = i % streams
        with torch.cuda.stream(ss[k]):
            dst[i * piece:(i + 1) * piece].copy_(srcs[k], non_blocking=True)
    torch.cuda.synchronize()
    return total / (time.perf_counter() - t) / 1e9


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--piece", type=int, default=8 << 20)
    ap.add_argument("--total", type=int, default=4 << 30)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = [{"streams": s, "piece": a.piece, "GBps": round(run(s, a.piece, a.total), 2)} for s in (1, 4, 8)]
    for r in rows:
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
