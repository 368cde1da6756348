#!/usr/bin/env python3
"""CRC32C kernel throughput (K10): per-page CRCs of a contiguous HBM range, every kernel variant,
plus the gathered-page kernel used at commit.  One JSON line per case.

    python tools/crc_bench.py --gb 4 --out gpurun_out/crc.jsonl
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=4.0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import torch
    from alluxio_amd.ops.native import lib
    C = lib()
    n = int(a.gb * (1 << 30))
    buf = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    rows = []

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.iters

    for piece in (2 << 20, 64 << 20):
        for variant in (0, 1, 2, 3, 4):
            C.set_crc_variant(variant)
            t = timeit(lambda: C.crc32c_device(buf.data_ptr(), n, piece, 0))
            rows.append({"case": "crc32c_pieces", "variant": variant, "piece_MB": piece >> 20, "GB": n / 1e9,
                         "ms": t * 1e3, "GBps": n / t / 1e9})
            print(json.dumps(rows[-1]), flush=True)
    C.set_crc_variant(4)
    # sanity: variants agree
    C.set_crc_variant(1)
    v1 = C.crc32c_device(buf.data_ptr(), 64 << 20, 2 << 20, 0)
    C.set_crc_variant(3)
    v3 = C.crc32c_device(buf.data_ptr(), 64 << 20, 2 << 20, 0)
    C.set_crc_variant(4)
    v5 = C.crc32c_device(buf.data_ptr(), 64 << 20, 2 << 20, 0)
    C.set_crc_variant(4)
    assert list(v1) == list(v3) == list(v5), "variants disagree"
    if hasattr(C, "crc32c_gather_device"):
        pages = [(buf.data_ptr() + i * (2 << 20), 2 << 20) for i in range(0, n // (2 << 20), 3)]
        t = timeit(lambda: C.crc32c_gather_device(pages, 0))
        nb = len(pages) * (2 << 20)
        rows.append({"case": "crc32c_gather", "pages": len(pages), "GB": nb / 1e9, "ms": t * 1e3, "GBps": nb / t / 1e9})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write("".join(json.dumps(r) + "\n" for r in rows))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
