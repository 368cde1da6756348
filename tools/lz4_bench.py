#!/usr/bin/env python3
"""K11 LZ4 decode/encode throughput sweep: data kind x chunk count x kernel variant.

    python tools/lz4_bench.py --out gpurun_out/lz4.jsonl
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, iters=5, warmup=1):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def datasets():
    import numpy as np
    rng = np.random.default_rng(0)
    out = {"random0-7": rng.integers(0, 8, 1 << 16, dtype=np.uint8).tobytes()}
    words = [b"alluxio", b"worker", b"block", b"hbm", b"page", b"read", b"mi355x", b"cache", b"\n", b",", b" "]
    out["text"] = b"".join(words[i] for i in rng.integers(0, len(words), 40000))[:1 << 16]
    # CSV-like rows: numbers + repeated column values (typical columnar/text datasets)
    rows = []
    for i in range(4000):
        rows.append(b"%d,%s,%d.%02d,%s\n" % (i, [b"GET", b"PUT", b"LIST"][i % 3], int(rng.integers(0, 999)),
                                               int(rng.integers(0, 99)), b"/data/part-%05d" % (i % 37)))
    out["csv"] = b"".join(rows)[:1 << 16]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="1024,4096,16384")
    ap.add_argument("--variants", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch
    from alluxio_amd.ops.native import lib
    C = lib()
    dev = torch.device("cuda", 0)
    variants = [int(v) for v in (a.variants or "1,2,3").split(",")]
    res = []
    for kind, raw in datasets().items():
        comp = C.lz4_compress(raw)
        assert C.lz4_decompress(comp, len(raw)) == raw
        src = torch.tensor(list(comp), dtype=torch.uint8, device=dev)
        for n in [int(x) for x in a.chunks.split(",")]:
            out = torch.empty(n * 65536, dtype=torch.uint8, device=dev)
            chunks = [(src.data_ptr(), out.data_ptr() + i * 65536, len(comp), 65536) for i in range(n)]
            for v in variants:
                C.set_lz4_decode_variant(v)
                out.zero_()
                sizes = C.lz4_device(chunks, False, 0)
                ok = all(s == len(raw) for s in sizes) and bytes(out[:65536].cpu().numpy()) == raw and \
                    bytes(out[-65536:].cpu().numpy()) == raw
                t = timeit(lambda: C.lz4_device(chunks, False, 0))
                k = C.lz4_device_kernel_ms(chunks, False, 5) / 1e3
                r = {"case": "lz4_decode", "data": kind, "ratio": round(len(raw) / len(comp), 3), "chunks": n,
                     "variant": v, "ok": ok, "call_ms": round(t * 1e3, 3), "kernel_ms": round(k * 1e3, 3),
                     "call_GBps": round(n * 65536 / t / 1e9, 2), "out_GBps": round(n * 65536 / k / 1e9, 2)}
                print(json.dumps(r), flush=True)
                res.append(r)
            if True:
                # encode of the decoded chunks (device encoder, K11)
                cb = C.lz4_compress_bound(65536)
                enc = torch.empty(n * cb, dtype=torch.uint8, device=dev)
                ech = [(out.data_ptr() + i * 65536, enc.data_ptr() + i * cb, 65536, cb) for i in range(n)]
                for ev in (2, 3, 4):
                    C.set_lz4_encode_variant(ev)
                    sizes = C.lz4_device(ech, True, 0)
                    ok = all(s_ > 0 for s_ in sizes) and C.lz4_decompress(
                        bytes(enc[:sizes[0]].cpu().numpy()), 65536) == raw
                    k = C.lz4_device_kernel_ms(ech, True, 3) / 1e3
                    r = {"case": "lz4_encode", "data": kind, "chunks": n, "encode_variant": ev, "ok": ok,
                         "ratio": round(n * 65536 / sum(sizes), 3), "kernel_ms": round(k * 1e3, 3),
                         "in_GBps": round(n * 65536 / k / 1e9, 2)}
                    print(json.dumps(r), flush=True)
                    res.append(r)
                C.set_lz4_encode_variant(4)
                del enc
            del out
    C.set_lz4_decode_variant(-1)
    if a.out:
        with open(a.out, "a") as f:
            for r in res:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
