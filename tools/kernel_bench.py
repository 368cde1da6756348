"""Micro-benchmarks of the data-plane kernels on one MI355X (prints one JSON line per case).

Cases: batched page-gather copy (bench-shaped: 256 readers x buffer from a cached file region,
and a large HBM-bound stream), torch D2D copy as the reference copy engine, CRC32C, LZ4 decode,
D2H into pinned host memory.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from alluxio_amd.ops.native import lib  # noqa: E402


def timeit(fn, iters, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    C = lib()
    dev = torch.device("cuda", 0)
    results = []

    def emit(**kw):
        results.append(kw)
        print(json.dumps(kw), flush=True)

    # --- bench-shaped gather: 256 readers x buf from a 128 MiB file region ---------------------
    for file_mb, buf_mb, readers in [(128, 4, 256), (128, 1, 256), (1024, 4, 256), (128, 0.25, 256)]:
        fbytes = int(file_mb * (1 << 20))
        bbytes = int(buf_mb * (1 << 20))
        src = torch.empty(fbytes, dtype=torch.uint8, device=dev)
        C.fill_pattern(src.data_ptr(), fbytes, 1, 0, 0)
        dst = torch.empty(readers * bbytes, dtype=torch.uint8, device=dev)
        nb = fbytes // bbytes
        step = [0]

        def run():
            k = step[0]
            step[0] += 1
            segs = [(src.data_ptr() + ((k + r) % nb) * bbytes, dst.data_ptr() + r * bbytes, bbytes)
                    for r in range(readers)]
            C.batched_copy(segs, 0)
        t = timeit(run, a.iters)
        emit(case="gather", file_mb=file_mb, buf_mb=buf_mb, readers=readers,
             ms=t * 1e3, GBps=readers * bbytes / t / 1e9)
        del src, dst

    # --- large streaming copy vs torch copy_ ----------------------------------------------------
    n = 4 << 30
    a_t = torch.empty(n, dtype=torch.uint8, device=dev)
    b_t = torch.empty(n, dtype=torch.uint8, device=dev)
    C.fill_pattern(a_t.data_ptr(), n, 3, 0, 0)
    t = timeit(lambda: C.batched_copy([(a_t.data_ptr(), b_t.data_ptr(), n)], 0), 5, 1)
    emit(case="stream_copy_kernel", GB=n / 1e9, ms=t * 1e3, copy_GBps=n / t / 1e9, hbm_rw_GBps=2 * n / t / 1e9)
    t = timeit(lambda: b_t.copy_(a_t), 5, 1)
    emit(case="stream_copy_torch", GB=n / 1e9, ms=t * 1e3, copy_GBps=n / t / 1e9, hbm_rw_GBps=2 * n / t / 1e9)
    del b_t

    # --- CRC32C ---------------------------------------------------------------------------------
    m = 1 << 30
    for variant in (0, 1, 2):
        C.set_crc_variant(variant)
        t = timeit(lambda: C.crc32c_device(a_t.data_ptr(), m, 2 << 20, 0), 5, 1)
        emit(case="crc32c", variant=variant, GB=m / 1e9, piece_mb=2, ms=t * 1e3, GBps=m / t / 1e9)
    C.set_crc_variant(4)

    # --- LZ4 decode of 64 KiB chunks -------------------------------------------------------------
    import numpy as np
    rng = np.random.default_rng(0)
    raw = rng.integers(0, 8, 1 << 16, dtype=np.uint8).tobytes()
    comp = C.lz4_compress(raw)
    nchunks = 4096
    csrc = torch.tensor(list(comp) * 1, dtype=torch.uint8, device=dev)
    out = torch.empty(nchunks * 65536, dtype=torch.uint8, device=dev)
    chunks = [(csrc.data_ptr(), out.data_ptr() + i * 65536, len(comp), 65536) for i in range(nchunks)]
    for variant in (0, 1, 2, 3):
        C.set_lz4_decode_variant(variant)
        t = timeit(lambda: C.lz4_device(chunks, False, 0), 5, 1)
        emit(case="lz4_decode", variant=variant, data="random 0..7", chunks=nchunks, ratio=len(raw) / len(comp),
             ms=t * 1e3, out_GBps=nchunks * 65536 / t / 1e9)
    # text-like data with long repeats (typical log/CSV blocks)
    words = [b"alluxio", b"worker", b"block", b"hbm", b"page", b"read", b"mi355x", b"cache", b"\n", b",", b" "]
    txt = b"".join(words[i] for i in rng.integers(0, len(words), 40000))[:1 << 16]
    tcomp = C.lz4_compress(txt)
    tsrc = torch.tensor(list(tcomp), dtype=torch.uint8, device=dev)
    tchunks = [(tsrc.data_ptr(), out.data_ptr() + i * 65536, len(tcomp), 65536) for i in range(nchunks)]
    for variant in (0, 1, 2, 3):
        C.set_lz4_decode_variant(variant)
        t = timeit(lambda: C.lz4_device(tchunks, False, 0), 5, 1)
        emit(case="lz4_decode", variant=variant, data="text", chunks=nchunks, ratio=len(txt) / len(tcomp),
             ms=t * 1e3, out_GBps=nchunks * 65536 / t / 1e9)
    C.set_lz4_decode_variant(-1)
    enc = torch.empty(nchunks * C.lz4_compress_bound(65536), dtype=torch.uint8, device=dev)
    cb = C.lz4_compress_bound(65536)
    echunks = [(out.data_ptr() + i * 65536, enc.data_ptr() + i * cb, 65536, cb) for i in range(nchunks)]
    t = timeit(lambda: C.lz4_device(echunks, True, 0), 5, 1)
    emit(case="lz4_encode", chunks=nchunks, ms=t * 1e3, in_GBps=nchunks * 65536 / t / 1e9)

    # --- D2H into pinned host -------------------------------------------------------------------
    h = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
    t = timeit(lambda: h.copy_(a_t[: 1 << 30], non_blocking=True), 5, 1)
    emit(case="d2h_pinned", GB=(1 << 30) / 1e9, ms=t * 1e3, GBps=(1 << 30) / t / 1e9)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
