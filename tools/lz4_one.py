#!/usr/bin/env python3
"""One LZ4 decode launch configuration (for rocprofv3 counter passes).

    python tools/lz4_one.py --variant 4 --data text --chunks 1024
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=4)
    ap.add_argument("--data", default="text")
    ap.add_argument("--chunks", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    from lz4_bench import datasets
    from alluxio_amd.ops.native import lib
    C = lib()
    raw = datasets()[a.data]
    comp = C.lz4_compress(raw)
    src = torch.tensor(list(comp), dtype=torch.uint8, device="cuda")
    out = torch.empty(a.chunks * 65536, dtype=torch.uint8, device="cuda")
    chunks = [(src.data_ptr(), out.data_ptr() + i * 65536, len(comp), 65536) for i in range(a.chunks)]
    C.set_lz4_decode_variant(a.variant)
    ms = C.lz4_device_kernel_ms(chunks, False, a.reps)
    print(f"variant {a.variant} {a.data} chunks {a.chunks}: {ms:.3f} ms, {a.chunks * 65536 / ms / 1e6:.2f} GB/s, "
          f"compressed {len(comp)} B", flush=True)


if __name__ == "__main__":
    main()
