"""HBM roofs on this GPU for the bench's large phase: device-to-device copy of buffers far larger
than the MALL (torch ``copy_`` = the runtime's blit kernel, and ``hipMemcpyDtoD``), plus a
read-only pass (int64 sum).  The large phase moves every byte HBM -> ring once, so its delivered
GB/s is bounded by the copy roof printed here."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n = int(a.gib * (1 << 30))
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    out = {"bytes": n}
    s = timed(lambda: dst.copy_(src), a.iters)
    out["torch_copy_GBps"] = round(n / s / 1e9, 1)
    from alluxio_amd.ops.native import lib     # the framework's own batched copy kernel, 1 segment
    C = lib()
    s = timed(lambda: C.batched_copy([(src.data_ptr(), dst.data_ptr(), n)], 0, False), a.iters)
    out["batched_copy_kernel_GBps"] = round(n / s / 1e9, 1)
    v = src.view(torch.int64)
    s = timed(lambda: v.sum(), a.iters)
    out["read_sum_GBps"] = round(n / s / 1e9, 1)
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
