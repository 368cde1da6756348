"""A/B the batched page-gather copy variants on the real bench path (interleaved rounds in one
process, per cdna guide §5.4 rule 24).  Prints one JSON line per (variant, grid cap) with the
median/min GB/s over rounds, for the bench shape and for a large HBM->HBM stream."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alluxio_amd.client.batch_reader import MultiStreamReader  # noqa: E402
from alluxio_amd.minicluster import LocalAlluxioCluster  # noqa: E402
from alluxio_amd.ops.native import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--file-mb", type=int, default=128)
    ap.add_argument("--buf-mb", type=float, default=4)
    ap.add_argument("--variants", default="0,1,2,3,4,5,8,9")
    ap.add_argument("--caps", default="1024,2048,4096")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    C = lib()
    dev = torch.device("cuda", 0)
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "hbm:0",
            "alluxio.worker.tieredstore.level0.dirs.quota": f"{max(1024, 2 * a.file_mb)}MB",
            "alluxio.worker.hbm.page.size": "2MB", "alluxio.user.block.size.bytes.default": "64MB"}
    results = []
    with LocalAlluxioCluster(num_workers=1, conf=conf, grpc=False) as c:
        fs = c.client(metadata_cache=True)
        data = np.random.default_rng(0).integers(0, 256, a.file_mb << 20, dtype=np.uint8)
        fs.write_file("/tune", data, write_type="MUST_CACHE")
        buf = int(a.buf_mb * (1 << 20))
        allb = torch.empty(256 * buf, dtype=torch.uint8, device=dev)
        r = MultiStreamReader(fs, "/tune", [allb[i * buf:(i + 1) * buf] for i in range(256)])
        big_a = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
        big_b = torch.empty(4 << 30, dtype=torch.uint8, device=dev)
        combos = [(int(v), int(cap)) for v in a.variants.split(",") for cap in a.caps.split(",")]
        bench_t = {k: [] for k in combos}
        stream_t = {k: [] for k in combos}
        for _ in range(a.rounds):
            for k in combos:
                C.set_copy_variant(*k)
                for _ in range(3):
                    r.step()
                torch.cuda.synchronize()
                b0 = r.total_bytes
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    r.step()
                torch.cuda.synchronize()
                bench_t[k].append((r.total_bytes - b0) / (time.perf_counter() - t0) / 1e9)
                C.batched_copy([(big_a.data_ptr(), big_b.data_ptr(), 4 << 30)], 0)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(3):
                    C.batched_copy([(big_a.data_ptr(), big_b.data_ptr(), 4 << 30)], 0)
                torch.cuda.synchronize()
                stream_t[k].append(3 * (4 << 30) / (time.perf_counter() - t0) / 1e9)
        C.set_copy_variant(0, 2048)
        r.close()
        for k in combos:
            row = {"variant": k[0], "grid_cap": k[1],
                   "bench_GBps_median": round(statistics.median(bench_t[k]), 1),
                   "bench_GBps_max": round(max(bench_t[k]), 1),
                   "stream_copy_GBps_median": round(statistics.median(stream_t[k]), 1)}
            results.append(row)
            print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
