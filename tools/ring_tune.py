"""A/B the device-cursor sequential-read kernel variants on the bench shape (4 KiB reads x 256
streams x depth), interleaved rounds in one process.  Prints one JSON line per (variant, cap)."""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from alluxio_amd.client.batch_reader import RingStreamReader  # noqa: E402
from alluxio_amd.minicluster import LocalAlluxioCluster  # noqa: E402
from alluxio_amd.ops.native import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--buf", type=int, default=4096)
    ap.add_argument("--depths", default="64,256")
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--caps", default="2048,4096,8192")
    ap.add_argument("--file-size", default="128m")
    ap.add_argument("--stagger", action="store_true", help="stream s starts at s/256 of the file")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from alluxio_amd.utils.format import parse_space_size
    fsize = parse_space_size(a.file_size)
    C = lib()
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "hbm:0",
            "alluxio.worker.tieredstore.level0.dirs.quota": str(max(1 << 30, fsize + (256 << 20))),
            "alluxio.worker.hbm.page.size": "2MB", "alluxio.user.block.size.bytes.default": "64MB"}
    res = []
    with LocalAlluxioCluster(num_workers=1, conf=conf, grpc=False) as c:
        fs = c.client(metadata_cache=True)
        data = torch.randint(0, 256, (fsize,), dtype=torch.uint8, device="cuda")
        fs.write_file("/tune", data, write_type="MUST_CACHE")
        del data
        starts = [((s_ * fsize) // 256) // a.buf * a.buf for s_ in range(256)] if a.stagger else None
        readers = {}
        for d in (int(x) for x in a.depths.split(",")):
            ring = torch.empty((256, d, a.buf), dtype=torch.uint8, device="cuda")
            readers[d] = (RingStreamReader(fs, "/tune", ring, start_offsets=starts), ring)
        combos = [(d, int(v), int(cap)) for d in readers for v in a.variants.split(",") for cap in a.caps.split(",")]
        t = {k: [] for k in combos}
        for _ in range(a.rounds):
            for k in combos:
                d, v, cap = k
                C.set_seq_read_variant(v, cap)
                r = readers[d][0]
                for _ in range(3):
                    r.step()
                torch.cuda.synchronize()
                b0, t0 = r.rs.total_bytes, time.perf_counter()
                for _ in range(a.steps):
                    r.step()
                torch.cuda.synchronize()
                t[k].append((r.rs.total_bytes - b0) / (time.perf_counter() - t0) / 1e9)
        for k in combos:
            row = {"file_size": fsize, "stagger": a.stagger, "depth": k[0], "variant": k[1], "grid_cap": k[2], "GBps_median": round(statistics.median(t[k]), 1),
                   "GBps_max": round(max(t[k]), 1)}
            res.append(row)
            print(json.dumps(row), flush=True)
        for r, _ in readers.values():
            r.close()
        fs.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
