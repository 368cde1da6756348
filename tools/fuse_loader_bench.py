#!/usr/bin/env python3
"""BASELINE config 4 through FUSE: a PyTorch DataLoader random-reads ImageNet-shaped 128 KB files
from an Alluxio FUSE mount (the reference's "TensorFlow/PyTorch via Alluxio FUSE" deployment,
docs/en/compute/Deep-Learning.md:94-96, which reports "nearly 2X" over reading the remote store).

    python tools/fuse_loader_bench.py --files 20000 --epochs 2 --workers 4 --out profiles/x.json

Setup: one in-process master + worker (DRAM tier: the measurement is the FUSE path, not the
device tier), the files written through the client API, the namespace mounted with this package's
/dev/fuse server (fuse/kernel.py).  The same DataLoader then reads the same files from the UFS
directory on local disk as the "storage without Alluxio" comparison.  Needs permission to
mount(2) a FUSE filesystem (root / CAP_SYS_ADMIN); CPU only.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class FileDataset:
    def __init__(self, paths, buffering=-1):
        self.paths = paths
        # -1: Python's default buffered open(), which probes isatty() -- one TCGETS ioctl per file,
        # a FUSE round trip on a mount but a local syscall on disk; 0: raw FileIO, no probe
        self.buffering = buffering

    def __len__(self):
        return len(self.paths)

    def __getitem__(self, i):
        import numpy as np
        import torch
        with open(self.paths[i], "rb", buffering=self.buffering) as f:
            b = f.read()
        return torch.from_numpy(np.frombuffer(b, dtype=np.uint8)[:16].copy()), len(b)


def _cpu():
    import resource
    s, c = resource.getrusage(resource.RUSAGE_SELF), resource.getrusage(resource.RUSAGE_CHILDREN)
    return s.ru_utime + s.ru_stime, c.ru_utime + c.ru_stime


def _thread_cpu() -> dict:
    """CPU seconds per thread name of this process (diagnostics: where the server time goes)."""
    out = {}
    tck = os.sysconf("SC_CLK_TCK")
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        f = st[st.rindex(")") + 2:].split()
        key = name.rstrip("0123456789")
        out[key] = out.get(key, 0.0) + (int(f[11]) + int(f[12])) / tck
    return out


def _scan(root: str, dirs: int) -> dict:
    """What torchvision's ImageFolder does before training: list every class directory."""
    t0 = time.perf_counter()
    n = sum(len(os.listdir(os.path.join(root, f"d{i:03d}"))) for i in range(dirs))
    return {"entries": n, "s": round(time.perf_counter() - t0, 3)}


def _epochs(paths, epochs, workers, batch, seed=0, buffering=-1):
    import torch
    from torch.utils.data import DataLoader, RandomSampler
    out = []
    for e in range(epochs):
        g = torch.Generator().manual_seed(seed + e)
        dl = DataLoader(FileDataset(paths, buffering), batch_size=batch, sampler=RandomSampler(paths, generator=g),
                        num_workers=workers, persistent_workers=False)
        t0 = time.perf_counter()
        c0 = _cpu()
        th0 = _thread_cpu()
        n = nbytes = 0
        for _, lens in dl:
            n += len(lens)
            nbytes += int(lens.sum())
        dt = time.perf_counter() - t0
        del dl
        c1 = _cpu()
        th1 = _thread_cpu()
        busy = {k: round(v - th0.get(k, 0.0), 2) for k, v in th1.items() if v - th0.get(k, 0.0) >= 0.05}
        out.append({"epoch": e, "files": n, "files_per_s": round(n / dt, 1), "GBps": round(nbytes / dt / 1e9, 3),
                    "s": round(dt, 3), "cpu_s_server_process": round(c1[0] - c0[0], 2),
                    "cpu_s_loader_workers": round(c1[1] - c0[1], 2), "cpu_s_by_thread": busy})
        print(json.dumps(out[-1]), flush=True)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=20000)
    ap.add_argument("--file-size", type=int, default=128 << 10)
    ap.add_argument("--dirs", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--fuse-threads", type=int, default=2)
    ap.add_argument("--server", choices=["native", "python"], default="native",
                    help="native: C++ /dev/fuse loop (csrc/fuse_server.cpp); python: the pure-Python loop")
    ap.add_argument("--no-embedded", action="store_true",
                    help="do not hand the worker's block store to the FUSE server (no native opens/reads)")
    ap.add_argument("--no-scan", action="store_true",
                    help="skip the ImageFolder-style directory scan before the epochs")
    ap.add_argument("--read-only", action="store_true",
                    help="-o ro mount: with the native server, zero-message opens (no OPEN/RELEASE per file)")
    ap.add_argument("--passthrough", action="store_true",
                    help="FUSE passthrough opens of single-block files held in a file tier (--tier DIR)")
    ap.add_argument("--tier", default="dram",
                    help="worker cache tier: dram (memfd arena) or a directory (e.g. /dev/shm/x: block files, "
                         "which the native server hands to the kernel as FUSE passthrough backing files)")
    ap.add_argument("--keep-cache", default="auto", help="auto | on | off (kernel page cache across opens)")
    ap.add_argument("--open-buffering", type=int, default=-1, choices=[-1, 0],
                    help="-1: default buffered open() (isatty ioctl per file); 0: unbuffered")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    import numpy as np
    from alluxio_amd.fuse import AlluxioFuseOps
    from alluxio_amd.fuse.kernel import mount_kernel
    from alluxio_amd.minicluster import LocalAlluxioCluster
    work = tempfile.mkdtemp(prefix="fusebench_")
    mnt = os.path.join(work, "mnt")
    os.makedirs(mnt)
    quota = max(1 << 30, int(a.files * a.file_size * 1.3))
    tier = a.tier
    if tier != "dram":
        tier = os.path.join(tier, f"fusebench_{os.getpid()}")
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": tier,
            "alluxio.worker.tieredstore.level0.dirs.mediumtype": "MEM",
            "alluxio.worker.tieredstore.level0.dirs.quota": str(quota),
            "alluxio.user.block.size.bytes.default": "1MB", "alluxio.worker.hbm.page.size": "128KB"}
    res = {"setup": f"{a.files} x {a.file_size} B files in {a.dirs} dirs, DataLoader workers={a.workers} "
                    f"batch={a.batch}, FUSE threads={a.fuse_threads}, tier={a.tier}, {os.cpu_count()} CPUs, "
                    f"keep_cache={a.keep_cache}, read_only={a.read_only}, open_buffering={a.open_buffering}"}
    try:
        with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=os.path.join(work, "c")) as c:
            fs = c.client(metadata_cache=True)
            rng = np.random.default_rng(0)
            blob = rng.integers(0, 256, a.file_size + 4096, dtype=np.uint8)
            rel = [f"d{i % a.dirs:03d}/f{i:07d}.jpg" for i in range(a.files)]
            t0 = time.perf_counter()
            for i, r in enumerate(rel):
                fs.write_file("/ds/" + r, blob[i % 4096:i % 4096 + a.file_size], write_type="CACHE_THROUGH")
            res["write_files_per_s"] = round(a.files / (time.perf_counter() - t0), 1)
            keep = {"auto": "auto", "on": True, "off": False}[a.keep_cache]
            store = None if a.no_embedded or a.server == "python" else c.workers[0].store
            srv = mount_kernel(AlluxioFuseOps(fs), mnt, threads=a.fuse_threads, native=a.server == "native",
                               store=store, keep_cache=keep, read_only=a.read_only,
                               passthrough=a.passthrough)
            res["server"] = a.server + ("" if store is None else " (worker-embedded: native open/read)")
            try:
                paths = [os.path.join(mnt, "ds", r) for r in rel]
                if not a.no_scan:
                    res["fuse_scan"] = _scan(os.path.join(mnt, "ds"), a.dirs)
                res["fuse"] = _epochs(paths, a.epochs, a.workers, a.batch, buffering=a.open_buffering)
                res["fuse_ops"] = srv.op_stats()
            finally:
                srv.unmount()
            ufs_dir = c.master.fs_master.mount_table.resolve("/ds").uri
            # the same files straight from the UFS directory on local disk, page cache dropped
            # where permitted (the "storage without Alluxio" side of the comparison)
            try:
                with open("/proc/sys/vm/drop_caches", "w") as f:
                    f.write("1\n")
                res["ufs_page_cache_dropped"] = True
            except OSError:
                res["ufs_page_cache_dropped"] = False
            if not a.no_scan:
                res["ufs_scan"] = _scan(ufs_dir, a.dirs)
            res["ufs_direct"] = _epochs([os.path.join(ufs_dir, r) for r in rel], a.epochs, a.workers, a.batch, buffering=a.open_buffering)
            fs.close()
    finally:
        shutil.rmtree(work, ignore_errors=True)
        if tier != "dram":
            shutil.rmtree(tier, ignore_errors=True)
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
