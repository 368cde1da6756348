#!/usr/bin/env python3
"""BASELINE config 4: a training input pipeline random-reading ImageNet-shaped 128 KB files.

Reference setup: FUSE mount -> PyTorch DataLoader over 1M 128 KB files (docs/en/compute/
Deep-Learning.md:94-96).  Here the trainer reads through the native client instead of a kernel
FUSE mount: ``FileListDataset`` takes every file's metadata (block ids + locations) from ONE
listStatus of the directory, and ``DeviceBatchLoader`` gathers each shuffled batch of files from
the worker's HBM arena into a ``[batch, 128 KB]`` device tensor with one array-planned page-gather
launch on a side stream, two batches in flight.

Phases (each timed): the files are created in the UFS (a local directory), their metadata is
loaded with one listing, every block is cached into HBM through the bulk ingest (native preads + batched H2D), then
``--epochs`` shuffled epochs are read.  Reported: files/s and GB/s per phase, plus where the time
goes (host planning vs device gather) for the epoch phase.

    python tools/dl_bench.py --files 100000 --out gpurun_out/dl_bench.jsonl
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _Done(Exception):
    pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=100_000)
    ap.add_argument("--file-size", type=int, default=128 * 1024)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--threads", type=int, default=16, help="native UFS reader threads")
    ap.add_argument("--work-dir", default=None)
    ap.add_argument("--ufs", choices=["local", "synthetic"], default="local",
                    help="synthetic: the files come from the synth:// UFS (content = function of the path, "
                         "backed by 4096 real files), so 1 M x 128 KB needs no 131 GB disk")
    ap.add_argument("--skip-cache", action="store_true", help="metadata phase only")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import numpy as np
    import torch

    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.models.dataset import DeviceBatchLoader, FileListDataset
    from alluxio_amd.proto import pb

    gpu = torch.cuda.is_available()
    work = tempfile.mkdtemp(prefix="dlbench_", dir=a.work_dir)
    res = {"files": a.files, "file_size": a.file_size, "batch": a.batch, "device": "cuda" if gpu else "cpu"}
    try:
        ufs = os.path.join(work, "ufs")
        d = os.path.join(ufs, "imagenet")
        os.makedirs(d)
        res["ufs"] = a.ufs
        if a.ufs == "local":
            base = np.random.default_rng(1).integers(0, 256, a.file_size + 4096, dtype=np.uint8).tobytes()
            t = time.perf_counter()
            for i in range(a.files):
                o = (i * 977) % 4096                     # distinct content per file
                with open(os.path.join(d, f"{i:07d}.JPEG"), "wb") as f:
                    f.write(base[o:o + a.file_size])
            res["ufs_write_s"] = round(time.perf_counter() - t, 2)
        total = a.files * a.file_size
        quota = int(total * 1.15) + (256 << 20)
        conf = {"alluxio.master.mount.table.root.ufs": ufs,
                "alluxio.worker.tieredstore.level0.dirs.path": "hbm" if gpu else "dram",
                "alluxio.worker.tieredstore.level0.dirs.quota": str(quota),
                "alluxio.worker.hbm.page.size": str(a.file_size),
                "alluxio.user.block.size.bytes.default": "64MB",
                "alluxio.worker.ufs.ingest.bulk.threads": str(a.threads),
                "alluxio.master.journal.type": "UFS"}
        with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=os.path.join(work, "c")) as c:
            fs = c.client()
            w = c.workers[0].worker
            root = "/imagenet"
            if a.ufs == "synthetic":
                os.rmdir(d)
                fs.mount("/syn", "synth:///dataset", properties={
                    "alluxio.underfs.synthetic.files": str(a.files), "alluxio.underfs.synthetic.size": str(a.file_size),
                    "alluxio.underfs.synthetic.dirs": "imagenet",
                    "alluxio.underfs.synthetic.backing.dir": os.path.join(work, "backing")})
                root = "/syn/imagenet"
            # metadata: one listing loads every file (LOAD_ONCE)
            t = time.perf_counter()
            ds = FileListDataset(fs, root, record_bytes=a.file_size)
            el = time.perf_counter() - t
            res["metadata_files_per_s"] = round(a.files / el, 1)
            res["metadata_s"] = round(el, 2)
            print(json.dumps({"phase": "metadata", "files_per_s": res["metadata_files_per_s"], "s": res["metadata_s"]}),
                  flush=True)
            if a.skip_cache:
                fs.close()
                raise _Done()
            # warm every block into HBM (the load job's bulk path: native preads into pinned
            # staging, batched H2D, one Python call per chunk of files), then refresh the listing
            t = time.perf_counter()
            st0 = fs.get_status(ds.paths[0])
            ufs_dir = st0.info.ufsPath.rsplit("/", 1)[0]
            items = [(f.blocks[0].blockId, pb.dataserver.OpenUfsBlockOptions(
                ufs_path=ufs_dir + "/" + p.rsplit("/", 1)[1], offset_in_file=0, block_size=f.blocks[0].length,
                mountId=st0.info.mountId)) for f, p in zip(ds.files, ds.paths)]
            cached = 0
            for i in range(0, len(items), 4096):
                cached += w.cache_blocks_from_ufs(items[i:i + 4096])
                if (i // 4096) % 32 == 31:
                    print(json.dumps({"phase": "cache", "files": i + 4096, "s": round(time.perf_counter() - t, 1)}),
                          flush=True)
            el = time.perf_counter() - t
            res["cache_all_done"] = cached == a.files
            res["cache_files_per_s"] = round(a.files / el, 1)
            res["cache_GBps"] = round(total / el / 1e9, 3)
            res["cache_breakdown_s"] = {k: round(v, 3) for k, v in w.bulk_stats.items()}
            ds = FileListDataset(fs, root, record_bytes=a.file_size)
            res["cached_fraction"] = round(float(np.mean([bool(f.blocks[0].locations) for f in ds.files])), 4)
            print(json.dumps({"phase": "cached", "files_per_s": res["cache_files_per_s"],
                              "cached_fraction": res["cached_fraction"]}), flush=True)
            # training epochs: shuffled batches gathered on the device
            dev = torch.device("cuda", 0) if gpu else torch.device("cpu")
            with DeviceBatchLoader(ds, batch_size=a.batch, shuffle=True, seed=7, device=dev) as dl:
                t = time.perf_counter()
                dl._single_worker()
                res["loader_setup_s"] = round(time.perf_counter() - t, 3)
                checksum = 0
                epochs = []
                for ep in range(a.epochs):
                    n = 0
                    t = time.perf_counter()
                    plan_s = 0.0
                    for batch in dl:
                        n += batch.shape[0]
                        checksum += int(batch[0, :8].sum().item()) if ep == 0 and n <= a.batch else 0
                    if gpu:
                        torch.cuda.synchronize()
                    el = time.perf_counter() - t
                    epochs.append({"files_per_s": round(n / el, 1), "GBps": round(n * a.file_size / el / 1e9, 3),
                                   "s": round(el, 3)})
                res["epochs"] = epochs
                # where the time goes: planning + launch alone, no device wait
                ix = np.arange(a.batch)
                buf = torch.empty((a.batch, a.file_size), dtype=torch.uint8, device=dev)
                t = time.perf_counter()
                reps = 200
                for _ in range(reps):
                    dl._fill(buf, ix)
                host_s = (time.perf_counter() - t) / reps
                if gpu:
                    torch.cuda.synchronize()
                    t = time.perf_counter()
                    for _ in range(reps):
                        dl._fill(buf, ix)
                    torch.cuda.synchronize()
                    full_s = (time.perf_counter() - t) / reps
                else:
                    full_s = host_s
                res["per_batch_host_plan_launch_ms"] = round(host_s * 1e3, 3)
                res["per_batch_total_ms"] = round(full_s * 1e3, 3)
                res["bottleneck"] = "host planning/launch" if host_s > 0.8 * full_s else "device gather"
            fs.close()
    except _Done:
        pass
    finally:
        shutil.rmtree(work, ignore_errors=True)
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
