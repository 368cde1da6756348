#!/usr/bin/env python3
"""BASELINE config 5: UFS async-cache into the HBM tier under 2x working-set pressure, with
HBM -> host-DRAM demotion.

One worker (GPU 0) with an HBM tier of ``--hbm`` bytes over a DRAM tier of ``--dram`` bytes; a
working set of ``--factor`` x HBM bytes of files sits in the UFS only.  Every block is requested
through the worker's async-cache path (AsyncCacheRequestManager semantics: deduplicated,
``alluxio.worker.network.async.cache.manager.threads.max`` concurrent blocks), the clock runs
until every block is cached; as HBM fills, eviction demotes the coldest blocks to DRAM in
batched moves.  Reported per ingest depth (1 = the serial read-then-copy loop, 3 = the K3
pipeline: UFS read of chunk i+1 overlapped with the H2D of chunk i on a side stream):

* ingest GB/s (UFS bytes cached / wall time), demoted blocks/bytes, final HBM / DRAM occupancy;
* re-read GB/s of the whole working set into a device buffer (hot in HBM or DRAM).

``--ufs s3`` serves the files from an S3 endpoint (this repository's S3 REST proxy in front of a
second, DRAM-only cluster whose own UFS holds the bytes), ``--ufs s3native`` from the native S3
endpoint (csrc/http_blob.cpp, sendfile) so that the worker's S3 read path rather than the endpoint
is the bound, ``--ufs local`` from a local directory.

    python tools/ufs_ingest_bench.py --ufs local --hbm 2g --dram 6g --factor 2 --out gpurun_out/ufs_ingest.jsonl
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


def _write_working_set(ufs_write, nfiles, file_size):
    import numpy as np
    rng = np.random.default_rng(7)
    piece = rng.integers(0, 256, 64 << 20, dtype=np.uint8).tobytes()
    for i in range(nfiles):
        # distinct content per file without generating every byte: rotate a random 64 MiB piece
        buf = bytearray()
        k = i * 4099
        while len(buf) < file_size:
            n = min(len(piece), file_size - len(buf))
            rot = k % len(piece)
            chunk = (piece[rot:] + piece[:rot])[:n]
            buf += chunk
            k += 7919
        ufs_write(f"/ws/f{i:04d}", bytes(buf))


def run(a, depth: int) -> dict:
    import torch

    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.proto import pb
    from alluxio_amd.utils.format import parse_space_size

    hbm, dram = parse_space_size(a.hbm), parse_space_size(a.dram)
    block = parse_space_size(a.block_size)
    file_size = parse_space_size(a.file_size)
    total = int(hbm * a.factor)
    nfiles = max(1, total // file_size)
    work = tempfile.mkdtemp(prefix="ufsbench_", dir=a.work_dir)
    backing = proxy = None
    try:
        conf = {
            "alluxio.worker.tieredstore.levels": "2",
            "alluxio.worker.tieredstore.level0.alias": "MEM",
            "alluxio.worker.tieredstore.level0.dirs.path": "hbm" if torch.cuda.is_available() else "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": str(hbm),
            "alluxio.worker.tieredstore.level1.alias": "SSD",
            "alluxio.worker.tieredstore.level1.dirs.path": "dram",
            "alluxio.worker.tieredstore.level1.dirs.mediumtype": "DRAM",
            "alluxio.worker.tieredstore.level1.dirs.quota": str(dram),
            "alluxio.worker.hbm.page.size": "2MB",
            "alluxio.user.block.size.bytes.default": str(block),
            "alluxio.worker.ufs.ingest.depth": str(depth),
            "alluxio.worker.network.async.cache.manager.threads.max": str(a.threads),
            "alluxio.worker.tieredstore.eviction.demote": "true",
            "alluxio.worker.tieredstore.free.ahead.bytes": a.free_ahead,
        }
        if a.ufs == "s3native":
            # the native S3 endpoint (csrc/http_blob.cpp: sendfile GETs) over a directory whose
            # bucket holds the files; the worker's S3 UFS reads ranges natively unless disabled
            from alluxio_amd.ops.native import lib
            blob_root = os.path.join(work, "blobs")
            os.makedirs(os.path.join(blob_root, "bench", "ws"))
            proxy = lib().BlobServer(blob_root, "127.0.0.1", 0)
            proxy.start()
            props = {"alluxio.underfs.s3.endpoint": f"http://127.0.0.1:{proxy.port}", "s3a.accessKeyId": "k",
                     "s3a.secretKey": "s", "alluxio.underfs.s3.native.reader.enabled": a.native_reader}
            for k, v in props.items():
                conf[f"alluxio.master.mount.table.root.option.{k}"] = v
            conf["alluxio.master.mount.table.root.ufs"] = "s3://bench/"

            def wr(p, d):
                with open(os.path.join(blob_root, "bench") + p, "wb") as f:
                    f.write(d)
            _write_working_set(wr, nfiles, file_size)
            cluster = LocalAlluxioCluster(num_workers=1, work_dir=os.path.join(work, "main"), conf=conf)
        elif a.ufs == "s3":
            from alluxio_amd.proxy import ProxyServer
            backing = LocalAlluxioCluster(num_workers=1, work_dir=os.path.join(work, "backing"), conf={
                "alluxio.worker.tieredstore.level0.dirs.path": "dram",
                "alluxio.worker.tieredstore.level0.dirs.quota": "256MB"}).start()
            bfs = backing.client()
            bfs.create_directory("/bench")
            proxy = ProxyServer(bfs, port=0)
            port = proxy.start()
            props = {"alluxio.underfs.s3.endpoint": f"http://127.0.0.1:{port}", "s3a.accessKeyId": "k",
                     "s3a.secretKey": "s"}
            for k, v in props.items():
                conf[f"alluxio.master.mount.table.root.option.{k}"] = v
            conf["alluxio.master.mount.table.root.ufs"] = "s3://bench/"
            from alluxio_amd.underfs import registry
            s3 = registry.create("s3://bench/", None, props)
            _write_working_set(lambda p, d: s3.write_all("s3://bench" + p, d), nfiles, file_size)
            cluster = LocalAlluxioCluster(num_workers=1, work_dir=os.path.join(work, "main"), conf=conf)
        else:
            ufs_dir = os.path.join(work, "ufs")
            os.makedirs(os.path.join(ufs_dir, "ws"))

            def wr(p, d):
                with open(ufs_dir + p, "wb") as f:
                    f.write(d)
            _write_working_set(wr, nfiles, file_size)
            conf["alluxio.master.mount.table.root.ufs"] = ufs_dir
            cluster = LocalAlluxioCluster(num_workers=1, work_dir=os.path.join(work, "main"), conf=conf)
        cluster.start()
        with cluster:
            fs = cluster.client()
            files = sorted((s for s in fs.list_status("/ws") if not s.is_folder), key=lambda s: s.path)
            w = cluster.workers[0].worker
            reqs = []
            for st in files:
                info = fs.get_status(st.path).info
                for idx, fbi in enumerate(info.fileBlockInfos):
                    opts = pb.dataserver.OpenUfsBlockOptions(
                        ufs_path=info.ufsPath, offset_in_file=idx * info.blockSizeBytes,
                        block_size=fbi.blockInfo.length, mountId=info.mountId)
                    reqs.append((fbi.blockInfo.blockId, opts))
            nbytes = sum(o.block_size for _, o in reqs)
            import logging
            fails = []

            class _Fail(logging.Handler):
                def emit(self, rec):
                    if rec.exc_info and len(fails) < 3:
                        fails.append(f"{rec.getMessage()}: {rec.exc_info[1]!r}")
            blog = logging.getLogger("alluxio_amd.worker.block_worker")
            blog.setLevel(logging.DEBUG)
            blog.addHandler(_Fail())
            t0 = time.perf_counter()
            for bid, opts in reqs:
                w.async_cache(bid, opts=opts)
            ok = w.wait_async_idle(timeout=a.timeout)
            el = time.perf_counter() - t0
            # where the ingest threads spent their time (the bound): UFS reads, waits for the H2D
            # DMA to free a staging buffer, and the per-page CRC32C kernel at commit
            pipes = list(w._ingest._free) if w._ingest is not None else []
            stage = {k: round(sum(p.stats[k] for p in pipes), 3) for k in ("read_s", "wait_s")}
            stage["chunks"] = sum(p.stats["chunks"] for p in pipes)
            crc_t = w.metrics.timer("Crc32cCommit")
            stage["crc_s"] = round(crc_t._fold_sum(), 3)
            stage["threads_x_wall_s"] = round(el * a.threads, 3)
            cached = sum(1 for bid, _ in reqs if w.has_block(bid))
            cached_bytes = sum(o.block_size for bid, o in reqs if w.has_block(bid))
            st = w.native.evict_stats()
            tiers = {}
            for bid in w.native.block_ids(-1):
                inf = w.native.block_info(bid)
                tiers[inf.medium] = tiers.get(inf.medium, 0) + inf.length
            # re-read the blocks that are still cached into one device buffer (hot read)
            dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
            buf = torch.empty(block, dtype=torch.uint8, device=dev)
            kind = 1 if dev.type == "cuda" else 0
            t1 = time.perf_counter()
            rb = 0
            for bid, opts in reqs:
                if not w.has_block(bid):
                    continue
                lk = w.lock_block(99, bid)
                try:
                    w.read(bid, 0, opts.block_size, buf.data_ptr(), kind, 0, False)
                finally:
                    w.unlock(lk)
                rb += opts.block_size
            if dev.type == "cuda":
                torch.cuda.synchronize()
            rel = time.perf_counter() - t1
            fs.close()
            return {"ufs": a.ufs if a.ufs != "s3native" else f"s3native(reader={a.native_reader})", "depth": depth, "hbm_bytes": hbm, "dram_bytes": dram, "working_set": nbytes,
                    "blocks": len(reqs), "cached_blocks": cached, "all_done": ok,
                    "ingest_GBps": round(cached_bytes / el / 1e9, 3), "ingest_s": round(el, 3),
                    "failed_blocks": w.metrics.counter("AsyncCacheFailedBlocks").value(), "first_failures": fails,
                    "demoted_blocks": st["demoted_blocks"], "demoted_bytes": st["demoted_bytes"],
                    "batched_moves": st["batched_moves"], "evict_waits": st.get("evict_waits"), "evict_retries": st.get("evict_retries"), "revalidated_away": st.get("revalidated_away"), "resident_by_medium": tiers,
                    "reread_GBps": round(rb / rel / 1e9, 3) if rel > 0 else None, "reread_bytes": rb,
                    "threads": a.threads, "free_ahead": a.free_ahead, "stages": stage}
    finally:
        if proxy is not None:
            proxy.stop()
        if backing is not None:
            backing.stop()
        shutil.rmtree(work, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ufs", choices=("local", "s3", "s3native"), default="local")
    ap.add_argument("--native-reader", choices=("true", "false"), default="true",
                    help="s3native: receive ranged GETs natively (else the requests client)")
    ap.add_argument("--hbm", default="2g")
    ap.add_argument("--dram", default="6g")
    ap.add_argument("--factor", type=float, default=2.0)
    ap.add_argument("--file-size", default="256m")
    ap.add_argument("--block-size", default="64m")
    ap.add_argument("--depths", default="1,3")
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--timeout", type=float, default=600)
    ap.add_argument("--work-dir", default=None)
    ap.add_argument("--free-ahead", default="0", help="alluxio.worker.tieredstore.free.ahead.bytes")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    for d in [int(x) for x in a.depths.split(",")]:
        r = run(a, d)
        line = json.dumps(r)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")


if __name__ == "__main__":
    main()
