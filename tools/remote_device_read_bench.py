#!/usr/bin/env python3
"""GPU consumer of a block held by another worker process, read over gRPC ``ReadBlock`` (the
path for data cached on another node; on one node short-circuit IPC is normally used instead).

A worker with an HBM tier caches a file in this process; a separate client process with
short-circuit off reads it with ``FileInStream.read_into(cuda_tensor)`` in ``--read-size`` pieces,
``--reps`` times.  The client reads either through the native client (``GrpcBlockSource``: frames
into pinned chunks, H2D DMA overlapped with the next chunk) or, with
``--grpcio``, through the grpcio stream plus a host copy.

    python tools/remote_device_read_bench.py --file-size 1g --out gpurun_out/remote_device_read.jsonl

A read larger than a block spans several blocks, which the client reads at once
(``alluxio.user.device.read.parallelism``, set with ``--client-prop``).  ``--dest host`` reads into
a numpy buffer instead of a device tensor; ``--cold`` writes the file THROUGH (UFS only) and times
the one read-through.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CLIENT = r"""
import json, sys, time
sys.path.insert(0, {root!r})
import torch
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.conf import Configuration
fs = FileSystem(conf=Configuration({props!r}), master_address={addr!r})
import numpy as np
dst = torch.empty({read}, dtype=torch.uint8, device="cuda") if {dest!r} == "cuda" else np.empty({read}, dtype=np.uint8)
def once():
    n = 0
    with fs.open_file("/rd/data") as f:
        while True:
            k = f.read_into(dst)
            if not k:
                break
            n += k
    if {dest!r} == "cuda":
        torch.cuda.synchronize()
    return n
if not {cold}:
    once()
else:
    # a cold read of a 4-block file first: registers the mount and warms as many block streams
    # (connections, client staging buffers) as the measured read uses
    with fs.open_file("/rd/warm") as f:
        wbuf = torch.empty(f.length, dtype=torch.uint8, device="cuda") if {dest!r} == "cuda" else np.empty(f.length, dtype=np.uint8)
        while f.read_into(wbuf):
            pass
import os
c0 = os.times()
t0 = time.perf_counter()
total = sum(once() for _ in range({reps}))
el = time.perf_counter() - t0
c1 = os.times()
cpu = (c1.user - c0.user) + (c1.system - c0.system)
print("RESULT " + json.dumps({{"bytes": total, "seconds": el, "client_cpu_cores": cpu / el,
                              "client_sys_cores": (c1.system - c0.system) / el}}), flush=True)
fs.close()
"""


def _io_thread_cpu() -> dict:
    """CPU seconds of this process's native RPC I/O threads ("frpc-io-N"), by thread id."""
    out = {}
    tck = os.sysconf("SC_CLK_TCK")
    for t in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{t}/stat") as f:
                s = f.read()
        except OSError:
            continue
        if "(frpc-io-" not in s:
            continue
        fl = s.rsplit(")", 1)[1].split()
        out[t] = (int(fl[11]) + int(fl[12])) / tck
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--file-size", default="1g")
    ap.add_argument("--read-size", default="64m")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dest", default="cuda", choices=("cuda", "host"),
                    help="read into a device tensor or a host (numpy) buffer")
    ap.add_argument("--cold", action="store_true",
                    help="the file is written THROUGH (in the UFS only): one timed read-through, no warm-up")
    ap.add_argument("--native-only", action="store_true", help="skip the grpcio comparison row")
    ap.add_argument("--client-prop", action="append", default=[], help="extra client property k=v")
    ap.add_argument("--worker-prop", action="append", default=[], help="extra worker property k=v")
    ap.add_argument("--tier", default="hbm:0", help="worker tier path (hbm:0, or dram for a host-only box)")
    ap.add_argument("--uds", action="store_true",
                    help="the worker also listens on a Unix domain socket and the client reaches it there")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    import numpy as np

    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.utils.format import parse_space_size
    size = parse_space_size(a.file_size)
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": a.tier,
            "alluxio.worker.tieredstore.level0.dirs.quota": str(size + (1 << 30)),
            "alluxio.worker.hbm.page.size": "2MB", "alluxio.user.block.size.bytes.default": "64MB",
            "alluxio.security.authorization.permission.enabled": "false"}
    uds_dir = None
    if a.uds:        # sun_path is limited to 108 bytes: a short directory under /tmp
        uds_dir = tempfile.mkdtemp(prefix="uds", dir="/tmp")
        conf["alluxio.worker.data.server.domain.socket.address"] = uds_dir
        conf["alluxio.worker.data.server.domain.socket.as.uuid"] = "true"
    else:            # loopback TCP (the worker's default same-node domain socket off)
        conf["alluxio.worker.data.server.domain.socket.default.enabled"] = "false"
    conf.update(dict(kv.split("=", 1) for kv in a.worker_prop))
    with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=tempfile.mkdtemp(prefix="rdbench_")) as c:
        fs = c.client()
        fs.write_file("/rd/data", np.random.default_rng(0).integers(0, 256, size, dtype=np.uint8),
                      write_type="THROUGH" if a.cold else "MUST_CACHE")
        fs.write_file("/rd/warm", np.zeros(min(size, 256 << 20), dtype=np.uint8), write_type="THROUGH")
        for native in ((True,) if a.native_only else (True, False)):
            if a.cold:       # every client starts from an empty cache
                fs.free("/rd", recursive=True)
                c.heartbeat_workers()
            ds = c.workers[0].data_server
            st0 = (ds.stats.cold_streams, ds.stats.declined, ds.stats.cold_cached, ds.stats.zero_copy_frames,
                   ds.stats.prefetched, ds.stats.domain_bytes, ds.stats.cold_timing_ns,
                   ds.stats.send_timing, ds.stats.cold_readahead_hits,
                   ds.stats.cold_readahead_bytes) if ds is not None else None
            props = {"alluxio.user.network.inprocess.transport.enabled": "false",
                     "alluxio.user.short.circuit.enabled": "false",
                     "alluxio.user.native.reader.enabled": str(native).lower(),
                     "alluxio.user.file.passive.cache.enabled": "false"}
            props.update(dict(kv.split("=", 1) for kv in a.client_prop))
            io0 = _io_thread_cpu()
            p = subprocess.run([sys.executable, "-c", CLIENT.format(root=ROOT, props=props, addr=c.master.address,
                                                                   read=parse_space_size(a.read_size), reps=1 if a.cold else a.reps, dest=a.dest,
                                                                   cold=a.cold)],
                               capture_output=True, text=True, timeout=900)
            line = next((ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")), None)
            if line is None:
                print(p.stdout[-2000:], p.stderr[-3000:], file=sys.stderr)
                return 1
            r = json.loads(line[7:])
            io1 = _io_thread_cpu()
            row = {"bench": "GPU consumer of a remote worker's blocks (gRPC ReadBlock into a device tensor)"
                   if a.dest == "cuda" else "host consumer of a remote worker's blocks (gRPC ReadBlock into a numpy buffer)",
                   "client": "native GrpcBlockSource + pinned H2D" if native else "grpcio stream + host copy",
                   "file_size": a.file_size, "read_size": a.read_size, "bytes": r["bytes"],
                   "seconds": round(r["seconds"], 3), "GBps": round(r["bytes"] / r["seconds"] / 1e9, 3),
                   "transport": "uds" if a.uds else "tcp", "client_props": a.client_prop, "worker_props": a.worker_prop, "cold": a.cold, "tier": a.tier,
                   "client_cpu_cores": round(r["client_cpu_cores"], 2), "client_sys_cores": round(r["client_sys_cores"], 2),
                   # the worker's I/O threads (busiest one): 1.0 = that thread is the bound
                   "worker_io_busiest_cores": round(max((io1.get(k, 0) - io0.get(k, 0) for k in io1), default=0)
                                                    / max(r["seconds"], 1e-9), 2)}
            if st0 is not None:
                row["worker_native_cold_streams"] = ds.stats.cold_streams - st0[0]
                row["worker_declined_to_python"] = ds.stats.declined - st0[1]
                row["worker_cold_cached_blocks"] = ds.stats.cold_cached - st0[2]
                row["worker_zero_copy_frames"] = ds.stats.zero_copy_frames - st0[3]
                row["worker_prefetched_chunks"] = ds.stats.prefetched - st0[4]
                row["worker_domain_socket_bytes"] = ds.stats.domain_bytes - st0[5]
                # next-block read-ahead: cold-stream UFS reads served by bytes read ahead, and those bytes
                row["worker_readahead_hits"] = ds.stats.cold_readahead_hits - st0[8]
                row["worker_readahead_bytes"] = ds.stats.cold_readahead_bytes - st0[9]
                # the send side per block stream (ms): call start -> first / last byte, and the gaps
                # with nothing to send (ack window full / next bytes not there yet)
                kind = "cold" if a.cold else "cached"
                t1, t0 = ds.stats.send_timing[kind], st0[7][kind]
                ns = max(t1["streams"] - t0["streams"], 1)
                row["worker_send_ms_per_block"] = {
                    "streams": t1["streams"] - t0["streams"],
                    **{k[:-3]: round((t1[k] - t0[k]) / ns / 1e6, 3) for k in ("life_ns", "first_ns", "window_ns", "data_ns")},
                    "window_stalls": round((t1["window_stalls"] - t0["window_stalls"]) / ns, 1),
                    "data_stalls": round((t1["data_stalls"] - t0["data_stalls"]) / ns, 1)}
                if a.cold:
                    # the cold readers' time per block stream (ms)
                    ct = ds.stats.cold_timing_ns
                    nb = max(row["worker_native_cold_streams"], 1)
                    row["worker_cold_ms_per_block"] = {k: round((v - st0[6][k]) / nb / 1e6, 3) for k, v in ct.items()}
            print(json.dumps(row), flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(json.dumps(row) + "\n")
        fs.close()
    if uds_dir:
        import shutil
        shutil.rmtree(uds_dir, ignore_errors=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
