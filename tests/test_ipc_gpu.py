"""HIP IPC short-circuit reads across processes on one MI355X.

A child process runs master + worker with an HBM tier and caches a file; this (client) process
has no worker of its own, so reads of that file go through ``OpenDeviceBlock`` + the IPC-mapped
arena + this process's batched copy kernel.  Compared against the bytes the child wrote
(reference analogue: short-circuit read tests, tests/.../client/fs/LocalBlockInStreamIntegrationTest).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SERVER = r"""
import os, sys, json
sys.path.insert(0, %(root)r)
import torch
import numpy as np
from alluxio_amd.minicluster import LocalAlluxioCluster
conf = {"alluxio.worker.tieredstore.level0.dirs.path": "hbm:0", "alluxio.worker.tieredstore.level0.dirs.quota": "256MB",
        "alluxio.worker.hbm.page.size": "1MB", "alluxio.user.block.size.bytes.default": "8MB"}
with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=%(work)r) as c:
    fs = c.client()
    data = np.random.default_rng(7).integers(0, 256, 20 * (1 << 20) + 333, dtype=np.uint8)
    fs.write_file("/ipc/f", data, write_type="MUST_CACHE")
    print(json.dumps({"master": c.master.address}), flush=True)
    sys.stdin.readline()
    fs.close()
"""


@pytest.mark.gpu
def test_ipc_read_from_other_process(gpu, tmp_path):
    import torch

    from alluxio_amd.client.file_system import FileSystem
    from alluxio_amd.conf import Configuration
    script = tmp_path / "server.py"
    script.write_text(SERVER % {"root": ROOT, "work": str(tmp_path / "work")})
    p = subprocess.Popen([sys.executable, str(script)], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        line = p.stdout.readline()
        assert line, p.stderr.read()[-3000:]
        master = json.loads(line)["master"]
        expect = np.random.default_rng(7).integers(0, 256, 20 * (1 << 20) + 333, dtype=np.uint8)
        fs = FileSystem(conf=Configuration({"alluxio.user.file.passive.cache.enabled": "false"}),
                        master_address=master)
        dst = torch.empty(len(expect), dtype=torch.uint8, device="cuda")
        with fs.open_file("/ipc/f") as f:
            n = f.read_into(dst)
            assert f._reader is not None and f._reader.source == "ipc"
        torch.cuda.synchronize()
        assert n == len(expect)
        assert np.array_equal(dst.cpu().numpy(), expect)
        # unaligned positioned read into a host buffer through the same mapping
        host = np.empty(3 << 20, dtype=np.uint8)
        with fs.open_file("/ipc/f") as f:
            assert f.pread(5 * (1 << 20) + 17, host) == len(host)
        assert np.array_equal(host, expect[5 * (1 << 20) + 17:5 * (1 << 20) + 17 + len(host)])
        # host read(buf) loop (StressWorkerBench's shape): the native reader refills its pinned
        # chunk buffer from the IPC-mapped HBM pages (D2H DMA) and serves each 4 KiB from it
        with fs.open_file("/ipc/f") as f:
            b = bytearray(4096)
            parts = []
            while True:
                n = f.readinto(b)
                if not n:
                    break
                parts.append(bytes(b[:n]))
            assert f._nreader is not None and f._nreader.source == "ipc"
            assert f._nat.refills >= len(expect) // (4 << 20)   # 4 MiB chunks (reader buffer default)
        assert b"".join(parts) == expect.tobytes()
        # short-circuit writes into the worker's HBM arena (OpenDeviceWrite + ArenaSink: pinned
        # staging, H2D DMA into the IPC-mapped pages), from host memory and from a device tensor
        wdata = np.random.default_rng(8).integers(0, 256, 19 * (1 << 20) + 5, dtype=np.uint8)
        with fs.create_file("/ipc/w", write_type="MUST_CACHE") as f:
            for i in range(0, len(wdata), 3 << 20):
                f.write(wdata[i:i + (3 << 20)])
            assert f._writers and type(f._writers[0]).__name__ == "IpcBlockWriter"
        with fs.create_file("/ipc/wd", write_type="MUST_CACHE") as f:
            f.write(torch.from_numpy(wdata[:5 << 20]).cuda())
        assert fs.read_file("/ipc/w") == wdata.tobytes()
        assert fs.read_file("/ipc/wd") == wdata[:5 << 20].tobytes()
        # one write() spanning whole blocks: they stream in parallel, one short-circuit writer each
        with fs.create_file("/ipc/big", write_type="MUST_CACHE") as f:
            f.write(wdata)
        assert fs.read_file("/ipc/big") == wdata.tobytes()
        fs.close()
        # native gRPC WriteBlock into the HBM tier (the server stages chunks through pinned memory)
        fs3 = FileSystem(conf=Configuration({"alluxio.user.file.passive.cache.enabled": "false",
                                             "alluxio.user.short.circuit.enabled": "false"}),
                         master_address=master)
        with fs3.create_file("/ipc/g", write_type="MUST_CACHE") as f:
            f.write(wdata)
            assert f._writers and type(f._writers[0]).__name__ == "GrpcBlockWriter"
            assert f._writers[0]._sink is not None
        assert fs3.read_file("/ipc/g") == wdata.tobytes()
        fs3.close()
        # the same bytes over the worker's native gRPC data port: HBM chunks staged D2H by the
        # server's I/O threads, frames parsed by the native client
        fs2 = FileSystem(conf=Configuration({"alluxio.user.file.passive.cache.enabled": "false",
                                             "alluxio.user.short.circuit.enabled": "false"}),
                         master_address=master)
        with fs2.open_file("/ipc/f") as f:
            got = f.read()
            assert f._nreader.source == "remote"
        assert got == expect.tobytes()
        # a GPU consumer of the remote worker: ReadBlock frames into pinned chunks DMA'd H2D
        dst2 = torch.zeros(len(expect), dtype=torch.uint8, device="cuda")
        with fs2.open_file("/ipc/f") as f:
            assert f.read_into(dst2) == len(expect)
            assert f._reader.source == "remote" and f._reader._nsrc
        torch.cuda.synchronize()
        assert np.array_equal(dst2.cpu().numpy(), expect)
        # the read spans 3 blocks: each went over its own stream (parallel device reads); an
        # unaligned positioned read across a block boundary, and the one-block-at-a-time path
        dst3 = torch.zeros(12 << 20, dtype=torch.uint8, device="cuda")
        with fs2.open_file("/ipc/f") as f:
            assert f.pread((3 << 20) + 7, dst3) == len(dst3)
        torch.cuda.synchronize()
        assert np.array_equal(dst3.cpu().numpy(), expect[(3 << 20) + 7:(15 << 20) + 7])
        # single-block reads into freshly zero-filled tensors: the native reader's H2D stream
        # must not overtake the fill still queued on torch's stream
        from alluxio_amd.client.streams import DEVICE
        for off, ln in [((3 << 20) + 7, (5 << 20) - 7), (3 << 20, 5 << 20), (7, 2 << 20), (0, 8 << 20)]:
            with fs2.open_file("/ipc/f") as f:
                d = torch.zeros(ln, dtype=torch.uint8, device="cuda")
                f._reader_for(0).read_into(off, ln, d.data_ptr(), DEVICE)
                torch.cuda.synchronize()
                assert np.array_equal(d.cpu().numpy(), expect[off:off + ln]), (off, ln)
        fs2.close()
        fs4 = FileSystem(conf=Configuration({"alluxio.user.file.passive.cache.enabled": "false",
                                             "alluxio.user.short.circuit.enabled": "false",
                                             "alluxio.user.device.read.parallelism": "1"}),
                         master_address=master)
        dst3.zero_()
        with fs4.open_file("/ipc/f") as f:
            assert f.pread((3 << 20) + 7, dst3) == len(dst3)
        torch.cuda.synchronize()
        assert np.array_equal(dst3.cpu().numpy(), expect[(3 << 20) + 7:(15 << 20) + 7])
        fs4.close()
    finally:
        p.stdin.write("\n")
        p.stdin.flush()
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()


def test_page_segments_merge_adjacent():
    from alluxio_amd.parallel.ipc import page_segments
    segs = page_segments(1000, [0, 1, 5], 100, 50, 200, 0)
    # bytes 50..150 from pages 0,1 (adjacent -> one seg), 150..250 page1 tail + page 5 head
    assert segs == [(1050, 0, 150), (1500, 150, 50)]


PLANE = r"""
import os, sys, json
sys.path.insert(0, %(root)r)
import numpy as np, torch, torch.distributed as dist
from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.worker.process import AlluxioWorkerProcess
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.parallel.transfer import TransferPlane
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = rank %% torch.cuda.device_count()      # one GPU per rank when the node has them
torch.cuda.set_device(dev)
backend = %(backend)r
dist.init_process_group(backend, init_method="tcp://127.0.0.1:%(port)d", rank=rank, world_size=world)
work = %(work)r
conf = Configuration({"alluxio.master.journal.folder": work + "/journal",
    "alluxio.worker.tieredstore.level0.dirs.path": "hbm:%%d" %% dev, "alluxio.worker.tieredstore.level0.dirs.quota": "256MB",
    "alluxio.worker.hbm.page.size": "1MB", "alluxio.user.block.size.bytes.default": "8MB"})
box = [None]
if rank == 0:
    m = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=work + "/ufs"); box[0] = m.start(start_heartbeats=False)
dist.broadcast_object_list(box, src=0)
w = AlluxioWorkerProcess(conf.copy(), master_address=box[0], port=0, device=dev, work_dir=work + "/w%%d" %% rank)
w.start(start_heartbeats=False)
plane = TransferPlane.establish(w.worker)
fs = FileSystem(conf=conf.copy(), master_address=box[0])
n = 20 * (1 << 20) + 11
data = np.random.default_rng(20 + rank).integers(0, 256, n, dtype=np.uint8)
fs.write_file("/gp/f%%d" %% rank, data, write_type="MUST_CACHE")
dist.barrier()
other = (rank + 1) %% world
odata = np.random.default_rng(20 + other).integers(0, 256, n, dtype=np.uint8)
st = fs.get_status("/gp/f%%d" %% other).info
ok = True
pulled = 0
for i, fbi in enumerate(st.fileBlockInfos):
    b = fbi.blockInfo
    pulled += plane.pull_block(b.blockId, b.locations[0].workerAddress, b.length)
    got = w.worker.read_bytes(b.blockId, 0, b.length)
    ok = ok and got == odata[i * (8 << 20):i * (8 << 20) + b.length].tobytes()
dist.barrier()
wm = w.worker.metrics
res = {"rank": rank, "ok": bool(ok), "pulled": pulled, "device_plane": plane.device_plane, "device": dev,
       "peer_devices": list(w.peer_devices), "xgmi": wm.counter("XgmiBytesReceived").count,
       "shared": wm.counter("PeerSharedBytesReceived").count,
       "stream": wm.counter("PeerStreamBytesReceived").count, "failures": wm.counter("PeerPullFailures").count}
if %(collective)r:
    # replicate_all: every rank contributes a fresh 2-block file; afterwards every worker holds all
    cdata = np.random.default_rng(40 + rank).integers(0, 256, (11 << 20) + 5 * rank, dtype=np.uint8)
    fs.write_file("/gp/c%%d" %% rank, torch.from_numpy(cdata).to("cuda"), write_type="MUST_CACHE")
    torch.cuda.synchronize()
    mine = [(b.blockInfo.blockId, b.blockInfo.length, rank) for b in fs.get_status("/gp/c%%d" %% rank).info.fileBlockInfos]
    allb = [None] * world
    dist.all_gather_object(allb, mine)
    blocks = [x for part in allb for x in part]
    moved = plane.replicate_all(blocks)
    good = True
    for r in range(world):
        exp = np.random.default_rng(40 + r).integers(0, 256, (11 << 20) + 5 * r, dtype=np.uint8)
        for i, (bid, n, _o) in enumerate(allb[r]):
            good = good and w.worker.read_bytes(bid, 0, n) == exp[i * (8 << 20):i * (8 << 20) + n].tobytes()
    res.update({"gathered": moved, "gather_ok": bool(good),
                "gather_expect": sum(n for _b, n, r in blocks if r != rank)})
if %(extra)r:
    from alluxio_amd.client.batch_reader import RemoteRingReader
    from alluxio_amd.client.context import worker_address_str
    from alluxio_amd.parallel.peer import fan_out
    me_addr = worker_address_str(w.worker.address)
    addrs = [None] * world
    dist.all_gather_object(addrs, me_addr)
    # fan_out: rank 0 writes one block; every other rank pulls it over xGMI (PeerTransfer)
    fdata = np.random.default_rng(77).integers(0, 256, (5 << 20) + 3, dtype=np.uint8)
    if rank == 0:
        fs.write_file("/gp/fo", fdata, write_type="MUST_CACHE")
        fb = fs.get_status("/gp/fo").info.fileBlockInfos[0].blockInfo
        errs = fan_out(me_addr, addrs[1:], fb.blockId, fb.length, fs.ctx.worker_stub)
        assert not errs, errs
    dist.barrier()
    fb = fs.get_status("/gp/fo").info.fileBlockInfos[0].blockInfo
    fan_ok = w.worker.has_block(fb.blockId) and w.worker.read_bytes(fb.blockId, 0, fb.length) == fdata.tobytes()
    # RemoteRingReader on this GPU over the next rank's HBM (the file it cached)
    streams, depth, buf = 8, 32, 4096
    ring = torch.empty((streams, depth, buf), dtype=torch.uint8, device="cuda")
    ring_ok = True
    with RemoteRingReader(fs, "/gp/f%%d" %% other, ring, addrs[other], start_offsets=[s * (1 << 20) for s in range(streams)]) as rr:
        for _ in range(3):
            rr.step()
        torch.cuda.synchronize()
        for s_ in range(streams):
            for k_ in (0, depth - 1):
                off, nb = rr.last_call(s_, k_)
                ring_ok = ring_ok and np.array_equal(ring[s_, k_, :nb].cpu().numpy(), odata[off:off + nb])
    res.update({"fan_ok": bool(fan_ok), "remote_ring_ok": bool(ring_ok)})
    if world >= 3:
        # replicate_ring, several rounds (one 8 MiB block per batch) pipelined over RCCL send/recv
        plane.batch_bytes = 8 << 20
        rdata = np.random.default_rng(60 + rank).integers(0, 256, (24 << 20) + 7, dtype=np.uint8)
        fs.write_file("/gp/r%%d" %% rank, torch.from_numpy(rdata).to("cuda"), write_type="MUST_CACHE")
        torch.cuda.synchronize()
        mine = [(b.blockInfo.blockId, b.blockInfo.length, rank) for b in fs.get_status("/gp/r%%d" %% rank).info.fileBlockInfos]
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        rblocks = [x for part in allr for x in part]
        rmoved = plane.replicate_ring(rblocks, 2)
        pred = (rank - 1) %% world
        exp = np.random.default_rng(60 + pred).integers(0, 256, (24 << 20) + 7, dtype=np.uint8)
        rgood = all(w.worker.read_bytes(b, 0, n) == exp[i * (8 << 20):i * (8 << 20) + n].tobytes()
                    for i, (b, n, _o) in enumerate(allr[pred]))
        rnot = not any(w.worker.has_block(b) for r2 in range(world) if r2 not in (rank, pred) for b, _n, _o in allr[r2])
        res.update({"ring_ok": bool(rgood and rnot), "ring_moved": rmoved, "ring_rounds": plane.rounds,
                    "ring_agreements": plane.agreements})
print(json.dumps(res), flush=True)
dist.barrier()
fs.close(); w.stop()
dist.barrier()
if rank == 0:
    m.stop()
dist.destroy_process_group()
"""


def _run_plane(tmp_path, backend: str, collective: bool, world: int = 2, extra: bool = False):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    path = tmp_path / "plane.py"
    path.write_text(PLANE % {"root": ROOT, "port": port, "work": str(tmp_path), "backend": backend,
                             "collective": collective, "extra": extra})
    procs = [subprocess.Popen([sys.executable, str(path)], env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(world)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("device pull rank timed out")
        assert p.returncode == 0, err[-3000:]
        outs.append(json.loads(out.strip().splitlines()[-1]))
    return outs


@pytest.mark.gpu
def test_transfer_plane_device_pull(gpu, tmp_path):
    """Two worker ranks (one GPU each when the node has two; else both on device 0) pull each
    other's blocks through the mapped plane; no byte may come through the gRPC fallback."""
    for o in _run_plane(tmp_path, "gloo", False):
        assert o["ok"] and o["device_plane"] and o["pulled"] == 20 * (1 << 20) + 11, o
        assert o["stream"] == 0 and o["failures"] == 0, o
        assert o["xgmi"] + o["shared"] == o["pulled"], o


@pytest.mark.gpu
def test_transfer_plane_two_gpus_xgmi_and_rccl(gpu, tmp_path):
    """Cross-device execution of the data plane: rank r runs on GPU r, enables peer access, pulls
    the peer's blocks out of the peer GPU's HBM over xGMI (counted as XgmiBytesReceived, never the
    gRPC fallback), then replicate_all moves blocks with RCCL all-gather (nccl backend)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    outs = _run_plane(tmp_path, "nccl", True)
    for o in outs:
        assert o["ok"] and o["pulled"] == 20 * (1 << 20) + 11, o
        other = 1 - o["rank"]
        assert o["device"] == o["rank"] and other in o["peer_devices"], o
        assert o["xgmi"] == o["pulled"] and o["stream"] == 0 and o["failures"] == 0, o
        assert o["gather_ok"] and o["gathered"] == o["gather_expect"], o


@pytest.mark.gpu
def test_multi_gpu_fan_out_remote_ring_and_replicate_ring(gpu, tmp_path):
    """One rank per GPU (2..4 GPUs) over RCCL: fan_out of a fresh block to every peer (xGMI pulls
    via PeerTransfer), RemoteRingReader on each GPU over the next GPU's HBM, and -- with >= 3
    GPUs -- a multi-round pipelined replicate_ring (copies=2) that leaves each block on exactly its
    owner and successor."""
    import torch
    n = min(torch.cuda.device_count(), 4)
    if n < 2:
        pytest.skip("needs two GPUs")
    outs = _run_plane(tmp_path, "nccl", True, world=n, extra=True)
    for o in outs:
        assert o["ok"] and o["gather_ok"], o
        assert o["fan_ok"] and o["remote_ring_ok"], o
        if n >= 3:
            assert o["ring_ok"] and o["ring_moved"] == (24 << 20) + 7 and o["ring_rounds"] >= 3, o


NCCL_DEATH = r"""
import os, sys, json
sys.path.insert(0, %(root)r)
import numpy as np, torch, torch.distributed as dist
from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.worker.process import AlluxioWorkerProcess
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.parallel.transfer import TransferPlane
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(rank)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%(port)d", rank=rank, world_size=world)
work = %(work)r
conf = Configuration({"alluxio.master.journal.folder": work + "/journal",
    "alluxio.worker.tieredstore.level0.dirs.path": "hbm:%%d" %% rank, "alluxio.worker.tieredstore.level0.dirs.quota": "256MB",
    "alluxio.worker.hbm.page.size": "1MB", "alluxio.user.block.size.bytes.default": "4MB"})
box = [None]
if rank == 0:
    m = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=work + "/ufs"); box[0] = m.start(start_heartbeats=False)
dist.broadcast_object_list(box, src=0)
w = AlluxioWorkerProcess(conf.copy(), master_address=box[0], port=0, device=rank, work_dir=work + "/w%%d" %% rank)
w.start(start_heartbeats=False)
plane = TransferPlane.establish(w.worker, rebuild_wait_s=3.0, timeout_s=20.0, batch_bytes=4 << 20)
fs = FileSystem(conf=conf.copy(), master_address=box[0])
data = np.random.default_rng(20 + rank).integers(0, 256, (12 << 20) + 11, dtype=np.uint8)
fs.write_file("/rb/f%%d" %% rank, data, write_type="MUST_CACHE")
mine = [(b.blockInfo.blockId, b.blockInfo.length, rank) for b in fs.get_status("/rb/f%%d" %% rank).info.fileBlockInfos]
allb = [None] * world
dist.all_gather_object(allb, mine)
blocks = [x for part in allb for x in part]
if rank == world - 1:
    orig = plane._scatter_batches
    def dying(*a, **kw):
        r = orig(*a, **kw)
        torch.cuda.synchronize()
        os._exit(0)           # dies after posting its first round
    plane._scatter_batches = dying
moved = plane.%(method)s
alive = list(range(world - 1))
have = all(w.worker.has_block(b) for b, _, o in blocks if o in alive) if %(method)r.startswith("replicate_all") else True
print(json.dumps({"rank": rank, "moved": moved, "rebuilds": plane.rebuilds, "members": plane.members,
                  "have_alive": have}), flush=True)
os._exit(0)
"""


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["replicate_all(blocks)", "replicate_ring(blocks, 2)"])
def test_nccl_rank_death_rebuilds_plane(gpu, tmp_path, method):
    """RCCL analogue of test_distributed.py::test_replicate_all_rebuilds_group_after_rank_death:
    one GPU rank dies mid-collective; the survivors' bounded waits fail (or see the rebuild
    marker), the communicator is aborted, and they finish on a rebuilt RCCL group without it --
    no survivor is torn down by the watchdog."""
    import socket

    import torch
    world = min(torch.cuda.device_count(), 4)
    if world < 3:
        pytest.skip("needs three GPUs")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    path = tmp_path / "death.py"
    path.write_text(NCCL_DEATH % {"root": ROOT, "port": port, "work": str(tmp_path), "method": method})
    procs = [subprocess.Popen([sys.executable, str(path)], env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(world)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    for r, p in enumerate(procs):
        try:
            out, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("rank death test timed out")
        if r < world - 1:
            assert p.returncode == 0, err[-3000:]
            outs.append(json.loads(out.strip().splitlines()[-1]))
    for o in outs:
        assert o["rebuilds"] >= 1 and o["members"] == list(range(world - 1)), o
        assert o["have_alive"], o


@pytest.mark.gpu
def test_remote_ring_reader_other_process(gpu, tmp_path):
    """RemoteRingReader: the device-cursor ring kernel on this process's GPU reads a file cached
    in another worker process's HBM arena (IPC-mapped), 4 KiB calls into a [streams, depth, buf]
    ring; every sampled call's bytes equal the file bytes at its offset."""
    import torch

    from alluxio_amd.client.batch_reader import RemoteRingReader
    from alluxio_amd.client.context import worker_address_str
    from alluxio_amd.client.file_system import FileSystem
    from alluxio_amd.conf import Configuration
    script = tmp_path / "server.py"
    script.write_text(SERVER % {"root": ROOT, "work": str(tmp_path / "work")})
    p = subprocess.Popen([sys.executable, str(script)], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        line = p.stdout.readline()
        assert line, p.stderr.read()[-3000:]
        master = json.loads(line)["master"]
        expect = np.random.default_rng(7).integers(0, 256, 20 * (1 << 20) + 333, dtype=np.uint8)
        fs = FileSystem(conf=Configuration({}), master_address=master)
        st = fs.get_status("/ipc/f")
        addr = worker_address_str(st.fileBlockInfos[0].blockInfo.locations[0].workerAddress)
        streams, depth, buf = 16, 64, 4096
        ring = torch.empty((streams, depth, buf), dtype=torch.uint8, device="cuda")
        starts = [s * (1 << 20) for s in range(streams)]
        with RemoteRingReader(fs, "/ipc/f", ring, addr, start_offsets=starts) as r:
            for _ in range(3):
                r.step()
            torch.cuda.synchronize()
            for s in range(streams):
                for k in (0, depth // 2, depth - 1):
                    off, n = r.last_call(s, k)
                    assert np.array_equal(ring[s, k, :n].cpu().numpy(), expect[off:off + n]), (s, k)
            assert r.total_bytes == 3 * streams * depth * buf
        fs.close()
    finally:
        p.stdin.write("\n")
        p.stdin.flush()
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()


SERVER_CORRUPT = r"""
import os, sys, json
sys.path.insert(0, %(root)r)
import torch
import numpy as np
from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.ops.native import lib
conf = {"alluxio.worker.tieredstore.level0.dirs.path": "hbm:0", "alluxio.worker.tieredstore.level0.dirs.quota": "256MB",
        "alluxio.worker.hbm.page.size": "1MB", "alluxio.user.block.size.bytes.default": "8MB"}
with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=%(work)r) as c:
    fs = c.client()
    data = np.random.default_rng(3).integers(0, 256, 5 * (1 << 20) + 17, dtype=np.uint8)
    fs.write_file("/crc/f", data, write_type="MUST_CACHE")
    bid = fs.get_status("/crc/f").info.blockIds[0]
    w = c.workers[0].worker
    print(json.dumps({"master": c.master.address, "worker": "127.0.0.1:%%d" %% w.address.rpcPort,
                      "block": bid, "crcs": len(w.crc.get(bid, (0, []))[1])}), flush=True)
    sys.stdin.readline()
    pages, d, ps, base = w.native.block_pages(bid)
    lib().fill_pattern(base + pages[1] * ps + 4096, 4096, 99, 0, 0)   # flip bytes in page 1
    torch.cuda.synchronize()
    print("corrupted", flush=True)
    sys.stdin.readline()
    fs.close()
"""


@pytest.mark.gpu
def test_ipc_open_verifies_crc(gpu, tmp_path):
    """HBM blocks carry per-page CRC32Cs from commit; a short-circuit reader verifying them at
    open accepts the intact block and rejects one whose page was overwritten."""
    from alluxio_amd.parallel.ipc import verify_handle_crc
    from alluxio_amd.proto import pb
    from alluxio_amd.rpc import Channel
    from alluxio_amd.utils.exceptions import DataLossException
    script = tmp_path / "server.py"
    script.write_text(SERVER_CORRUPT % {"root": ROOT, "work": str(tmp_path / "work")})
    p = subprocess.Popen([sys.executable, str(script)], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        line = p.stdout.readline()
        assert line, p.stderr.read()[-3000:]
        info = json.loads(line)
        assert info["crcs"] == 6          # one block of 5 MB + 17 B: a CRC per 1 MB page
        stub = Channel(info["worker"], force_grpc=True).stub("alluxio.grpc.block.BlockWorker")

        def open_verify():
            h = stub.OpenDeviceBlock(pb.block.OpenDeviceBlockRequest(block_id=info["block"], session_id=4242))
            try:
                assert len(h.crc32c) == 6
                verify_handle_crc(h, 0)
            finally:
                stub.UnlockDeviceBlock(pb.block.UnlockDeviceBlockRequest(block_id=info["block"], lock_id=h.lock_id,
                                                                         session_id=4242))
        open_verify()
        p.stdin.write("go\n")
        p.stdin.flush()
        assert p.stdout.readline().strip() == "corrupted"
        with pytest.raises(DataLossException):
            open_verify()
    finally:
        try:
            p.stdin.write("quit\n")
            p.stdin.flush()
        except Exception:  # noqa: BLE001
            pass
        p.wait(timeout=60)


ARENA_CHILD = r"""
import sys, json
sys.path.insert(0, %(root)r)
import torch
from alluxio_amd.ops.native import lib
handle, offset, nbytes, probes = bytes.fromhex(%(handle)r), %(offset)d, %(nbytes)d, %(probes)r
base = lib().ipc_open_bounded(handle, 0, %(timeout_ms)d) + offset
out = {}
for off in probes:                       # read 4 KiB at each probe, write its complement back
    dst = torch.empty(4096, dtype=torch.uint8, device="cuda")
    lib().batched_copy([(base + off, dst.data_ptr(), 4096)], 0)
    torch.cuda.synchronize()
    out[off] = int(dst.to(torch.int64).sum().item())
    inv = (255 - dst).contiguous()
    lib().batched_copy([(inv.data_ptr(), base + off, 4096)], 0)
torch.cuda.synchronize()
print(json.dumps({str(k): v for k, v in out.items()}), flush=True)
"""


def _import_probe(tmp_path, handle, offset, nbytes, probes, timeout_ms=60000):
    script = tmp_path / "child.py"
    script.write_text(ARENA_CHILD % {"root": ROOT, "handle": handle.hex(), "offset": offset, "nbytes": nbytes,
                                     "probes": probes, "timeout_ms": timeout_ms})
    return subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=150)


@pytest.mark.gpu
def test_unpadded_arena_import_times_out(gpu, tmp_path):
    """Pins why worker/store.py pads HBM arenas (ipc_safe_size): a plain 3 GiB hipMalloc (bit 31 of
    the size set) cannot be imported by another process -- hipIpcOpenMemHandle does not return --
    and the bounded open turns that into IpcTimeout instead of a hung reader."""
    from alluxio_amd.ops.native import lib
    from alluxio_amd.parallel.ipc import export_handle
    from alluxio_amd.worker.store import _device_tensor, ipc_safe_size
    nbytes = 3 << 30
    assert ipc_safe_size(nbytes) == 4 << 30 and ipc_safe_size(5 << 30) == 5 << 30
    ptr = lib().device_arena_alloc(nbytes, 0)
    try:
        t = _device_tensor(ptr, nbytes, 0)
        handle, offset = export_handle(t)
        p = _import_probe(tmp_path, handle, offset, nbytes, [0], timeout_ms=15000)
        assert p.returncode != 0 and "IpcTimeout" in p.stderr, (p.stdout, p.stderr[-2000:])
    finally:
        lib().device_arena_free(ptr, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("gib", [3, 6])
def test_native_hbm_arena_imports_from_other_process(gpu, tmp_path, gib):
    """The worker's HBM arena is one native hipMalloc (worker/store.py Arena), padded to an
    importable size: another process imports a 3 or 6 GiB tier's arena through the bounded HIP IPC
    open, reads pages at its start, middle and end and writes into them; both sides see the same
    bytes."""
    import torch

    from alluxio_amd.parallel.ipc import export_handle
    from alluxio_amd.worker.store import Arena, ipc_safe_size
    nbytes = gib << 30
    a = Arena("hbm", nbytes, 0, ipc_safe_size(nbytes))
    probes = [0, nbytes // 2 + 12288, nbytes - 4096]
    for off in probes:
        a.tensor[off:off + 4096].copy_(torch.arange(4096, device="cuda", dtype=torch.int64).remainder(251)
                                       .to(torch.uint8) + (off % 3))
    torch.cuda.synchronize()
    handle, offset = export_handle(a.tensor)
    p = _import_probe(tmp_path, handle, offset, nbytes, probes)
    assert p.returncode == 0, p.stderr[-3000:]
    sums = json.loads(p.stdout.strip().splitlines()[-1])
    for off in probes:
        want = torch.arange(4096, dtype=torch.int64).remainder(251) + (off % 3)
        assert sums[str(off)] == int(want.sum())
        got = a.tensor[off:off + 4096].cpu().to(torch.int64)
        assert torch.equal(got, 255 - want)
    from alluxio_amd.ops.native import lib
    lib().device_arena_free(a._dptr, 0)
