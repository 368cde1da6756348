"""Multi-process cluster over gloo (the CPU rehearsal of the one-worker-per-GPU layout).

Rank 0 hosts the master; every rank hosts a worker and a client, writes its own file to its
local worker, then reads the *other* rank's file (remote gRPC ReadBlock path) and its own file
through the batched read session.  The reference's equivalent is MultiProcessCluster-based
tests (minicluster/.../MultiProcessCluster.java, MultiWorkerIntegrationTest.java).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER_SCRIPT = r"""
import os, sys, json, hashlib
sys.path.insert(0, %(root)r)
import numpy as np, torch, torch.distributed as dist
from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.worker.process import AlluxioWorkerProcess
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.client.batch_reader import MultiStreamReader
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d", rank=rank, world_size=world)
work = %(work)r
conf = Configuration({"alluxio.master.journal.folder": work + "/journal",
    "alluxio.worker.tieredstore.level0.dirs.path": "dram", "alluxio.worker.tieredstore.level0.dirs.quota": "64MB",
    "alluxio.worker.hbm.page.size": "1MB", "alluxio.user.block.size.bytes.default": "4MB",
    "alluxio.security.authorization.permission.enabled": "false"})
box = [None]
if rank == 0:
    m = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=work + "/ufs"); box[0] = m.start(start_heartbeats=False)
dist.broadcast_object_list(box, src=0)
w = AlluxioWorkerProcess(conf.copy(), master_address=box[0], port=0, work_dir=work + "/w%%d" %% rank)
w.start(start_heartbeats=False)
fs = FileSystem(conf=conf.copy(), master_address=box[0], metadata_cache=True)
data = np.random.default_rng(rank).integers(0, 256, 10 * (1 << 20) + 5, dtype=np.uint8)
fs.write_file("/dist/f%%d" %% rank, data, write_type="CACHE_THROUGH")
dist.barrier()
other = (rank + 1) %% world
peer = np.random.default_rng(other).integers(0, 256, 10 * (1 << 20) + 5, dtype=np.uint8)
got = fs.read_file("/dist/f%%d" %% other)
ok_remote = got == peer.tobytes()
bufs = [torch.empty(1 << 20, dtype=torch.uint8) for _ in range(4)]
r = MultiStreamReader(fs, "/dist/f%%d" %% rank, bufs, start_offsets=[0, 1 << 20, 2 << 20, 3 << 20])
for _ in range(3):
    r.step()
ok_local = all(np.array_equal(b.numpy(), data[(i + 2) << 20:(i + 3) << 20]) for i, b in enumerate(bufs))
r.close()
workers = len(fs.workers())
dist.barrier()
print(json.dumps({"rank": rank, "remote": bool(ok_remote), "local": bool(ok_local), "workers": workers}), flush=True)
fs.close(); w.stop()
dist.barrier()
if rank == 0:
    m.stop()
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_cluster(tmp_path):
    script = WORKER_SCRIPT % {"root": ROOT, "port": _free_port(), "work": str(tmp_path)}
    path = tmp_path / "rank.py"
    path.write_text(script)
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, str(path)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            pytest.fail("distributed rank timed out")
        assert p.returncode == 0, err[-3000:]
        outs.append(json.loads(out.strip().splitlines()[-1]))
    for o in outs:
        assert o["remote"] and o["local"] and o["workers"] == 2, o


def test_bench_cpu_smoke(tmp_path, capsys):
    sys.path.insert(0, ROOT)
    import bench
    rc = bench.main(["--steps", "5", "--warmup", "1", "--threads", "8", "--file-size", "8m", "--block-size", "4m",
                     "--buffer-size", "1m", "--page-size", "1m", "--duration", "0.1", "--work-dir", str(tmp_path)])
    assert rc == 0
    line = capsys.readouterr().out.strip().splitlines()[-1]
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["config"]["verified"] and out["value"] > 0


PLANE_SCRIPT = r"""
import os, sys, json
sys.path.insert(0, %(root)r)
import numpy as np, torch, torch.distributed as dist
from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.worker.process import AlluxioWorkerProcess
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.parallel.transfer import TransferPlane
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d", rank=rank, world_size=world)
work = %(work)r
conf = Configuration({"alluxio.master.journal.folder": work + "/journal",
    "alluxio.worker.tieredstore.level0.dirs.path": "dram", "alluxio.worker.tieredstore.level0.dirs.quota": "128MB",
    "alluxio.worker.hbm.page.size": "1MB", "alluxio.user.block.size.bytes.default": "4MB"})
box = [None]
if rank == 0:
    m = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=work + "/ufs"); box[0] = m.start(start_heartbeats=False)
dist.broadcast_object_list(box, src=0)
w = AlluxioWorkerProcess(conf.copy(), master_address=box[0], port=0, work_dir=work + "/w%%d" %% rank)
w.start(start_heartbeats=False)
plane = TransferPlane.establish(w.worker)
fs = FileSystem(conf=conf.copy(), master_address=box[0])
sizes = [9 * (1 << 20) + 7, 5 * (1 << 20) + 1]
data = np.random.default_rng(10 + rank).integers(0, 256, sizes[rank %% 2], dtype=np.uint8)
fs.write_file("/plane/f%%d" %% rank, data, write_type="MUST_CACHE")
st = fs.get_status("/plane/f%%d" %% rank)
mine = [(b.blockInfo.blockId, b.blockInfo.length, rank) for b in st.info.fileBlockInfos]
allb = [None] * world
dist.all_gather_object(allb, mine)
blocks = [x for part in allb for x in part]
moved = plane.replicate_all(blocks)
ok_all = all(w.worker.has_block(b) for b, _, _ in blocks)
# bytes of the other rank's first block now readable from this worker's own store
other = (rank + 1) %% world
odata = np.random.default_rng(10 + other).integers(0, 256, sizes[other %% 2], dtype=np.uint8)
ok_bytes, at = True, 0
for ob, olen, _ in allb[other]:      # every block of the peer's packed batch landed intact
    ok_bytes = ok_bytes and w.worker.read_bytes(ob, 0, olen) == odata[at:at + olen].tobytes()
    at += olen
dist.barrier()
w.sync.heartbeat()
dist.barrier()
locs = len(fs.get_status("/plane/f%%d" %% other).info.fileBlockInfos[0].blockInfo.locations)
# on-demand pull of a block that only the peer holds (gRPC fallback on CPU)
fs.write_file("/plane/g%%d" %% rank, data[:(1 << 20) + 3], write_type="MUST_CACHE")
dist.barrier()
g = fs.get_status("/plane/g%%d" %% other).info.fileBlockInfos[0].blockInfo
pulled = plane.pull_block(g.blockId, g.locations[0].workerAddress, g.length)
ok_pull = w.worker.read_bytes(g.blockId, 0, g.length) == odata[:(1 << 20) + 3].tobytes()
print(json.dumps({"rank": rank, "all": ok_all, "bytes": bool(ok_bytes), "moved": moved, "locs": locs,
                  "pulled": pulled, "pull_ok": bool(ok_pull), "reach": plane.can_reach(g.locations[0].workerAddress)}), flush=True)
dist.barrier()
fs.close(); w.stop()
dist.barrier()
if rank == 0:
    m.stop()
dist.destroy_process_group()
"""


def test_transfer_plane_gloo(tmp_path):
    script = PLANE_SCRIPT % {"root": ROOT, "port": _free_port(), "work": str(tmp_path)}
    path = tmp_path / "plane.py"
    path.write_text(script)
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, str(path)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            pytest.fail("transfer plane rank timed out")
        assert p.returncode == 0, err[-3000:]
        outs.append(json.loads(out.strip().splitlines()[-1]))
    for o in outs:
        assert o["all"] and o["bytes"] and o["pull_ok"] and o["reach"], o
        assert o["locs"] == 2 and o["pulled"] > 0 and o["moved"] > 0, o


def test_cross_page_segments():
    from alluxio_amd.parallel.transfer import cross_page_segments
    # src pages of 4 bytes [2, 3] (contiguous), dst pages of 2 bytes [0, 5, 6, 7]
    segs = cross_page_segments(100, [2, 3], 4, 1000, [0, 5, 6, 7], 2, 0, 8)
    assert segs == [(108, 1000, 2), (110, 1010, 6)]


def test_bench_two_ranks_gloo(tmp_path):
    """The driver's multi-GPU launch shape (torch.distributed.run, one rank per worker), on gloo."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--threads", "4", "--file-size", "8m",
           "--block-size", "4m", "--work-dir", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1                      # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "workers2" and out["config"]["verified"]


COLLECTIVE_LOAD_SCRIPT = r"""
import os, sys, json, time
sys.path.insert(0, %(root)r)
import numpy as np, torch.distributed as dist
from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.worker.process import AlluxioWorkerProcess
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.parallel.transfer import TransferPlane
from alluxio_amd.job import JobClient, LoadConfig
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d", rank=rank, world_size=world)
work = %(work)r
conf = Configuration({"alluxio.master.journal.folder": work + "/journal",
    "alluxio.worker.tieredstore.level0.dirs.path": "dram", "alluxio.worker.tieredstore.level0.dirs.quota": "128MB",
    "alluxio.worker.hbm.page.size": "1MB", "alluxio.user.block.size.bytes.default": "2MB",
    "alluxio.job.master.worker.heartbeat.interval": "20ms", "alluxio.worker.block.heartbeat.interval": "50ms"})
box = [None]
if rank == 0:
    m = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=work + "/ufs"); box[0] = m.start(start_heartbeats=False)
dist.broadcast_object_list(box, src=0)
w = AlluxioWorkerProcess(conf.copy(), master_address=box[0], port=0, work_dir=work + "/w%%d" %% rank)
w.start(start_heartbeats=True)
plane = TransferPlane.establish(w.worker)
fs = FileSystem(conf=conf.copy(), master_address=box[0])
cached = np.random.default_rng(1).integers(0, 256, 5 * (1 << 20) + 11, dtype=np.uint8)
ufs_only = np.random.default_rng(2).integers(0, 256, 3 * (1 << 20) + 5, dtype=np.uint8)
if rank == 0:
    fs.write_file("/dl/cached", cached, write_type="MUST_CACHE")      # blocks on worker 0 only
    fs.write_file("/dl/ufs", ufs_only, write_type="THROUGH")          # blocks in no worker
dist.barrier()
# every worker's job worker must be registered before the job is planned
deadline = time.time() + 60
jc = JobClient(fs.ctx.master_channel())
while len(jc.worker_health()) < world and time.time() < deadline:
    time.sleep(0.05)
if rank == 0:
    status, result, err = jc.run_and_wait(LoadConfig(path="/dl", replication=%(replication)d), timeout=120)
    open(work + "/job.json.tmp", "w").write(json.dumps([status, result, err]))
    os.replace(work + "/job.json.tmp", work + "/job.json")      # readers never see a partial file
while not os.path.exists(work + "/job.json"):
    time.sleep(0.05)
status, result, err = json.load(open(work + "/job.json"))
blocks = []
for p, arr in (("/dl/cached", cached), ("/dl/ufs", ufs_only)):
    blocks += [(b.blockInfo.blockId, b.blockInfo.length, arr[i * (2 << 20):i * (2 << 20) + b.blockInfo.length].tobytes())
               for i, b in enumerate(fs.get_status(p).info.fileBlockInfos)]
held = [b for b, _, _ in blocks if w.worker.has_block(b)]
ok_all = len(held) == len(blocks)
ok_bytes = all(w.worker.read_bytes(b, 0, n) == exp for b, n, exp in blocks if w.worker.has_block(b))
print(json.dumps({"rank": rank, "status": status, "err": err, "all": ok_all, "bytes": bool(ok_bytes),
                  "gathered": plane.bytes_gathered, "held": held, "nblocks": len(blocks)}), flush=True)
time.sleep(0.3)
fs.close(); w.stop()
dist.barrier()
if rank == 0:
    m.stop()
dist.destroy_process_group()
"""


def _run_collective_load(tmp_path, world, replication):
    script = COLLECTIVE_LOAD_SCRIPT % {"root": ROOT, "port": _free_port(), "work": str(tmp_path),
                                       "replication": replication}
    path = tmp_path / "cload.py"
    path.write_text(script)
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, str(path)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            pytest.fail("collective load rank timed out")
        assert p.returncode == 0, err[-3000:]
        outs.append(json.loads(out.strip().splitlines()[-1]))
    return outs


def test_distributed_load_replication_all_uses_collective(tmp_path):
    """``distributedLoad --replication`` >= worker count: owners load from the UFS, then every
    worker receives every block through the transfer plane's all-gather (C4 on the product path)."""
    outs = _run_collective_load(tmp_path, 2, -1)
    for o in outs:
        assert o["status"] == "COMPLETED", o
        assert o["all"] and o["bytes"], o
    # rank 0 already held the cached file, so it receives only rank 1's UFS-loaded blocks; rank 1
    # receives the cached file plus rank 0's share of the UFS file -- both through the all-gather
    assert all(o["gathered"] > 0 for o in outs), outs


REBUILD_SCRIPT = r"""
import os, sys, json
from datetime import timedelta
sys.path.insert(0, %(root)r)
import numpy as np, torch, torch.distributed as dist
from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.worker.process import AlluxioWorkerProcess
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.parallel.transfer import TransferPlane
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d", rank=rank, world_size=world,
                        timeout=timedelta(seconds=60))
work = %(work)r
conf = Configuration({"alluxio.master.journal.folder": work + "/journal",
    "alluxio.worker.tieredstore.level0.dirs.path": "dram", "alluxio.worker.tieredstore.level0.dirs.quota": "128MB",
    "alluxio.user.block.size.bytes.default": "1MB"})
box = [None]
if rank == 0:
    m = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=work + "/ufs"); box[0] = m.start(start_heartbeats=False)
dist.broadcast_object_list(box, src=0)
w = AlluxioWorkerProcess(conf.copy(), master_address=box[0], port=0, work_dir=work + "/w%%d" %% rank)
w.start(start_heartbeats=False)
# one block per round, so the death lands between rounds
plane = TransferPlane.establish(w.worker, rebuild_wait_s=3.0, timeout_s=30.0, batch_bytes=1 << 20)
fs = FileSystem(conf=conf.copy(), master_address=box[0])
data = np.random.default_rng(20 + rank).integers(0, 256, 3 * (1 << 20) + 11, dtype=np.uint8)
fs.write_file("/rb/f%%d" %% rank, data, write_type="MUST_CACHE")
mine = [(b.blockInfo.blockId, b.blockInfo.length, rank) for b in fs.get_status("/rb/f%%d" %% rank).info.fileBlockInfos]
allb = [None] * world
dist.all_gather_object(allb, mine)
blocks = [x for part in allb for x in part]
if rank == world - 1:
    # this rank dies after the first round of the collective
    orig = plane._scatter_batches
    def dying(*a, **kw):
        r = orig(*a, **kw)
        os._exit(0)
    plane._scatter_batches = dying
moved = plane.replicate_ring(blocks, 2) if %(method)r == "ring" else plane.replicate_all(blocks)
alive = [r for r in range(world - 1)]
if %(method)r == "ring":     # own + ring predecessor (in the rebuilt ring) blocks
    pred = plane.members[(plane.members.index(rank) - 1) %% len(plane.members)]
    have_alive = all(w.worker.has_block(b) for b, _, o in blocks if o in (rank, pred))
else:
    have_alive = all(w.worker.has_block(b) for b, _, o in blocks if o in alive)
first_dead = allb[world - 1][0][0]
print(json.dumps({"rank": rank, "moved": moved, "rebuilds": plane.rebuilds, "members": plane.members,
                  "have_alive": have_alive, "dead_round0": w.worker.has_block(first_dead),
                  "dead_later": any(w.worker.has_block(b) for b, _, _ in allb[world - 1][1:])}), flush=True)
plane._pg.barrier().wait()
fs.close(); w.stop()
plane._pg.barrier().wait()
if rank == 0:
    m.stop()
os._exit(0)
"""


@pytest.mark.parametrize("method", ["all", "ring"])
def test_replicate_all_rebuilds_group_after_rank_death(tmp_path, method):
    """A rank dies in the middle of replicate_all / replicate_ring: the survivors' round fails,
    they agree on a new group through the rendezvous store and finish replicating among
    themselves (the ring runs 4 ranks with 2 copies, so only the dead rank's neighbours see the
    point-to-point failure; the bounded waits plus the store's rebuild marker bring every
    survivor along)."""
    world = 4 if method == "ring" else 3
    script = REBUILD_SCRIPT % {"root": ROOT, "port": _free_port(), "work": str(tmp_path), "method": method}
    path = tmp_path / "rebuild.py"
    path.write_text(script)
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, str(path)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for rank, p in enumerate(procs):
        try:
            out, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("rebuild rank timed out")
        if rank < world - 1:
            assert p.returncode == 0, err[-3000:]
            outs.append(json.loads(out.strip().splitlines()[-1]))
    for o in outs:
        assert o["rebuilds"] == 1 and o["members"] == list(range(world - 1)), o
        assert o["have_alive"] and not o["dead_later"], o
        if method == "all":
            assert o["dead_round0"], o
        assert o["moved"] > 0, o


RING_SCRIPT = r"""
import os, sys, json
sys.path.insert(0, %(root)r)
import numpy as np, torch.distributed as dist
from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.worker.process import AlluxioWorkerProcess
from alluxio_amd.client.file_system import FileSystem
from alluxio_amd.parallel.transfer import TransferPlane
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d", rank=rank, world_size=world)
work = %(work)r
conf = Configuration({"alluxio.master.journal.folder": work + "/journal",
    "alluxio.worker.tieredstore.level0.dirs.path": "dram", "alluxio.worker.tieredstore.level0.dirs.quota": "128MB",
    "alluxio.worker.hbm.page.size": "1MB", "alluxio.user.block.size.bytes.default": "2MB"})
box = [None]
if rank == 0:
    m = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=work + "/ufs"); box[0] = m.start(start_heartbeats=False)
dist.broadcast_object_list(box, src=0)
w = AlluxioWorkerProcess(conf.copy(), master_address=box[0], port=0, work_dir=work + "/w%%d" %% rank)
w.start(start_heartbeats=False)
plane = TransferPlane.establish(w.worker, batch_bytes=%(batch)d)
fs = FileSystem(conf=conf.copy(), master_address=box[0])
size = (1 + rank) * (1 << 20) + 333 * rank + 5       # rank r owns ceil(size/2MB) blocks
data = np.random.default_rng(40 + rank).integers(0, 256, size, dtype=np.uint8)
fs.write_file("/ring/f%%d" %% rank, data, write_type="MUST_CACHE")
st = fs.get_status("/ring/f%%d" %% rank)
mine = [(b.blockInfo.blockId, b.blockInfo.length, rank) for b in st.info.fileBlockInfos]
allb = [None] * world
dist.all_gather_object(allb, mine)
blocks = [x for part in allb for x in part]
moved = plane.replicate_ring(blocks, 2)
prev = (rank - 1) %% world
pdata = np.random.default_rng(40 + prev).integers(0, 256, (1 + prev) * (1 << 20) + 333 * prev + 5, dtype=np.uint8)
ok_prev = all(w.worker.read_bytes(b, 0, n) == pdata[i * (2 << 20):i * (2 << 20) + n].tobytes()
              for i, (b, n, _) in enumerate(allb[prev]))
held = {r: all(w.worker.has_block(b) for b, _, _ in allb[r]) for r in range(world)}
print(json.dumps({"rank": rank, "moved": moved, "ok_prev": bool(ok_prev), "held": held,
                  "expect": sum(n for _, n, _ in allb[prev]), "rounds": plane.rounds}), flush=True)
dist.barrier()
fs.close(); w.stop()
dist.barrier()
if rank == 0:
    m.stop()
dist.destroy_process_group()
"""


@pytest.mark.parametrize("batch", [256 << 20, 2 << 20])
def test_replicate_ring_p2p_gloo(tmp_path, batch):
    """k-copy ring replication with point-to-point send/recv: with 2 copies each rank ends up
    holding exactly its own and its predecessor's blocks (4 ranks, uneven block counts).  With
    2 MiB batches the owners' blocks go one per round (several pipelined rounds); with 256 MiB
    batches every owner's blocks travel packed in one round."""
    world = 4
    script = RING_SCRIPT % {"root": ROOT, "port": _free_port(), "work": str(tmp_path), "batch": batch}
    path = tmp_path / "ring.py"
    path.write_text(script)
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, str(path)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            pytest.fail("ring rank timed out")
        assert p.returncode == 0, err[-3000:]
        outs.append(json.loads(out.strip().splitlines()[-1]))
    for o in outs:
        r = o["rank"]
        assert o["ok_prev"] and o["moved"] == o["expect"], o
        held = {int(k): v for k, v in o["held"].items()}
        assert held == {x: x in (r, (r - 1) % world) for x in range(world)}, o
        assert o["rounds"] == (1 if batch > (8 << 20) else 3), o      # rank 3 owns 3 blocks


def test_distributed_load_two_copies_uses_ring(tmp_path):
    """``distributedLoad --replication 2`` on 3 workers: blocks not yet on 2 workers are loaded by
    an owner and sent to its ring successor with point-to-point send/recv; every block ends up on
    exactly 2 workers with the right bytes."""
    outs = _run_collective_load(tmp_path, 3, 2)
    counts = {}
    for o in outs:
        assert o["status"] == "COMPLETED" and o["bytes"], o
        for b in o["held"]:
            counts[b] = counts.get(b, 0) + 1
    assert len(counts) == outs[0]["nblocks"] and set(counts.values()) == {2}, counts
    assert sum(o["gathered"] for o in outs) > 0
