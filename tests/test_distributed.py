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
                     "--buffer-size", "1m", "--page-size", "1m", "--dest", "host", "--work-dir", str(tmp_path)])
    assert rc == 0
    line = capsys.readouterr().out.strip().splitlines()[-1]
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["config"]["verified"] and out["value"] > 0
