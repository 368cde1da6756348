"""Peer-to-peer block pulls under failure (SURVEY §5.3 for the GPU data plane; reference behaviour:
AsyncCacheRequestManager falls back to the UFS / another source when a remote read fails,
RemoteBlockReader surfaces the error and the client retries elsewhere).

A worker in a separate OS process holds the blocks; this process runs its own BlockWorker and
pulls from it: the mapped (shared-arena) pull works, a failing mapped pull falls back to the gRPC
block stream and puts the peer on cooldown, and a SIGKILLed peer makes a pull fail fast with no
temp block left behind."""
import os
import time

import numpy as np
import pytest

from alluxio_amd.conf import Configuration
from alluxio_amd.minicluster.multi_process import MultiProcessCluster
from alluxio_amd.parallel import peer
from alluxio_amd.proto import pb

MB = 1 << 20


@pytest.fixture
def env(tmp_path):
    c = MultiProcessCluster(num_masters=1, num_workers=1, journal_type="UFS", work_dir=str(tmp_path / "mpc"),
                            conf={"alluxio.user.block.size.bytes.default": "2MB"}).start()
    try:
        c.wait_for_workers(1)
        fs = c.client()
        datas = {}
        for i in range(4):
            datas[i] = np.random.default_rng(i).integers(0, 256, 2 * MB, dtype=np.uint8)
            fs.write_file(f"/pf/{i}", datas[i], write_type="MUST_CACHE")
        infos = {i: fs.get_status(f"/pf/{i}").info for i in datas}
        loc = infos[0].fileBlockInfos[0].blockInfo.locations[0].workerAddress
        addr = f"{loc.host}:{loc.rpcPort}"
        from alluxio_amd.worker.block_worker import BlockWorker
        from alluxio_amd.worker.store import TieredStore
        conf = Configuration({"alluxio.worker.tieredstore.levels": "1",
                              "alluxio.worker.tieredstore.level0.alias": "MEM",
                              "alluxio.worker.tieredstore.level0.dirs.path": "dram",
                              "alluxio.worker.tieredstore.level0.dirs.quota": "64MB",
                              "alluxio.worker.hbm.page.size": "1MB",
                              "alluxio.worker.peer.rpc.timeout": "2sec",
                              "alluxio.worker.peer.failure.cooldown": "30sec"})
        w = BlockWorker(conf, TieredStore(conf))
        peer.clear_failures()
        yield c, fs, w, addr, datas, infos
        fs.close()
        w.close()
    finally:
        c.stop()


def _bid(infos, i):
    return infos[i].fileBlockInfos[0].blockInfo.blockId


def _read(w, bid):
    return np.frombuffer(w.read_bytes(bid, 0, w.block_info(bid).length), dtype=np.uint8)


def test_mapped_pull_then_fallback_and_cooldown(env, monkeypatch):
    c, fs, w, addr, datas, infos = env
    # 1) healthy peer: the block comes through the shared DRAM arena (no payload on the RPC)
    # (worker metrics are process-wide: compare deltas)
    shared0 = w.metrics.counter("PeerSharedBytesReceived").count
    fail0 = w.metrics.counter("PeerPullFailures").count
    n = peer.pull_block(w, _bid(infos, 0), addr, 2 * MB)
    assert n == 2 * MB and np.array_equal(_read(w, _bid(infos, 0)), datas[0])
    assert w.metrics.counter("PeerSharedBytesReceived").count - shared0 == 2 * MB
    # 2) the mapped path breaks: the pull falls back to the gRPC block stream, marks the peer
    import alluxio_amd.parallel.ipc as ipc
    calls = []

    def broken(h, device):
        calls.append(h.block_id)
        raise RuntimeError("mapping failed")
    monkeypatch.setattr(ipc, "map_handle", broken)
    assert peer.pull_block(w, _bid(infos, 1), addr, 2 * MB) == 2 * MB
    assert np.array_equal(_read(w, _bid(infos, 1)), datas[1])
    assert calls == [_bid(infos, 1)] and peer.peer_failed(w, addr)
    assert w.metrics.counter("PeerPullFailures").count - fail0 == 1
    assert not w.native.has_temp_block(_bid(infos, 1))
    # 3) during the cooldown the mapped path is not tried again
    assert peer.pull_block(w, _bid(infos, 2), addr, 2 * MB) == 2 * MB
    assert calls == [_bid(infos, 1)]
    assert np.array_equal(_read(w, _bid(infos, 2)), datas[2])


def test_killed_peer_fails_fast_without_leftovers(env):
    c, fs, w, addr, datas, infos = env
    c.stop_worker(0)                     # SIGKILL the peer process
    t = time.time()
    with pytest.raises(Exception):
        peer.pull_block(w, _bid(infos, 3), addr, 2 * MB)
    assert time.time() - t < 30          # bounded by the peer RPC deadline, no hang
    assert not w.native.has_block(_bid(infos, 3)) and not w.native.has_temp_block(_bid(infos, 3))
    assert peer.peer_failed(w, addr)
