"""The native block commit of the worker's data server (csrc/data_server.cpp BlockCommitter).

Reference behaviour pinned here: BlockWriteHandler.java:124-149 answers a WriteBlock only after
DefaultBlockWorker.commitBlock (:274-306) committed the block locally -- read-locked -- and told the
master (BlockMasterClient.commitBlock, retried by the client's retry policy); a block whose
master commit fails does not stay committed here (the stream fails instead).
"""
import threading
import time

import numpy as np
import pytest

from alluxio_amd.ops.native import lib

from test_data_server import _blocks, _cluster, _remote_fs

pytestmark = pytest.mark.skipif(not lib().FrameRpcServer.grpc_available(), reason="libnghttp2 not present")

MB = 1 << 20


def _count_python_commits(monkeypatch, worker):
    """Counts per-block Python commits (NativeWriteCommit -> BlockWorker.commit_block), the path the
    native committer replaces."""
    calls = []
    bw = worker.worker
    orig = bw.commit_block

    def counting(session_id, block_id, pin=False, hold=False):
        calls.append(block_id)
        return orig(session_id, block_id, pin, hold)
    monkeypatch.setattr(bw, "commit_block", counting)
    return calls


def test_parallel_writes_commit_natively_in_batches(tmp_path, monkeypatch):
    with _cluster(tmp_path, {"alluxio.worker.data.crc.enabled": "true"}) as c:
        fs = c.client()
        rfs = _remote_fs(c)
        w = c.workers[0]
        st = w.data_server.stats
        py_commits = _count_python_commits(monkeypatch, w)
        rng = np.random.default_rng(1)
        files = {f"/nc/f{i}": rng.integers(0, 256, 9 * MB + 37 * i, dtype=np.uint8) for i in range(8)}
        c0, b0 = st.commits, st.commit_batches
        errs = []

        def write(p, d):
            try:
                rfs.write_file(p, d, write_type="MUST_CACHE")
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        ts = [threading.Thread(target=write, args=kv) for kv in files.items()]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs, errs
        nblocks = sum(len(_blocks(rfs, p)) for p in files)
        assert st.commits - c0 == nblocks
        assert 1 <= st.commit_batches - b0 <= nblocks
        assert not py_commits                        # no per-block Python commit
        for p, d in files.items():
            assert rfs.get_status(p).in_alluxio_percentage == 100
            assert rfs.read_file(p) == d.tobytes()
            for bid, _ in _blocks(rfs, p):
                # CRCs of the committed bytes (host tier: computed by the committer) reach the worker
                piece, crcs = w.worker.crc[bid]
                assert crcs == list(w.worker.native.checksum(bid, 0)) and piece > 0
        rfs.close()
        fs.close()


def test_master_outage_during_commit_retries_then_removes_the_block(tmp_path, monkeypatch):
    """CommitBlocks failing: the report is retried for alluxio.user.rpc.retry.max.duration, then
    the block is removed again and the WriteBlock fails UNAVAILABLE; once the master answers again
    the same write succeeds."""
    with _cluster(tmp_path, {"alluxio.user.rpc.retry.max.duration": "600ms",
                             "alluxio.user.rpc.retry.base.sleep": "20ms",
                             "alluxio.user.rpc.retry.max.sleep": "100ms"}) as c:
        fs = c.client()
        rfs = _remote_fs(c, **{"alluxio.user.block.write.retry.max": "0"})
        w = c.workers[0]
        st = w.data_server.stats
        bw = w.worker
        real = bw._bm()
        attempts = []

        class Down:
            def __getattr__(self, name):
                return getattr(real, name)

            def CommitBlocks(self, req):
                attempts.append(time.monotonic())
                from alluxio_amd.utils.exceptions import UnavailableException
                raise UnavailableException("master is down")
        monkeypatch.setattr(bw, "_block_master", Down())
        data = np.random.default_rng(2).integers(0, 256, 5 * MB, dtype=np.uint8)
        f0 = st.commit_failures
        t0 = time.monotonic()
        with pytest.raises(Exception) as ei:
            rfs.write_file("/mo/a", data, write_type="MUST_CACHE")
        assert time.monotonic() - t0 < 10
        assert "UNAVAILABLE" in str(ei.value).upper() or "master was not told" in str(ei.value), ei.value
        assert len(attempts) >= 2                    # retried before giving up
        assert st.commit_failures > f0
        for b in bw.native.block_ids(-1):            # nothing committed here stayed
            assert b not in [x for x, _ in _blocks(fs, "/mo/a")] if fs.exists("/mo/a") else True
        assert not any(bw.native.has_temp_block(b) for b in bw.native.block_ids(-1))
        monkeypatch.setattr(bw, "_block_master", real)
        rfs.write_file("/mo/b", data, write_type="MUST_CACHE")
        assert rfs.read_file("/mo/b") == data.tobytes()
        assert rfs.get_status("/mo/b").in_alluxio_percentage == 100
        rfs.close()
        fs.close()


def test_cold_read_through_commits_natively(tmp_path, monkeypatch):
    """A cold block read through by the data server is committed by the native committer (no
    Python NativeWriteCommit), reported to the master, and readable as cached afterwards."""
    with _cluster(tmp_path) as c:
        fs = c.client()
        rfs = _remote_fs(c)
        w = c.workers[0]
        st = w.data_server.stats
        rng = np.random.default_rng(4)
        a = rng.integers(0, 256, 6 * MB + 1, dtype=np.uint8)
        b = rng.integers(0, 256, 9 * MB + 3, dtype=np.uint8)
        fs.write_file("/cold/a", a, write_type="THROUGH")
        fs.write_file("/cold/b", b, write_type="THROUGH")
        assert rfs.read_file("/cold/a") == a.tobytes()        # Python registers the mount
        deadline = time.time() + 10
        while rfs.get_status("/cold/a").in_alluxio_percentage != 100:   # its Python commit is done
            assert time.time() < deadline
            time.sleep(0.05)
        py_commits = _count_python_commits(monkeypatch, w)
        c0 = st.commits
        assert rfs.read_file("/cold/b") == b.tobytes()
        blocks = _blocks(rfs, "/cold/b")
        deadline = time.time() + 10
        while st.commits - c0 < len(blocks):
            assert time.time() < deadline
            time.sleep(0.02)
        assert not py_commits
        deadline = time.time() + 10
        while rfs.get_status("/cold/b").in_alluxio_percentage != 100:
            assert time.time() < deadline
            time.sleep(0.05)
        assert rfs.read_file("/cold/b") == b.tobytes()
        rfs.close()
        fs.close()


def test_python_commit_path_still_serves_when_disabled(tmp_path, monkeypatch):
    with _cluster(tmp_path, {"alluxio.worker.data.server.native.commit.enabled": "false"}) as c:
        fs = c.client()
        rfs = _remote_fs(c)
        w = c.workers[0]
        py_commits = _count_python_commits(monkeypatch, w)
        data = np.random.default_rng(3).integers(0, 256, 5 * MB, dtype=np.uint8)
        rfs.write_file("/pc/a", data, write_type="MUST_CACHE")
        assert len(py_commits) == len(_blocks(rfs, "/pc/a")) and w.data_server.stats.commits == 0
        assert rfs.read_file("/pc/a") == data.tobytes()
        rfs.close()
        fs.close()


@pytest.mark.gpu
def test_streamed_crc_of_hbm_blocks_equals_checksum(tmp_path):
    """HBM blocks written over the data port get their per-page CRC32C from the kernel enqueued on
    the write stream behind the last H2D; it equals the store's checksum() of the committed bytes."""
    with _cluster(tmp_path, {"alluxio.worker.tieredstore.level0.dirs.path": "hbm:0",
                             "alluxio.worker.tieredstore.level0.dirs.quota": "256MB",
                             "alluxio.worker.hbm.page.size": "1MB"}) as c:
        fs = c.client()
        rfs = _remote_fs(c)
        w = c.workers[0]
        st = w.data_server.stats
        # holes in the arena first: the blocks below get scattered pages, which the CRC kernel
        # reads through the block's page index array in one launch
        for i in range(16):
            rfs.write_file(f"/crc/f{i}", np.full(MB, i, dtype=np.uint8), write_type="MUST_CACHE")
        for i in range(0, 16, 2):
            rfs.delete(f"/crc/f{i}")
        c.heartbeat_workers()
        s0 = st.crc_streamed
        data = np.random.default_rng(5).integers(0, 256, 10 * MB + 12345, dtype=np.uint8)
        rfs.write_file("/crc/a", data, write_type="MUST_CACHE")
        blocks = _blocks(rfs, "/crc/a")
        assert st.crc_streamed - s0 == len(blocks)
        scattered = 0
        for bid, _ in blocks:
            pages = list(w.worker.native.block_pages(bid)[0])
            scattered += any(b != a + 1 for a, b in zip(pages, pages[1:]))
        for bid, n in blocks:
            piece, crcs = w.worker.crc[bid]
            assert piece == 1 * MB
            assert crcs == list(w.worker.native.checksum(bid, 0))
            assert len(crcs) == -(-n // MB)
        assert rfs.read_file("/crc/a") == data.tobytes()
        print(f"blocks with scattered pages: {scattered} of {len(blocks)}")
        rfs.close()
        fs.close()


def test_tee_block_is_held_from_eviction_until_appended(tmp_path):
    """CACHE_THROUGH tee: the committed block stays locked for the file's UFS stream (an append
    hold) until its AppendBlock copy has its own lock, so eviction between the commit and the append
    cannot take it; the hold goes once the append ran (block evicted before its append)."""
    with _cluster(tmp_path) as c:
        rfs = _remote_fs(c)
        w = c.workers[0]
        native = w.worker.native
        rng = np.random.default_rng(6)
        rfs.write_file("/tee0", rng.integers(0, 256, MB, dtype=np.uint8), write_type="CACHE_THROUGH")
        data = rng.integers(0, 256, 9 * MB + 777, dtype=np.uint8)
        g = rfs.create_file("/tee1", write_type="CACHE_THROUGH", block_size=4 * MB)
        orig = g._ufs.append_block
        seen = []

        def evict_then_append(block_id, length):
            held = native.holds
            try:                                        # evict everything evictable
                native.free_space(12345, 512 * MB, -1, -1)
            except Exception:  # noqa: BLE001 - OutOfSpace: not all of it could go
                pass
            seen.append((block_id, held, native.has_block(block_id), block_id in native.eviction_order(-1, 0)))
            orig(block_id, length)
        g._ufs.append_block = evict_then_append
        for i in range(0, len(data), MB):
            g.write(data[i:i + MB])
        g.close()
        assert len(seen) == 3
        for bid, held, present, evictable in seen:
            assert held >= 1 and present and not evictable, (bid, held, present, evictable)
        st = rfs.get_status("/tee1")
        with open(st.info.ufsPath.replace("file://", ""), "rb") as fh:
            assert fh.read() == data.tobytes()
        deadline = time.time() + 10
        while native.holds:
            assert time.time() < deadline
            time.sleep(0.02)
        rfs.close()


def test_writes_into_a_full_tier_evict_off_the_io_thread(tmp_path):
    """A WriteBlock whose block needs eviction is created on a pool thread while the stream queues
    what arrives (receive window held back past 8 MiB): no call goes to the Python servicer, the
    older blocks are evicted, and the new file is cached byte-exact."""
    with _cluster(tmp_path, {"alluxio.worker.tieredstore.level0.dirs.quota": "24MB",
                             "alluxio.worker.tieredstore.free.ahead.bytes": "0"}) as c:
        fs = c.client()
        rfs = _remote_fs(c)
        st = c.workers[0].data_server.stats
        rng = np.random.default_rng(9)
        files = [rng.integers(0, 256, 7 * MB + i, dtype=np.uint8) for i in range(6)]   # 42 MB > 24 MB
        d0, e0 = st.write_declined, st.write_evict_waits
        for i, d in enumerate(files):
            rfs.write_file(f"/full/f{i}", d, write_type="MUST_CACHE")
        assert st.write_declined == d0
        assert st.write_evict_waits > e0
        last = rfs.get_status("/full/f5")
        assert last.in_alluxio_percentage == 100
        assert rfs.read_file("/full/f5") == files[5].tobytes()
        rfs.close()
        fs.close()


def test_cache_promote_read_moves_the_block_natively(tmp_path):
    """ReadBlock with promote of a block in a lower tier (CACHE_PROMOTE): the data server moves it
    to the top tier on a pool thread and streams it from there, without the Python servicer
    (BlockReadHandler.openBlock:159-175)."""
    import os
    for n in ("ssd0",):
        os.makedirs(tmp_path / n, exist_ok=True)
    conf = {"alluxio.worker.tieredstore.levels": "2",
            "alluxio.worker.tieredstore.level0.alias": "MEM",
            "alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": "64MB",
            "alluxio.worker.tieredstore.level1.alias": "SSD",
            "alluxio.worker.tieredstore.level1.dirs.path": str(tmp_path / "ssd0"),
            "alluxio.worker.tieredstore.level1.dirs.quota": "64MB",
            "alluxio.worker.tieredstore.level1.dirs.mediumtype": "SSD",
            "alluxio.worker.management.tier.promote.enabled": "false",
            "alluxio.worker.management.tier.align.enabled": "false"}
    with _cluster(tmp_path, conf) as c:
        fs = c.client()
        w = c.workers[0]
        st = w.data_server.stats
        data = np.random.default_rng(11).integers(0, 256, 6 * MB + 3, dtype=np.uint8)
        wfs = _remote_fs(c)
        with wfs.create_file("/pr/a", write_type="MUST_CACHE", write_tier=1) as f:
            f.write(data)
        blocks = _blocks(wfs, "/pr/a")
        assert all(w.worker.native.block_info(b).tier == 1 for b, _ in blocks)
        rfs = _remote_fs(c, **{"alluxio.user.file.readtype.default": "CACHE_PROMOTE"})
        d0, p0 = st.declined, st.promoted
        assert rfs.read_file("/pr/a") == data.tobytes()
        assert st.declined == d0
        assert st.promoted - p0 == len(blocks)
        assert all(w.worker.native.block_info(b).tier == 0 for b, _ in blocks)
        assert rfs.read_file("/pr/a") == data.tobytes()
        wfs.close()
        rfs.close()
        fs.close()
