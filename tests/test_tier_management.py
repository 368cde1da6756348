"""Tier management (reference tests/.../worker/block/management/tier/*TaskTest: promote fills the
upper tier with the hottest lower-tier blocks up to the quota, align swaps hot-lower with
cold-upper, swap-restore frees reserved space; all gated on user-I/O idleness)."""
import os

from alluxio_amd.minicluster import LocalAlluxioCluster

MB = 1 << 20


def test_promote_align_restore(tmp_path):
    conf = {"alluxio.worker.tieredstore.levels": "2",
            "alluxio.worker.tieredstore.level0.alias": "MEM",
            "alluxio.worker.tieredstore.level0.dirs.path": "dram",
            "alluxio.worker.tieredstore.level0.dirs.quota": "4MB",
            "alluxio.worker.tieredstore.level1.alias": "SSD",
            "alluxio.worker.tieredstore.level1.dirs.path": str(tmp_path / "ssd"),
            "alluxio.worker.tieredstore.level1.dirs.quota": "64MB",
            "alluxio.worker.tieredstore.level1.dirs.mediumtype": "SSD",
            "alluxio.worker.hbm.page.size": "256KB",
            "alluxio.user.block.size.bytes.default": "1MB",
            "alluxio.worker.management.tier.align.reserved.bytes": "0",
            "alluxio.worker.management.load.detection.cool.down.time": "10min"}
    os.makedirs(tmp_path / "ssd", exist_ok=True)
    with LocalAlluxioCluster(num_workers=1, conf=conf) as c:
        fs = c.client()
        w = c.workers[0]
        data = {i: os.urandom(MB) for i in range(6)}
        for i, d in data.items():
            fs.write_file(f"/t/{i}", d, write_type="MUST_CACHE", write_tier=1)
        bid = {i: fs.get_status(f"/t/{i}").block_ids[0] for i in data}
        assert all(w.worker.native.block_info(b).tier == 1 for b in bid.values())
        for i in (3, 4, 5):
            fs.read_file(f"/t/{i}")
        tm = w.tier_manager
        assert tm.user_io_active()            # reads just happened: the coordinator backs off
        assert tm.run_once()["promoted"] == 0
        tm.cool_down_s = 0
        tm.align_enabled = False
        tm.run_once()
        up = {i for i, b in bid.items() if w.worker.native.block_info(b).tier == 0}
        assert up == {3, 4, 5}                 # hottest promoted, up to the 90% quota of 4MB
        # blocks 0,1 become the hottest: align swaps them with the coldest MEM blocks
        for _ in range(2):
            for i in (0, 1):
                fs.read_file(f"/t/{i}")
        tm.align_enabled, tm.promote_enabled = True, False
        tm.run_once()
        up = {i for i, b in bid.items() if w.worker.native.block_info(b).tier == 0}
        assert {0, 1} <= up and len(up) == 3
        # bytes intact after the moves
        for i, d in data.items():
            assert fs.read_file(f"/t/{i}") == d
        # swap-restore: demand 2MB reserved in MEM -> coldest MEM blocks move down
        tm.reserved = 2 * MB
        tm.align_enabled = False
        tm.swap_restore(0, 1)
        cap, avail = tm._tier_space(0)
        assert avail >= min(tm.reserved, cap // 10)
        fs.close()
