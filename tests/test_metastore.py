"""ROCKS-style metastore (reference core/server/master/src/test/.../metastore/InodeStoreTest and
the "caching inode store" tests): the namespace behaves identically with a disk-backed inode store
whose object cache is far smaller than the namespace, including across a master restart."""
import os

import pytest

from alluxio_amd.minicluster import LocalAlluxioCluster


def _exercise(c):
    fs = c.client()
    for d in range(6):
        fs.create_directory(f"/ms/d{d}/sub", recursive=True)
        for f in range(5):
            fs.write_file(f"/ms/d{d}/f{f}", bytes([d, f]) * 100, write_type="CACHE_THROUGH")
    fs.rename("/ms/d0", "/ms/r0")
    fs.delete("/ms/d1", recursive=True)
    fs.set_attribute("/ms/d2/f3", pinned=True, mode=0o600)
    fs.set_attribute("/ms/d3", ttl=3_600_000, ttl_action="FREE")
    fs.write_file("/ms/async", b"later", write_type="ASYNC_THROUGH")
    snapshot = {}
    for s in fs.list_status("/ms", recursive=True):
        i = s.info
        snapshot[i.path] = (i.folder, i.length, i.mode, i.pinned, i.ttl, i.persistenceState, list(i.blockIds))
    got = {p: fs.read_file(p) for p, v in snapshot.items() if not v[0]}
    fs.close()
    return snapshot, got


@pytest.mark.parametrize("store", ["HEAP", "ROCKS"])
def test_namespace_identical(store, tmp_path):
    conf = {"alluxio.worker.tieredstore.level0.dirs.path": "dram", "alluxio.master.metastore": store,
            "alluxio.master.metastore.dir": str(tmp_path / "ms"),
            "alluxio.master.metastore.inode.cache.max.size": "16"}
    with LocalAlluxioCluster(num_workers=1, conf=conf, work_dir=str(tmp_path / "c")) as c:
        snap, data = _exercise(c)
        assert snap["/ms/r0/sub"][0] and "/ms/d1/f0" not in snap
        assert snap["/ms/d2/f3"][2] == 0o600 and snap["/ms/d2/f3"][3]
        assert snap["/ms/async"][5] == "TO_BE_PERSISTED"
        assert data["/ms/d4/f2"] == bytes([4, 2]) * 100
        tree = c.master.fs_master.tree
        if store == "ROCKS":
            assert tree.inodes.kind == "ROCKS" and tree.inodes.loads > 0   # cache (16) << namespace
            assert os.path.exists(tmp_path / "ms" / "inodes.sqlite")
        c.restart_master()
        fs = c.client()
        again = {s.info.path: (s.info.folder, s.info.length, s.info.mode, s.info.pinned, s.info.ttl,
                               s.info.persistenceState, list(s.info.blockIds))
                 for s in fs.list_status("/ms", recursive=True)}
        assert again == snap
        fs.close()
