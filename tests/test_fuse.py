"""FUSE operation-layer tests (reference integration/fuse/src/test: AlluxioFuseFileSystemTest —
ops invoked with paths/handles exactly as a FUSE binding would)."""
import errno
import os
import stat

import pytest

from alluxio_amd.fuse import AlluxioFuseOps, FuseOSError
from alluxio_amd.minicluster import LocalAlluxioCluster


@pytest.fixture(scope="module")
def ops():
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                                                  "alluxio.user.block.size.bytes.default": "1MB"}) as c:
        fs = c.client()
        yield AlluxioFuseOps(fs, "/mnt")
        fs.close()


def test_create_write_read(ops):
    ops.fs.create_directory("/mnt", allow_exists=True)
    ops.mkdir("/d", 0o755)
    fd = ops.create("/d/f", 0o644)
    data = os.urandom(300_000)
    off = 0
    for i in range(0, len(data), 128 << 10):
        chunk = data[i:i + (128 << 10)]
        assert ops.write("/d/f", chunk, off, fd) == len(chunk)
        off += len(chunk)
    # duplicate write of an already-written range is ignored; random write rejected
    assert ops.write("/d/f", b"zz", 0, fd) == 2
    with pytest.raises(FuseOSError) as e:
        ops.write("/d/f", b"zz", off + 10, fd)
    assert e.value.errno == errno.EOPNOTSUPP
    assert ops.getattr("/d/f")["st_size"] == len(data)   # size visible while open
    ops.release("/d/f", fd)
    a = ops.getattr("/d/f")
    assert stat.S_ISREG(a["st_mode"]) and a["st_size"] == len(data) and a["st_mode"] & 0o777 == 0o644
    fd = ops.open("/d/f", os.O_RDONLY)
    assert ops.read("/d/f", 1000, 5000, fd) == data[5000:6000]
    assert ops.read("/d/f", 1 << 20, len(data) - 10, fd) == data[-10:]
    ops.release("/d/f", fd)
    assert ops.readdir("/d") == [".", "..", "f"]
    assert stat.S_ISDIR(ops.getattr("/d")["st_mode"])


def test_namespace_ops(ops):
    ops.fs.create_directory("/mnt", allow_exists=True)
    ops.mkdir("/n", 0o700)
    fd = ops.create("/n/a", 0o600)
    ops.write("/n/a", b"abc", 0, fd)
    ops.release("/n/a", fd)
    ops.rename("/n/a", "/n/b")
    with pytest.raises(FuseOSError) as e:
        ops.getattr("/n/a")
    assert e.value.errno == errno.ENOENT
    ops.chmod("/n/b", 0o640)
    assert ops.getattr("/n/b")["st_mode"] & 0o777 == 0o640
    with pytest.raises(FuseOSError) as e:
        ops.rmdir("/n")
    assert e.value.errno == errno.ENOTEMPTY
    # write-once: opening an existing non-empty file for write without O_TRUNC is refused
    with pytest.raises(FuseOSError) as e:
        ops.open("/n/b", os.O_WRONLY)
    assert e.value.errno == errno.EACCES
    fd = ops.open("/n/b", os.O_WRONLY | os.O_TRUNC)
    ops.write("/n/b", b"new", 0, fd)
    ops.release("/n/b", fd)
    fd = ops.open("/n/b", os.O_RDONLY)
    assert ops.read("/n/b", 10, 0, fd) == b"new"
    ops.release("/n/b", fd)
    with pytest.raises(FuseOSError) as e:
        ops.truncate("/n/b", 1)
    assert e.value.errno == errno.EOPNOTSUPP
    ops.truncate("/n/b", 0)
    assert ops.getattr("/n/b")["st_size"] == 0
    ops.unlink("/n/b")
    ops.rmdir("/n")
    with pytest.raises(FuseOSError):
        ops.getattr("/n")
    sf = ops.statfs("/")
    assert sf["f_blocks"] > 0 and sf["f_bavail"] <= sf["f_blocks"]
    assert ops.open_files() == 0
    with pytest.raises(FuseOSError) as e:
        ops.read("/x", 1, 0, 999)
    assert e.value.errno == errno.EBADF
