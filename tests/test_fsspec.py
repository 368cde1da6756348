"""fsspec ``alluxio://`` filesystem (reference core/client/hdfs AbstractFileSystemTest /
HdfsFileInputStreamTest: open/read/seek/pread, list, mkdir, rename, delete, block locations)."""
import os

import fsspec
import pytest

from alluxio_amd.client.fsspec import AlluxioFileSystem
from alluxio_amd.minicluster import LocalAlluxioCluster


@pytest.fixture(scope="module")
def afs():
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                                                  "alluxio.user.block.size.bytes.default": "1MB"}) as c:
        yield c, AlluxioFileSystem(master=c.master.address, skip_instance_cache=True)


def test_url_roundtrip(afs):
    c, fs = afs
    data = os.urandom(2_500_000)
    url = f"alluxio://{c.master.address}/fss/a/data.bin"
    with fsspec.open(url, "wb") as f:
        f.write(data[:1_000_000])
        f.write(data[1_000_000:])
    with fsspec.open(url, "rb") as f:
        assert f.read() == data
    with fs.open("/fss/a/data.bin", "rb") as f:
        f.seek(123_456)
        assert f.read(1000) == data[123_456:124_456]
    assert fs.info("/fss/a/data.bin")["size"] == len(data)
    assert fs.ls("/fss/a", detail=False) == ["/fss/a/data.bin"]
    locs = fs.block_locations("/fss/a/data.bin")
    assert sum(l["length"] for l in locs) == len(data) and locs[0]["hosts"] == ["127.0.0.1"]
    fs.mv("/fss/a/data.bin", "/fss/b.bin")
    assert fs.exists("/fss/b.bin") and not fs.exists("/fss/a/data.bin")
    fs.cp_file("/fss/b.bin", "/fss/c.bin")
    assert fs.cat_file("/fss/c.bin") == data
    fs.makedirs("/fss/x/y", exist_ok=True)
    assert fs.isdir("/fss/x/y")
    fs.rm("/fss/x", recursive=True)
    assert not fs.exists("/fss/x")
    with pytest.raises(FileNotFoundError):
        fs.info("/nope")


def test_pandas_through_fsspec(afs):
    pd = pytest.importorskip("pandas")
    c, fs = afs
    df = pd.DataFrame({"a": range(100), "b": [f"s{i}" for i in range(100)]})
    url = f"alluxio://{c.master.address}/fss/df.csv"
    with fsspec.open(url, "w") as f:
        df.to_csv(f, index=False)
    with fsspec.open(url, "r") as f:
        back = pd.read_csv(f)
    assert back.equals(df)
