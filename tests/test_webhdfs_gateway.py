"""WebHDFS gateway on the proxy (proxy/webhdfs.py): Hadoop clients reach the namespace over
``webhdfs://`` (reference: core/client/hdfs AbstractFileSystem.java -- the Hadoop-facing surface).
The UFS contract suite runs through this package's own WebHDFS client against the gateway, and the
wire shapes (FileStatus JSON, RemoteException, two-step CREATE, OPEN ranges) are checked directly."""
import io
import os
import sys

import numpy as np
import pytest
import requests

sys.path.insert(0, os.path.dirname(__file__))

from alluxio_amd.minicluster import LocalAlluxioCluster  # noqa: E402
from alluxio_amd.proxy import ProxyServer  # noqa: E402


@pytest.fixture
def gateway(tmp_path):
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                                                  "alluxio.user.block.size.bytes.default": "1MB",
                                                  "alluxio.security.authorization.permission.enabled": "false"},
                             work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        srv = ProxyServer(fs, "127.0.0.1", 0)
        port = srv.start()
        try:
            yield fs, f"http://127.0.0.1:{port}/webhdfs/v1", port
        finally:
            srv.stop()
            fs.close()


def test_webhdfs_wire_shapes(gateway):
    fs, base, _ = gateway
    data = np.random.default_rng(1).integers(0, 256, 3 * (1 << 20) + 77, dtype=np.uint8).tobytes()
    # two-step create: the "namenode" answers 307 to the "datanode" URL
    r = requests.put(base + "/d/x.bin", params={"op": "CREATE", "user.name": "u"}, allow_redirects=False)
    assert r.status_code == 307 and "datanode=true" in r.headers["Location"]
    r2 = requests.put(r.headers["Location"], data=data)
    assert r2.status_code == 201 and r2.headers["Location"].startswith("webhdfs://")
    assert fs.read_file("/d/x.bin") == data
    # without overwrite an existing file is refused
    r = requests.put(base + "/d/x.bin", params={"op": "CREATE"}, allow_redirects=False)
    assert r.status_code == 403 and r.json()["RemoteException"]["exception"] == "FileAlreadyExistsException"
    st = requests.get(base + "/d/x.bin", params={"op": "GETFILESTATUS"}).json()["FileStatus"]
    assert st["type"] == "FILE" and st["length"] == len(data) and st["pathSuffix"] == "" and st["blockSize"] == 1 << 20
    assert set(st) >= {"accessTime", "blockSize", "group", "length", "modificationTime", "owner", "pathSuffix",
                       "permission", "replication", "type"}
    ls = requests.get(base + "/d", params={"op": "LISTSTATUS"}).json()["FileStatuses"]["FileStatus"]
    assert [e["pathSuffix"] for e in ls] == ["x.bin"]
    # ranged OPEN through the redirect (requests follows 307)
    r = requests.get(base + "/d/x.bin", params={"op": "OPEN", "offset": 1000, "length": 5000})
    assert r.status_code == 200 and r.content == data[1000:6000]
    r = requests.get(base + "/d/x.bin", params={"op": "OPEN", "noredirect": "true"})
    assert "Location" in r.json()
    assert requests.get(base + "/d/x.bin", params={"op": "OPEN", "offset": len(data) - 10}).content == data[-10:]
    # missing paths: RemoteException + 404
    r = requests.get(base + "/nope", params={"op": "GETFILESTATUS"})
    assert r.status_code == 404
    assert r.json()["RemoteException"]["javaClassName"] == "java.io.FileNotFoundException"
    # write-once: append refused like AbstractFileSystem.append
    r = requests.post(base + "/d/x.bin", params={"op": "APPEND"})
    assert r.status_code == 403 and r.json()["RemoteException"]["exception"] == "UnsupportedOperationException"
    # checksum: COMPOSITE-CRC32C of the bytes
    from alluxio_amd.ops.native import lib
    ck = requests.get(base + "/d/x.bin", params={"op": "GETFILECHECKSUM"}).json()["FileChecksum"]
    assert ck == {"algorithm": "COMPOSITE-CRC32C", "bytes": format(lib().crc32c(data), "08x"), "length": 4}
    # namespace ops
    assert requests.put(base + "/d/sub/deep", params={"op": "MKDIRS", "permission": "750"}).json() == {"boolean": True}
    assert requests.get(base + "/d/sub/deep", params={"op": "GETFILESTATUS"}).json()["FileStatus"]["permission"] == "750"
    cs = requests.get(base + "/d", params={"op": "GETCONTENTSUMMARY"}).json()["ContentSummary"]
    assert cs["fileCount"] == 1 and cs["directoryCount"] == 3 and cs["length"] == len(data)
    assert requests.put(base + "/d/x.bin", params={"op": "RENAME", "destination": "/d/sub/y.bin"}).json() == {"boolean": True}
    assert requests.put(base + "/d/gone", params={"op": "RENAME", "destination": "/d/z"}).json() == {"boolean": False}
    r = requests.delete(base + "/d", params={"op": "DELETE", "recursive": "false"})
    assert r.status_code == 403 and "PathIsNotEmptyDirectory" in r.json()["RemoteException"]["exception"]
    assert requests.put(base + "/d/sub/y.bin", params={"op": "SETPERMISSION", "permission": "600"}).status_code == 200
    assert fs.get_status("/d/sub/y.bin").info.mode & 0o777 == 0o600
    assert requests.delete(base + "/d", params={"op": "DELETE", "recursive": "true"}).json() == {"boolean": True}
    assert not fs.exists("/d")
    assert requests.get(base + "/", params={"op": "GETHOMEDIRECTORY", "user.name": "bob"}).json() == {"Path": "/user/bob"}
    batch = requests.get(base + "/", params={"op": "LISTSTATUS_BATCH"}).json()["DirectoryListing"]
    assert batch["remainingEntries"] == 0
    r = requests.get(base + "/", params={"op": "NOSUCHOP"})
    assert r.status_code == 400 and r.json()["RemoteException"]["exception"] == "IllegalArgumentException"


def test_ufs_contract_through_the_gateway(gateway):
    """This package's WebHDFS under file system, pointed at the gateway, passes the UFS contract:
    an Alluxio namespace can serve as a Hadoop-compatible store for another cluster."""
    from alluxio_amd.cli import ufs_contract
    _, _, port = gateway
    out = io.StringIO()
    res = ufs_contract.run(f"webhdfs://127.0.0.1:{port}/contract", out=out, large_file_size=1 << 20,
                           properties={"alluxio.underfs.webhdfs.user": "u"})
    assert res["failed"] == [], out.getvalue()[-3000:]
    assert len(res["passed"]) >= 40


def test_redirect_ignores_spoofed_host_header(gateway):
    """The 307 of OPEN/CREATE names the proxy itself, not whatever Host the request carried (an
    open redirect would send a client -- and its CREATE body -- to an arbitrary server)."""
    fs, base, port = gateway
    fs.write_file("/r.bin", b"abc")
    for method, op in (("put", "CREATE"), ("get", "OPEN")):
        r = getattr(requests, method)(base + "/r.bin", params={"op": op, "overwrite": "true"},
                                      headers={"Host": "evil.example:666"}, allow_redirects=False)
        assert r.status_code == 307, r.text
        loc = r.headers["Location"]
        assert "evil.example" not in loc and f":{port}/" in loc, loc
