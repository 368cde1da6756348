"""Kernel FUSE mount of the namespace through this package's /dev/fuse protocol server
(fuse/kernel.py; reference integration/fuse AlluxioFuse + AlluxioFuseFileSystem and its
AlluxioFuseFileSystemTest / FuseIntegrationTest).  POSIX calls run in a child process with a
timeout, so a protocol bug fails the test instead of hanging it.  Skipped where mount(2) of a FUSE
filesystem is not permitted."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from alluxio_amd.fuse import AlluxioFuseOps
from alluxio_amd.minicluster import LocalAlluxioCluster

MB = 1 << 20


@pytest.fixture
def mounted(tmp_path):
    if not os.path.exists("/dev/fuse"):
        pytest.skip("/dev/fuse not present")
    from alluxio_amd.fuse.kernel import mount_kernel
    mnt = tmp_path / "mnt"
    mnt.mkdir()
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                                                  "alluxio.user.block.size.bytes.default": "4MB"},
                             work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        try:
            srv = mount_kernel(AlluxioFuseOps(fs), str(mnt))
        except OSError as e:
            pytest.skip(f"FUSE mount not permitted here: {e}")
        try:
            yield fs, str(mnt), srv
        finally:
            srv.unmount()
            fs.close()


def _posix(script: str, timeout: float = 60.0) -> dict:
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_posix_read_write_namespace(mounted):
    fs, mnt, srv = mounted
    data = np.random.default_rng(3).integers(0, 256, 9 * MB + 5, dtype=np.uint8)
    fs.write_file("/data/big.bin", data, write_type="MUST_CACHE")
    for i in range(300):                                  # several READDIR pages
        fs.write_file(f"/many/f{i:03d}", b"", write_type="MUST_CACHE")
    out = _posix(f"""
import hashlib, json, os
m = {mnt!r}
r = {{}}
r["root"] = sorted(os.listdir(m))
r["many"] = len(os.listdir(m + "/many"))
with open(m + "/data/big.bin", "rb") as f:
    b = f.read()
r["big_len"], r["big_md5"] = len(b), hashlib.md5(b).hexdigest()
with open(m + "/data/big.bin", "rb") as f:
    f.seek(4 * 1024 * 1024 - 3)
    r["mid"] = f.read(6).hex()
payload = bytes(range(256)) * 4099
with open(m + "/out/w.bin", "wb") if os.path.isdir(m + "/out") else open(m + "/w.bin", "wb") as f:
    for i in range(0, len(payload), 70000):
        f.write(payload[i:i + 70000])
r["w_size"] = os.stat(m + "/w.bin").st_size
r["w_ok"] = open(m + "/w.bin", "rb").read() == payload
os.makedirs(m + "/x/y")
os.rename(m + "/w.bin", m + "/x/y/w2.bin")
r["moved"] = os.listdir(m + "/x/y")
r["isdir"] = os.path.isdir(m + "/x") and not os.path.exists(m + "/w.bin")
try:
    open(m + "/nope/zz", "rb")
except FileNotFoundError:
    r["enoent"] = True
os.remove(m + "/x/y/w2.bin"); os.rmdir(m + "/x/y")
r["after_rm"] = os.listdir(m + "/x")
st = os.statvfs(m)
r["statfs"] = st.f_bsize > 0
print(json.dumps(r))
""")
    assert out["root"] == ["data", "many"] and out["many"] == 300
    import hashlib
    assert out["big_len"] == data.size and out["big_md5"] == hashlib.md5(data.tobytes()).hexdigest()
    assert out["mid"] == data[4 * MB - 3:4 * MB + 3].tobytes().hex()
    assert out["w_size"] == 256 * 4099 and out["w_ok"]
    assert out["moved"] == ["w2.bin"] and out["isdir"] and out.get("enoent")
    assert out["after_rm"] == [] and out["statfs"]
    # the writes landed in the namespace as completed files
    assert fs.exists("/x") and not fs.exists("/w.bin")
    assert srv.requests > 0


def test_existing_file_is_write_once(mounted):
    fs, mnt, _ = mounted
    fs.write_file("/wo/f", b"abc", write_type="MUST_CACHE")
    out = _posix(f"""
import errno, json, os
m = {mnt!r}
r = {{}}
try:
    with open(m + "/wo/f", "r+b") as f:
        f.write(b"zz")
except OSError as e:
    r["err"] = e.errno
with open(m + "/wo/f", "wb") as f:       # O_TRUNC rewrites the file
    f.write(b"new-bytes")
r["now"] = open(m + "/wo/f", "rb").read().decode()
print(json.dumps(r))
""")
    assert out["err"] in (13, 95) and out["now"] == "new-bytes"
