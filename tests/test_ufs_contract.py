"""``alluxio runUfsTests``: the UFS contract runner against the local UFS, an object store (S3 via
this project's S3 proxy, with the multipart-specific operations), Swift simulation, WebHDFS, Azure
Blob (wasb, against the in-tree fake) and ADL (WebHDFS + OAuth2 fake).

Parity: integration/tools/validation/src/main/java/alluxio/cli/UnderFileSystemContractTest.java,
UnderFileSystemCommonOperations.java, S3ASpecificOperations.java.
"""
import io
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
from ufs_fakes import azure_server, webhdfs_server  # noqa: E402

from alluxio_amd.cli import main as cli  # noqa: E402
from alluxio_amd.cli import ufs_contract  # noqa: E402


def _ok(res):
    assert res["failed"] == [], res["failed"]
    assert len(res["passed"]) >= 40


def test_local_contract_via_cli(tmp_path):
    out = io.StringIO()
    rc = cli.main(["runUfsTests", "--path", str(tmp_path), "--large-file-size", "1000000"], out=out)
    assert rc == 0, out.getvalue()
    assert "Tests completed with 42 passed and 0 failed." in out.getvalue()
    assert os.listdir(tmp_path) == []           # the runner cleans its scratch directory


def test_single_operation_and_failure_reporting(tmp_path, monkeypatch):
    res = ufs_contract.run(str(tmp_path), test="rename_file_test", out=io.StringIO())
    assert res["passed"] == ["rename_file_test"]
    # a connector that breaks a contract is reported, not crashed on
    monkeypatch.setattr(ufs_contract.CommonOperations, "exists_test",
                        lambda self: ufs_contract._check(False, "broken"))
    res = ufs_contract.run(str(tmp_path), test="exists_test", out=io.StringIO())
    assert res["failed"] == [{"test": "exists_test", "error": "ContractFailure: broken"}]


def test_swift_simulation_contract():
    _ok(ufs_contract.run("swift://contractbkt/", properties={"fs.swift.simulation": "true"},
                         out=io.StringIO(), large_file_size=1 << 20))


def test_webhdfs_contract():
    srv, _ = webhdfs_server()
    try:
        _ok(ufs_contract.run(f"webhdfs://127.0.0.1:{srv.port}/", out=io.StringIO(), large_file_size=1 << 20,
                             properties={"alluxio.underfs.webhdfs.user": "u"}))
    finally:
        srv.stop()


def test_s3_contract_through_proxy(tmp_path):
    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.proxy import ProxyServer
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"},
                             work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        fs.create_directory("/contract")
        proxy = ProxyServer(fs, port=0)
        port = proxy.start()
        try:
            out = io.StringIO()
            res = ufs_contract.run("s3a://contract/", properties={"alluxio.underfs.s3.endpoint":
                                                                  f"http://127.0.0.1:{port}"},
                                   out=out, large_file_size=1 << 20)
            _ok(res)
            assert "S3ASpecificOperations#create_multipart_file_test" in out.getvalue()
        finally:
            proxy.stop()


def test_wasb_contract():
    srv, st = azure_server()
    try:
        props = {"fs.azure.account.key.acct.blob.core.windows.net": st.key, "fs.azure.endpoint": srv.url}
        _ok(ufs_contract.run("wasb://cont@acct.blob.core.windows.net/", properties=props, out=io.StringIO(),
                             large_file_size=1 << 20))
    finally:
        srv.stop()


def test_adl_contract():
    srv, _ = webhdfs_server(require_token="T0K")
    try:
        props = {"alluxio.underfs.adl.endpoint": srv.url + "/webhdfs/v1",
                 "fs.adl.account.myacct.oauth2.client.id": "cid",
                 "fs.adl.account.myacct.oauth2.credential": "sec",
                 "fs.adl.account.myacct.oauth2.refresh.url": srv.url + "/oauth2/token"}
        _ok(ufs_contract.run("adl://myacct.azuredatalakestore.net/", properties=props, out=io.StringIO(),
                             large_file_size=1 << 20))
    finally:
        srv.stop()


def test_local_ufs_writer_never_truncates_silently(tmp_path):
    """A write(2) may store fewer bytes than asked (one call stops at 2 GiB - 4 KiB); the local
    UFS writer loops, so a short write either completes or raises.  Here the file-size limit cuts
    the first write short and the next one fails with EFBIG: the caller sees an error, not a
    truncated file recorded at full length."""
    import subprocess
    import sys
    code = r"""
import resource, signal, sys
sys.path.insert(0, %r)
from alluxio_amd.underfs.base import CreateOptions
from alluxio_amd.underfs.local import LocalUnderFileSystem
signal.signal(signal.SIGXFSZ, signal.SIG_IGN)
resource.setrlimit(resource.RLIMIT_FSIZE, (1 << 20, resource.getrlimit(resource.RLIMIT_FSIZE)[1]))
ufs = LocalUnderFileSystem(%r)
for atomic in (True, False):
    f = ufs.create(%r + ("/a" if atomic else "/b"), CreateOptions(ensure_atomic=atomic))
    try:
        f.write(b"x" * (3 << 19))
    except OSError as e:
        print("raised", e.errno)
    else:
        print("no error")
""" % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), str(tmp_path), str(tmp_path))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.stdout.split("\n")[:2] == ["raised 27", "raised 27"], out.stdout + out.stderr


def test_local_delete_large_file_reclaims_in_background(tmp_path):
    """A large local file's delete returns once its name is gone; the kernel frees its pages when
    the reclaim thread closes the last descriptor (``unlink_deferred``).  Small files, symlinks
    and missing paths behave as ``os.remove`` does."""
    import os
    import time

    from alluxio_amd.ops.native import lib
    from alluxio_amd.underfs.local import LocalUnderFileSystem
    m = lib()
    ufs = LocalUnderFileSystem(str(tmp_path))
    big = tmp_path / "big.bin"
    big.write_bytes(b"\1" * (16 << 20))
    small = tmp_path / "small.bin"
    small.write_bytes(b"x" * 100)
    before = m.reclaimed_files()
    assert ufs.delete_file(str(big)) and not big.exists()
    assert ufs.delete_file(str(small)) and not small.exists()
    assert not ufs.delete_file(str(tmp_path / "missing"))
    deadline = time.time() + 10
    while m.reclaimed_files() < before + 1 and time.time() < deadline:
        time.sleep(0.01)
    assert m.reclaimed_files() == before + 1     # only the large one went through the thread
    # a name re-created right after the delete is a new file
    big.write_bytes(b"\2" * 10)
    assert big.read_bytes() == b"\2" * 10
    # a symlink is removed itself, never followed
    target = tmp_path / "target.bin"
    target.write_bytes(b"\3" * (16 << 20))
    link = tmp_path / "link"
    os.symlink(target, link)
    assert m.unlink_deferred(str(link)) == 0
    assert not os.path.lexists(link) and target.exists()
    assert m.unlink_deferred(str(tmp_path / "missing")) == 2     # ENOENT
