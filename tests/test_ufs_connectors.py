"""Swift / Azure Blob (wasb) / WebHDFS / ADL / Ozone connectors against in-process fakes.

Reference coverage model: underfs/*/src/test (factory scheme tests, Swift ACL->mode, WASB/ADL
configuration) plus the UFS contract suite (tests/.../UnderFileSystemContractTest.java: create,
open at offset, list, mkdirs, rename file/dir, delete empty/non-empty dir).
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(__file__))
from ufs_fakes import azure_server, swift_server, webhdfs_server  # noqa: E402

from alluxio_amd.underfs import registry  # noqa: E402
from alluxio_amd.underfs.base import DeleteOptions, ListOptions, MkdirsOptions, OpenOptions  # noqa: E402


def contract(ufs, root=""):
    P = lambda p: root + p  # noqa: E731
    assert ufs.mkdirs(P("/d1/d2"))
    assert ufs.is_directory(P("/d1")) and ufs.is_directory(P("/d1/d2"))
    assert not ufs.mkdirs(P("/x/y"), MkdirsOptions(create_parent=False))
    ufs.write_all(P("/d1/f"), b"x" * 1000 + b"y" * 1000)
    st = ufs.get_status(P("/d1/f"))
    assert st.is_file and st.content_length == 2000 and st.name == "f"
    with ufs.open(P("/d1/f"), OpenOptions(offset=1500)) as f:
        assert f.read() == b"y" * 500
    assert ufs.read_all(P("/d1/f"))[995:1005] == b"xxxxxyyyyy"
    assert sorted(s.name for s in ufs.list_status(P("/d1"))) == ["d2", "f"]
    ufs.write_all(P("/d1/d2/h"), b"hh")
    rec = sorted(s.name for s in ufs.list_status(P("/d1"), ListOptions(recursive=True)))
    assert rec == ["d2", "d2/h", "f"]
    assert ufs.rename_file(P("/d1/f"), P("/d1/g"))
    assert not ufs.exists(P("/d1/f")) and ufs.read_all(P("/d1/g")) == b"x" * 1000 + b"y" * 1000
    assert ufs.rename_directory(P("/d1"), P("/e1"))
    assert not ufs.exists(P("/d1")) and ufs.read_all(P("/e1/d2/h")) == b"hh"
    assert not ufs.delete_directory(P("/e1"))                       # not empty
    assert ufs.delete_directory(P("/e1"), DeleteOptions(recursive=True))
    assert not ufs.exists(P("/e1")) and not ufs.delete_file(P("/nope"))
    assert ufs.get_status(P("/missing")) is None and ufs.list_status(P("/missing")) is None


@pytest.mark.parametrize("method", ["tempauth", "keystonev3"])
def test_swift(method):
    srv, st = swift_server()
    try:
        props = {"fs.swift.user": "alice", "fs.swift.tenant": "proj", "fs.swift.password": "pw",
                 "fs.swift.auth.method": method, "fs.swift.region": "r1",
                 "fs.swift.auth.url": srv.url + ("/auth/v1.0" if method == "tempauth" else "/v3")}
        ufs = registry.create("swift://bkt/", properties=props)
        assert ufs.ufs_type == "swift" and ufs.mode == 0o500          # read ACL names the owner
        contract(ufs)
        assert ufs.get_status("/").is_directory
        st.tokens.clear()                                            # expired token -> re-auth once
        ufs.write_all("/again", b"1")
        assert ufs.read_all("/again") == b"1" and st.auth_calls == 2
        with pytest.raises(PermissionError):
            registry.create("swift://bkt/", properties=dict(props, **{"fs.swift.password": "bad"}))
    finally:
        srv.stop()


def test_swift_simulation():
    ufs = registry.create("swift://simbkt/", properties={"fs.swift.simulation": "true"})
    contract(ufs)


def test_wasb_shared_key_and_paging():
    srv, st = azure_server()
    try:
        props = {"fs.azure.account.key.acct.blob.core.windows.net": st.key, "fs.azure.endpoint": srv.url}
        ufs = registry.create("wasb://cont@acct.blob.core.windows.net/", properties=props)
        assert ufs.ufs_type == "wasb"
        contract(ufs)
        ufs.block_threshold, ufs.block_size_put = 1000, 300     # Put Block + Put Block List
        data = os.urandom(2500)
        ufs.write_all("/big", data)
        assert ufs.read_all("/big") == data
        for i in range(7):                                      # listing pages of 3 (NextMarker)
            ufs.write_all(f"/many/f{i}", b"z")
        assert len(ufs.list_status("/many")) == 7
        assert st.bad_sigs == 0
        bad = registry.create("wasb://cont@acct.blob.core.windows.net/", properties={
            "fs.azure.account.key.acct.blob.core.windows.net": "d3Jvbmc=", "fs.azure.endpoint": srv.url})
        with pytest.raises(OSError):
            bad.write_all("/x", b"1")
    finally:
        srv.stop()


def test_webhdfs_two_step_create_and_metadata():
    srv, st = webhdfs_server()
    try:
        ufs = registry.create(f"webhdfs://127.0.0.1:{srv.port}/", properties={"alluxio.underfs.webhdfs.user": "u"})
        contract(ufs)
        ufs.write_all("/m/f", b"abc")
        ufs.set_mode("/m/f", 0o600)
        ufs.set_owner("/m/f", "bob", "staff")
        s = ufs.get_status("/m/f")
        assert (s.mode, s.owner, s.group) == (0o600, "bob", "staff")
        from alluxio_amd.underfs.base import SpaceType
        assert ufs.get_space("/m", SpaceType.SPACE_USED) == 3
    finally:
        srv.stop()


def test_adl_oauth2():
    srv, st = webhdfs_server(require_token="T0K")
    try:
        props = {"alluxio.underfs.adl.endpoint": srv.url + "/webhdfs/v1",
                 "fs.adl.account.myacct.oauth2.client.id": "cid",
                 "fs.adl.account.myacct.oauth2.credential": "sec",
                 "fs.adl.account.myacct.oauth2.refresh.url": srv.url + "/oauth2/token"}
        ufs = registry.create("adl://myacct.azuredatalakestore.net/", properties=props)
        assert ufs.ufs_type == "adl" and ufs.is_object_storage()
        contract(ufs)
        assert st.token_requests == 1                            # cached bearer token
    finally:
        srv.stop()


def test_ozone_via_s3_gateway(tmp_path):
    """o3fs / ofs URIs resolve to the Ozone S3 gateway; exercised against this project's S3 proxy."""
    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.proxy import ProxyServer
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"},
                             work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        fs.create_directory("/ozbucket")
        proxy = ProxyServer(fs, port=0)
        port = proxy.start()
        try:
            props = {"alluxio.underfs.ozone.s3g.endpoint": f"http://127.0.0.1:{port}"}
            for uri in ("o3fs://ozbucket.vol1.om-host/", "ofs://om-host/vol1/ozbucket/"):
                ufs = registry.create(uri, properties=props)
                assert ufs.ufs_type == "ozone"
                ufs.write_all(uri + "k/obj", b"ozone")
                assert ufs.read_all("/k/obj") == b"ozone"
                assert [s.name for s in ufs.list_status("/k")] == ["obj"]
                assert ufs.delete_file("/k/obj")
        finally:
            proxy.stop()
            fs.close()
