"""S3 proxy + REST API tests, and the S3 UFS driven end-to-end against the proxy.

Mirrors core/server/proxy's S3 handler behavior (reference tests/.../proxy/s3/S3ClientRestApiTest)
and the UFS contract checks (integration/tools/validation UnderFileSystemContractTest) with the
project's own S3 client as the counterpart — no external S3 service is reachable here."""
import json
import os
import xml.etree.ElementTree as ET

import pytest
import requests

from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.proxy import ProxyServer

CONF = {"alluxio.worker.tieredstore.level0.dirs.path": "dram", "alluxio.user.block.size.bytes.default": "1MB"}


@pytest.fixture(scope="module")
def env():
    with LocalAlluxioCluster(num_workers=1, conf=CONF) as c:
        fs = c.client()
        srv = ProxyServer(fs, "127.0.0.1", 0)
        port = srv.start()
        yield c, fs, f"http://127.0.0.1:{port}"
        srv.stop()
        fs.close()


def _tags(xml_bytes, tag):
    return [e.text for e in ET.fromstring(xml_bytes).iter() if e.tag.split("}")[-1] == tag]


def test_bucket_and_object_lifecycle(env):
    c, fs, url = env
    assert requests.put(f"{url}/bkt").status_code == 200
    assert requests.put(f"{url}/bkt").status_code == 409
    assert "bkt" in _tags(requests.get(f"{url}/").content, "Name")
    data = os.urandom(3 * (1 << 20) + 5)
    r = requests.put(f"{url}/bkt/dir/obj.bin", data=data)
    assert r.status_code == 200 and r.headers["ETag"].strip('"')
    assert fs.read_file("/bkt/dir/obj.bin") == data
    h = requests.head(f"{url}/bkt/dir/obj.bin")
    assert h.status_code == 200 and int(h.headers["Content-Length"]) == len(data)
    assert requests.get(f"{url}/bkt/dir/obj.bin").content == data
    r = requests.get(f"{url}/bkt/dir/obj.bin", headers={"Range": "bytes=100-199"})
    assert r.status_code == 206 and r.content == data[100:200]
    r = requests.get(f"{url}/bkt/dir/obj.bin", headers={"Range": "bytes=-10"})
    assert r.content == data[-10:]
    assert requests.get(f"{url}/bkt/nope").status_code == 404
    assert requests.put(f"{url}/bkt/copy.bin", headers={"x-amz-copy-source": "/bkt/dir/obj.bin"}).status_code == 200
    assert fs.read_file("/bkt/copy.bin") == data
    assert requests.delete(f"{url}/bkt").status_code == 409
    assert requests.delete(f"{url}/bkt/copy.bin").status_code == 204
    assert not fs.exists("/bkt/copy.bin")
    # S3 API under the reference's /api/v1/s3 prefix too
    assert requests.get(f"{url}/api/v1/s3/bkt/dir/obj.bin").content == data


def test_list_objects(env):
    c, fs, url = env
    requests.put(f"{url}/lst")
    for k in ["a/1", "a/2", "b/x/3", "c"]:
        requests.put(f"{url}/lst/{k}", data=k.encode())
    r = requests.get(f"{url}/lst", params={"list-type": "2"})
    keys = _tags(r.content, "Key")
    assert [k for k in keys if not k.endswith("/")] == ["a/1", "a/2", "b/x/3", "c"]
    r = requests.get(f"{url}/lst", params={"list-type": "2", "delimiter": "/"})
    assert _tags(r.content, "Key") == ["c"] and _tags(r.content, "Prefix")[1:] == ["a/", "b/"]
    r = requests.get(f"{url}/lst", params={"list-type": "2", "prefix": "a/", "delimiter": "/"})
    assert [k for k in _tags(r.content, "Key") if k != "a/"] == ["a/1", "a/2"]
    # pagination
    r = requests.get(f"{url}/lst", params={"list-type": "2", "max-keys": "2", "delimiter": "/"})
    assert _tags(r.content, "IsTruncated") == ["true"]
    tok = _tags(r.content, "NextContinuationToken")[0]
    r2 = requests.get(f"{url}/lst", params={"list-type": "2", "max-keys": "2", "delimiter": "/",
                                            "continuation-token": tok})
    assert _tags(r2.content, "IsTruncated") == ["false"]
    body = "<Delete><Object><Key>a/1</Key></Object><Object><Key>c</Key></Object></Delete>"
    r = requests.post(f"{url}/lst", params={"delete": ""}, data=body)
    assert r.status_code == 200 and sorted(_tags(r.content, "Key")) == ["a/1", "c"]
    assert not fs.exists("/lst/c")


def test_multipart(env):
    c, fs, url = env
    requests.put(f"{url}/mp")
    r = requests.post(f"{url}/mp/big", params={"uploads": ""})
    uid = _tags(r.content, "UploadId")[0]
    parts = [os.urandom(1 << 20) for _ in range(3)]
    for i, p in enumerate(parts, start=1):
        assert requests.put(f"{url}/mp/big", params={"partNumber": i, "uploadId": uid}, data=p).status_code == 200
    r = requests.get(f"{url}/mp/big", params={"uploadId": uid})
    assert _tags(r.content, "PartNumber") == ["1", "2", "3"]
    done = "<CompleteMultipartUpload>" + "".join(f"<Part><PartNumber>{i}</PartNumber></Part>" for i in (1, 2, 3)) + \
        "</CompleteMultipartUpload>"
    assert requests.post(f"{url}/mp/big", params={"uploadId": uid}, data=done).status_code == 200
    assert fs.read_file("/mp/big") == b"".join(parts)
    r = requests.post(f"{url}/mp/gone", params={"uploads": ""})
    uid2 = _tags(r.content, "UploadId")[0]
    assert requests.delete(f"{url}/mp/gone", params={"uploadId": uid2}).status_code == 204
    assert requests.get(f"{url}/mp/gone", params={"uploadId": uid2}).status_code == 404


def test_paths_and_streams_api(env):
    c, fs, url = env
    assert requests.post(f"{url}/api/v1/paths//rest/d/create-directory", json={"recursive": True}).status_code == 200
    sid = requests.post(f"{url}/api/v1/paths//rest/d/f/create-file", json={}).json()
    assert requests.post(f"{url}/api/v1/streams/{sid}/write", data=b"payload").json() == 7
    requests.post(f"{url}/api/v1/streams/{sid}/close")
    st = requests.post(f"{url}/api/v1/paths//rest/d/f/get-status").json()
    assert st["length"] == 7 and not st["folder"]
    assert requests.post(f"{url}/api/v1/paths//rest/d/f/exists").json() is True
    rid = requests.post(f"{url}/api/v1/paths//rest/d/f/open-file").json()
    assert requests.post(f"{url}/api/v1/streams/{rid}/read").content == b"payload"
    requests.post(f"{url}/api/v1/streams/{rid}/close")
    ls = requests.post(f"{url}/api/v1/paths//rest/d/list-status").json()
    assert [x["name"] for x in ls] == ["f"]
    assert requests.post(f"{url}/api/v1/paths//rest/d/f/rename", params={"dst": "/rest/d/g"}).status_code == 200
    assert requests.get(f"{url}/api/v1/paths//rest/d/g/download-file").content == b"payload"
    assert requests.post(f"{url}/api/v1/paths//rest/d/g/delete").status_code == 200
    assert requests.post(f"{url}/api/v1/paths//rest/nope/get-status").status_code == 404


def test_s3_ufs_against_proxy(env):
    """Mount an s3:// UFS served by the proxy (bucket backed by this same cluster) and run the
    UFS contract + Alluxio read/write through it."""
    c, fs, url = env
    requests.put(f"{url}/ufsbucket")
    from alluxio_amd.underfs import registry
    props = {"alluxio.underfs.s3.endpoint": url, "s3a.accessKeyId": "k", "s3a.secretKey": "s"}
    ufs = registry.create("s3://ufsbucket/", None, props)
    root = "s3://ufsbucket/contract"
    ufs.mkdirs(root)
    assert ufs.is_directory(root)
    with ufs.create(root + "/f1") as f:
        f.write(b"hello s3")
    assert ufs.is_file(root + "/f1") and ufs.get_file_status(root + "/f1").content_length == 8
    with ufs.open(root + "/f1") as f:
        assert f.read() == b"hello s3"
    assert sorted(s.name for s in ufs.list_status(root)) == ["f1"]
    assert ufs.rename_file(root + "/f1", root + "/f2")
    assert not ufs.exists(root + "/f1") and ufs.exists(root + "/f2")
    assert ufs.delete_file(root + "/f2")
    # mount it into the namespace and go through the client
    ufs.mkdirs("s3://ufsbucket/mnt")
    fs.mount("/s3mnt", "s3://ufsbucket/mnt", properties=props)
    fs.write_file("/s3mnt/x", b"through s3" * 1000, write_type="CACHE_THROUGH")
    assert fs.get_status("/s3mnt/x").is_persisted
    assert fs.read_file("/ufsbucket/mnt/x") == b"through s3" * 1000  # the object landed in the bucket
    fs.free("/s3mnt/x")
    assert fs.read_file("/s3mnt/x") == b"through s3" * 1000
    fs.unmount("/s3mnt")
