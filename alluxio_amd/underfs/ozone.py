"""Apache Ozone UFS: ``o3fs://<bucket>.<volume>[.<om-host>[:port]]/<path>`` and
``ofs://<om-host>/<volume>/<bucket>/<path>``.

Parity: underfs/ozone/src/main/java/alluxio/underfs/ozone/OzoneUnderFileSystemFactory.java (an
HDFS-API UFS registered for the ``o3fs`` scheme, delegating to Ozone's Hadoop client).  There is no
JVM here, so the connector talks to Ozone's S3 gateway (the ``s3g`` service every Ozone cluster
ships; ``alluxio.underfs.ozone.s3g.endpoint``, default ``http://<om-host>:9878``): buckets of the
S3 volume are addressed by name, and the object-store semantics (folder markers, copy-based
rename, ranged reads, multipart upload) come from the S3 connector.
"""
from __future__ import annotations

import urllib.parse

from .registry import UnderFileSystemFactory, register_factory
from .s3 import S3UnderFileSystem


def _split(uri: str) -> tuple[str, str, str]:
    """-> (om host[:port] or "", bucket, key prefix)."""
    u = urllib.parse.urlsplit(uri)
    if u.scheme == "o3fs":
        parts = u.netloc.split(".", 2)
        if len(parts) < 2:
            raise ValueError(f"o3fs URI needs <bucket>.<volume>: {uri}")
        om = parts[2] if len(parts) == 3 else ""
        return om, parts[0], u.path.lstrip("/")
    segs = [s for s in u.path.split("/") if s]      # ofs://om/volume/bucket/key
    if len(segs) < 2:
        raise ValueError(f"ofs URI needs /<volume>/<bucket>: {uri}")
    return u.netloc, segs[1], "/".join(segs[2:])


class OzoneUnderFileSystem(S3UnderFileSystem):
    scheme = "o3fs"
    ufs_type = "ozone"

    def __init__(self, root_uri, conf=None, properties=None):
        om, bucket, prefix = _split(root_uri)
        p = dict(properties or {})
        ep = p.get("alluxio.underfs.ozone.s3g.endpoint") or (
            conf.get_raw("alluxio.underfs.ozone.s3g.endpoint") if conf is not None else None)
        if not ep:
            host = (om or "localhost").split(":")[0]
            ep = f"http://{host}:9878"
        p.setdefault("alluxio.underfs.s3.endpoint", ep)
        self._prefix = prefix
        super().__init__(f"s3://{bucket}/{prefix}", conf, p)
        self.root_uri = root_uri

    def _key(self, path: str) -> str:
        if "://" in path:
            om, bucket, key = _split(path)
            return key
        return path.lstrip("/")


class _OzoneFactory(UnderFileSystemFactory):
    def __init__(self, scheme):
        self.scheme = scheme

    def create(self, uri, conf=None, properties=None):
        u = OzoneUnderFileSystem(uri, conf, properties)
        u.scheme = self.scheme
        return u


register_factory(_OzoneFactory("o3fs"))
register_factory(_OzoneFactory("ofs"))
