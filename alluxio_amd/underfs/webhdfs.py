"""WebHDFS-protocol UFS: ``webhdfs://`` / ``swebhdfs://`` (HDFS over REST) and ``adl://`` (Azure
Data Lake Storage Gen1, which serves the WebHDFS API with OAuth2 bearer tokens).

Parity: underfs/adl/src/main/java/alluxio/underfs/adl/AdlUnderFileSystem.java:38-110 (an
HdfsUnderFileSystem configured with ``fs.adl.oauth2.client.id`` / ``credential`` /
``refresh.url`` — account-scoped ``fs.adl.account.<account>.oauth2.*`` keys win — and the
default block size because ADL is object-store backed) and the HDFS UFS operations it inherits
(underfs/hdfs/.../HdfsUnderFileSystem.java: create/open/delete/rename/list/mkdirs/setOwner/
setMode/getStatus).  Without a JVM/libhdfs in the image, both go through the WebHDFS REST API:
GETFILESTATUS, LISTSTATUS, MKDIRS, CREATE (two-step redirect, or ``write=true`` on ADL),
OPEN with offset/length, DELETE, RENAME, SETPERMISSION, SETOWNER, GETCONTENTSUMMARY.
"""
from __future__ import annotations

import io
import posixpath
import threading
import time
import urllib.parse

from .base import (CreateOptions, DeleteOptions, ListOptions, MkdirsOptions, OpenOptions, SpaceType,
                   UfsDirectoryStatus, UfsFileStatus, UnderFileSystem)
from .registry import UnderFileSystemFactory, register_factory


class _OAuth2ClientCredentials:
    """Client-credential token source (ADL's ClientCredsTokenProvider)."""

    def __init__(self, session, refresh_url: str, client_id: str, secret: str,
                 resource: str = "https://datalake.azure.net/"):
        self.session, self.url, self.client_id, self.secret, self.resource = \
            session, refresh_url, client_id, secret, resource
        self._token, self._expiry = None, 0.0
        self._lock = threading.Lock()

    def token(self) -> str:
        with self._lock:
            if self._token is None or time.time() > self._expiry - 60:
                r = self.session.post(self.url, data={"grant_type": "client_credentials", "client_id": self.client_id,
                                                      "client_secret": self.secret, "resource": self.resource},
                                      timeout=30)
                if r.status_code >= 400:
                    raise PermissionError(f"OAuth2 token request failed: HTTP {r.status_code}")
                d = r.json()
                self._token = d["access_token"]
                self._expiry = time.time() + float(d.get("expires_in", 3600))
            return self._token


class _WebHdfsWriter(io.RawIOBase):
    def __init__(self, ufs: "WebHdfsUnderFileSystem", path: str, options: CreateOptions | None):
        super().__init__()
        self._ufs, self._path, self._opts = ufs, path, options
        self._buf = io.BytesIO()

    def writable(self):
        return True

    def write(self, b):
        return self._buf.write(b)

    def close(self):
        if not self.closed:
            self._ufs._create(self._path, self._buf.getvalue(), self._opts)
        super().close()


class _WebHdfsReader(io.RawIOBase):
    def __init__(self, ufs, path, size, offset, chunk):
        super().__init__()
        self._ufs, self._path, self._size, self._pos, self._chunk = ufs, path, size, offset, chunk

    def readable(self):
        return True

    def seekable(self):
        return True

    def seek(self, off, whence=0):
        self._pos = {0: off, 1: self._pos + off, 2: self._size + off}[whence]
        return self._pos

    def tell(self):
        return self._pos

    def readinto(self, b):
        if self._pos >= self._size:
            return 0
        n = min(len(b), self._size - self._pos, self._chunk)
        data = self._ufs._read(self._path, self._pos, n)
        b[:len(data)] = data
        self._pos += len(data)
        return len(data)


class WebHdfsUnderFileSystem(UnderFileSystem):
    scheme = "webhdfs"
    ufs_type = "webhdfs"
    read_chunk = 8 << 20

    def __init__(self, root_uri, conf=None, properties=None):
        super().__init__(root_uri, conf, properties)
        import requests
        p = dict(properties or {})
        self._opt = lambda name, default=None: p.get(name) if name in p else (
            conf.get_raw(name) if conf is not None and conf.get_raw(name) is not None else default)
        u = urllib.parse.urlsplit(root_uri)
        self.host = u.netloc
        self.session = requests.Session()
        self.timeout = 60.0
        self.user = self._opt("alluxio.underfs.webhdfs.user") or self._opt("hadoop.user.name")
        self.auth = None
        self.base = self._base_url(u)
        self.block_size = 64 << 20

    def _base_url(self, u) -> str:
        https = u.scheme == "swebhdfs"
        return self._opt("alluxio.underfs.webhdfs.endpoint") or \
            f"{'https' if https else 'http'}://{u.netloc}/webhdfs/v1"

    # ---- transport --------------------------------------------------------------------------
    def _path(self, path: str) -> str:
        if "://" in path:
            path = urllib.parse.urlsplit(path).path
        return "/" + path.lstrip("/")

    def _req(self, method, path, op, params=None, data=None, redirect=True, ok=(200, 201)):
        q = {"op": op}
        q.update(params or {})
        if self.user and self.auth is None:
            q["user.name"] = self.user
        h = {}
        if self.auth is not None:
            h["Authorization"] = f"Bearer {self.auth.token()}"
        url = self.base + urllib.parse.quote(self._path(path))
        r = self.session.request(method, url, params=q, data=data, headers=h, timeout=self.timeout,
                                 allow_redirects=redirect)
        if r.status_code == 404:
            raise FileNotFoundError(path)
        if r.status_code in (401, 403):
            raise PermissionError(f"webhdfs {op} {path}: HTTP {r.status_code}")
        if r.status_code not in ok:
            raise OSError(f"webhdfs {op} {path}: HTTP {r.status_code} {r.text[:200]}")
        return r

    def _create(self, path, data: bytes, options: CreateOptions | None) -> None:
        params = {"overwrite": "true"}
        if options is not None and getattr(options, "mode", None):
            params["permission"] = format(options.mode & 0o7777, "o")
        # step 1 asks the namenode for a datanode location, step 2 sends the bytes there
        r = self._req("PUT", path, "CREATE", params, redirect=False, ok=(200, 201, 307))
        if r.status_code == 307:
            loc = r.headers["Location"]
            h = {"Content-Type": "application/octet-stream"}
            if self.auth is not None:
                h["Authorization"] = f"Bearer {self.auth.token()}"
            rr = self.session.put(loc, data=data, headers=h, timeout=self.timeout)
            if rr.status_code not in (200, 201):
                raise OSError(f"webhdfs CREATE {path} (datanode): HTTP {rr.status_code}")

    def _read(self, path, offset, length) -> bytes:
        return self._req("GET", path, "OPEN", {"offset": offset, "length": length}).content

    @staticmethod
    def _status(name: str, fs: dict):
        mode = int(fs.get("permission", "755"), 8)
        mtime = fs.get("modificationTime")
        if fs.get("type") == "DIRECTORY":
            return UfsDirectoryStatus(name, fs.get("owner", ""), fs.get("group", ""), mode, mtime)
        return UfsFileStatus(name, int(fs.get("length", 0)), f"{fs.get('length', 0)}:{mtime}", mtime,
                             fs.get("owner", ""), fs.get("group", ""), mode, int(fs.get("blockSize") or 64 << 20))

    # ---- UnderFileSystem --------------------------------------------------------------------
    def create(self, path, options: CreateOptions | None = None):
        parent = posixpath.dirname(self._path(path))
        if parent not in ("", "/") and not self.is_directory(parent):
            if options is None or getattr(options, "create_parent", True):
                self.mkdirs(parent)
            else:
                # WebHDFS CREATE makes missing parents on the server (HDFS create()); a
                # non-recursive create is enforced here, as createNonRecursive would be
                raise FileNotFoundError(f"parent of {path} does not exist")
        return _WebHdfsWriter(self, path, options)

    def open(self, path, options: OpenOptions | None = None):
        st = self.get_status(path)
        if st is None or st.is_directory:
            raise FileNotFoundError(path)
        off = options.offset if options else 0
        return io.BufferedReader(_WebHdfsReader(self, path, st.content_length, off, self.read_chunk), 1 << 20)

    def get_status(self, path):
        try:
            fs = self._req("GET", path, "GETFILESTATUS").json()["FileStatus"]
        except FileNotFoundError:
            return None
        name = posixpath.basename(self._path(path).rstrip("/")) or "/"
        st = self._status(name, fs)
        if st.is_file and self.ufs_type == "adl":
            st.block_size = self.block_size
        return st

    def list_status(self, path, options: ListOptions | None = None):
        st = self.get_status(path)
        if st is None or not st.is_directory:
            return None
        out = []
        base = self._path(path).rstrip("/")
        for fs in self._req("GET", path, "LISTSTATUS").json()["FileStatuses"]["FileStatus"]:
            name = fs["pathSuffix"]
            out.append(self._status(name, fs))
            if options and options.recursive and fs.get("type") == "DIRECTORY":
                for c in self.list_status(f"{base}/{name}", options) or []:
                    c.name = f"{name}/{c.name}"
                    out.append(c)
        return sorted(out, key=lambda s: s.name)

    def mkdirs(self, path, options: MkdirsOptions | None = None):
        if self.exists(path):
            return False
        if options is not None and not options.create_parent:
            parent = posixpath.dirname(self._path(path).rstrip("/"))
            if parent not in ("", "/") and not self.is_directory(parent):
                return False
        params = {}
        if options is not None and getattr(options, "mode", None):
            params["permission"] = format(options.mode & 0o7777, "o")
        return bool(self._req("PUT", path, "MKDIRS", params).json().get("boolean"))

    def delete_file(self, path):
        st = self.get_status(path)
        if st is None or st.is_directory:
            return False
        return bool(self._req("DELETE", path, "DELETE", {"recursive": "false"}).json().get("boolean"))

    def delete_directory(self, path, options: DeleteOptions | None = None):
        st = self.get_status(path)
        if st is None or not st.is_directory:
            return False
        rec = bool(options and options.recursive)
        if not rec and self.list_status(path):
            return False
        return bool(self._req("DELETE", path, "DELETE", {"recursive": str(rec).lower()}).json().get("boolean"))

    def _rename(self, src, dst):
        if self.exists(dst):
            return False
        return bool(self._req("PUT", src, "RENAME", {"destination": self._path(dst)}).json().get("boolean"))

    def rename_file(self, src, dst):
        return self.is_file(src) and self._rename(src, dst)

    def rename_directory(self, src, dst):
        return self.is_directory(src) and self._rename(src, dst)

    def set_owner(self, path, owner, group):
        params = {}
        if owner:
            params["owner"] = owner
        if group:
            params["group"] = group
        if params:
            self._req("PUT", path, "SETOWNER", params)

    def set_mode(self, path, mode):
        self._req("PUT", path, "SETPERMISSION", {"permission": format(mode & 0o7777, "o")})

    def get_space(self, path, space_type: SpaceType) -> int:
        try:
            cs = self._req("GET", path, "GETCONTENTSUMMARY").json()["ContentSummary"]
        except (OSError, KeyError, ValueError):
            return -1
        if space_type == SpaceType.SPACE_USED:
            return int(cs.get("spaceConsumed", cs.get("length", 0)))
        quota = int(cs.get("spaceQuota", -1))
        if space_type == SpaceType.SPACE_TOTAL:
            return quota
        return quota - int(cs.get("spaceConsumed", 0)) if quota >= 0 else -1

    def resolve_uri(self, base, alluxio_path):
        return base.rstrip("/") + "/" + alluxio_path.lstrip("/")


class AdlUnderFileSystem(WebHdfsUnderFileSystem):
    scheme = "adl"
    ufs_type = "adl"

    def __init__(self, root_uri, conf=None, properties=None):
        super().__init__(root_uri, conf, properties)
        account = self.host.split(".", 1)[0]

        def key(suffix):
            return self._opt(f"fs.adl.account.{account}.oauth2.{suffix}") or self._opt(f"fs.adl.oauth2.{suffix}")
        cid, secret, url = key("client.id"), key("credential"), key("refresh.url")
        if cid and url:
            self.auth = _OAuth2ClientCredentials(self.session, url, cid, secret or "")
        ufs_bs = self._opt("alluxio.user.block.size.bytes.default")
        if ufs_bs:
            from ..utils.format import parse_space_size
            self.block_size = parse_space_size(ufs_bs)

    def _base_url(self, u) -> str:
        return self._opt("alluxio.underfs.adl.endpoint") or f"https://{u.netloc}/webhdfs/v1"

    def _create(self, path, data, options):
        # ADL accepts the bytes on the first request (write=true), no datanode redirect
        params = {"overwrite": "true", "write": "true"}
        if options is not None and getattr(options, "mode", None):
            params["permission"] = format(options.mode & 0o7777, "o")
        self._req("PUT", path, "CREATE", params, data=data, ok=(200, 201))

    def is_object_storage(self) -> bool:
        return True


class _Factory(UnderFileSystemFactory):
    def __init__(self, scheme, cls):
        self.scheme, self.cls = scheme, cls

    def create(self, uri, conf=None, properties=None):
        u = self.cls(uri, conf, properties)
        u.scheme = self.scheme
        return u


register_factory(_Factory("webhdfs", WebHdfsUnderFileSystem))
register_factory(_Factory("swebhdfs", WebHdfsUnderFileSystem))
register_factory(_Factory("adl", AdlUnderFileSystem))
