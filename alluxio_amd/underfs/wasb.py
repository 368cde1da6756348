"""Azure Blob Storage UFS (``wasb://`` / ``wasbs://<container>@<account>.blob.core.windows.net/<path>``).

Parity: underfs/wasb/src/main/java/alluxio/underfs/wasb/WasbUnderFileSystem.java:38-120 (scheme
pair wasb/wasbs, account key from ``fs.azure.account.key.<account>.blob.core.windows.net``,
object-store semantics with the default block size) — the reference reaches Azure through
hadoop-azure's NativeAzureFileSystem; here the Blob service REST API is spoken directly with
SharedKey request signing: Put Blob / Put Block + Put Block List (large objects), Get Blob with
``x-ms-range``, Get Blob Properties, Delete Blob, List Blobs (prefix/delimiter/marker paging) and
Copy Blob (polled until ``x-ms-copy-status`` is success).
"""
from __future__ import annotations

import base64
import datetime
import hashlib
import hmac
import time
import urllib.parse
import xml.etree.ElementTree as ET

from .object_store import ObjectMeta, ObjectUnderFileSystem
from .registry import UnderFileSystemFactory, register_factory

API_VERSION = "2019-12-12"
_STD = ("Content-Encoding", "Content-Language", "Content-Length", "Content-MD5", "Content-Type", "Date",
        "If-Modified-Since", "If-Match", "If-None-Match", "If-Unmodified-Since", "Range")


def shared_key_signature(account: str, key_b64: str, method: str, path: str, query: dict, headers: dict) -> str:
    """SharedKey ``Authorization`` value for a Blob service request (storage services auth spec)."""
    h = {k.lower(): str(v) for k, v in headers.items()}
    std = []
    for name in _STD:
        v = h.get(name.lower(), "")
        if name == "Content-Length" and v == "0":
            v = ""
        std.append(v)
    canon_h = "".join(f"{k}:{h[k].strip()}\n" for k in sorted(h) if k.startswith("x-ms-"))
    canon_r = f"/{account}{path}"
    for k in sorted(query, key=str.lower):
        canon_r += f"\n{k.lower()}:{query[k]}"
    sts = f"{method}\n" + "\n".join(std) + "\n" + canon_h + canon_r
    sig = base64.b64encode(hmac.new(base64.b64decode(key_b64), sts.encode(), hashlib.sha256).digest()).decode()
    return f"SharedKey {account}:{sig}"


def _http_date() -> str:
    return datetime.datetime.now(datetime.timezone.utc).strftime("%a, %d %b %Y %H:%M:%S GMT")


def _parse_http_date(s: str | None) -> int | None:
    if not s:
        return None
    try:
        return int(datetime.datetime.strptime(s, "%a, %d %b %Y %H:%M:%S GMT")
                   .replace(tzinfo=datetime.timezone.utc).timestamp() * 1000)
    except ValueError:
        return None


class WasbUnderFileSystem(ObjectUnderFileSystem):
    scheme = "wasb"
    ufs_type = "wasb"
    block_threshold = 256 << 20     # single Put Blob up to here, then blocks
    block_size_put = 64 << 20

    def __init__(self, root_uri, conf=None, properties=None):
        super().__init__(root_uri, conf, properties)
        import requests
        p = dict(properties or {})
        u = urllib.parse.urlsplit(root_uri)
        if "@" not in u.netloc:
            raise ValueError(f"wasb URI needs <container>@<account-host>: {root_uri}")
        self.container, host = u.netloc.split("@", 1)
        self.account = host.split(".", 1)[0]

        def opt(name, default=None):
            if name in p:
                return p[name]
            if conf is not None and conf.get_raw(name) is not None:
                return conf.get_raw(name)
            return default
        self.key = opt(f"fs.azure.account.key.{host}") or opt(f"fs.azure.account.key.{self.account}.blob.core.windows.net")
        secure = u.scheme == "wasbs"
        self.endpoint = (opt("fs.azure.endpoint") or opt("alluxio.underfs.azure.endpoint")
                         or f"{'https' if secure else 'http'}://{host}").rstrip("/")
        self.session = requests.Session()
        self.timeout = 60.0

    # ---- transport --------------------------------------------------------------------------
    def _req(self, method, key="", query=None, data=b"", headers=None, ok=(200, 201, 202, 206)):
        query = dict(query or {})
        path = f"/{self.container}" + (("/" + urllib.parse.quote(key)) if key else "")
        h = {"x-ms-date": _http_date(), "x-ms-version": API_VERSION}
        h.update(headers or {})
        if method in ("PUT", "POST"):
            h["Content-Length"] = str(len(data))
        if self.key:
            h["Authorization"] = shared_key_signature(self.account, self.key, method, path, query, h)
        r = self.session.request(method, self.endpoint + path, params=query, data=data, headers=h,
                                 timeout=self.timeout)
        if r.status_code == 404:
            raise FileNotFoundError(key)
        if r.status_code not in ok:
            raise OSError(f"azure {method} {path}: HTTP {r.status_code} {r.text[:200]}")
        return r

    # ---- primitives -------------------------------------------------------------------------
    def _put(self, key, data):
        if len(data) <= self.block_threshold:
            self._req("PUT", key, data=data, headers={"x-ms-blob-type": "BlockBlob"})
            return
        ids = []
        for n, off in enumerate(range(0, len(data), self.block_size_put)):
            bid = base64.b64encode(f"{n:08d}".encode()).decode()
            self._req("PUT", key, query={"comp": "block", "blockid": bid}, data=data[off:off + self.block_size_put])
            ids.append(bid)
        body = "<?xml version=\"1.0\" encoding=\"utf-8\"?><BlockList>" + \
            "".join(f"<Latest>{i}</Latest>" for i in ids) + "</BlockList>"
        self._req("PUT", key, query={"comp": "blocklist"}, data=body.encode())

    def _get_range(self, key, offset, length):
        if length <= 0:
            return b""
        r = self._req("GET", key, headers={"x-ms-range": f"bytes={offset}-{offset + length - 1}"})
        return r.content

    def _head(self, key):
        try:
            r = self._req("HEAD", key)
        except FileNotFoundError:
            return None
        return ObjectMeta(key, int(r.headers.get("Content-Length", 0)), r.headers.get("ETag", "").strip('"'),
                          _parse_http_date(r.headers.get("Last-Modified")))

    def _delete(self, keys):
        for k in keys:
            if k:
                try:
                    self._req("DELETE", k)
                except FileNotFoundError:
                    pass

    def _list(self, prefix, delimiter):
        objs, prefixes, marker = [], [], None
        while True:
            q = {"restype": "container", "comp": "list", "prefix": prefix}
            if delimiter:
                q["delimiter"] = delimiter
            if marker:
                q["marker"] = marker
            root = ET.fromstring(self._req("GET", query=q).content)
            blobs = root.find("Blobs")
            for el in (blobs if blobs is not None else []):
                if el.tag == "Blob":
                    props = el.find("Properties")

                    def prop(name):
                        v = props.find(name) if props is not None else None
                        return v.text if v is not None else None
                    objs.append(ObjectMeta(el.findtext("Name"), int(prop("Content-Length") or 0),
                                           (prop("Etag") or "").strip('"'), _parse_http_date(prop("Last-Modified"))))
                elif el.tag == "BlobPrefix":
                    prefixes.append(el.findtext("Name"))
            marker = root.findtext("NextMarker")
            if not marker:
                return objs, prefixes

    def _copy(self, src, dst):
        src_url = f"{self.endpoint}/{self.container}/{urllib.parse.quote(src)}"
        r = self._req("PUT", dst, headers={"x-ms-copy-source": src_url})
        status = r.headers.get("x-ms-copy-status", "success")
        deadline = time.time() + 300
        while status == "pending" and time.time() < deadline:
            time.sleep(0.2)
            status = self._req("HEAD", dst).headers.get("x-ms-copy-status", "success")
        if status != "success":
            raise OSError(f"azure copy {src} -> {dst}: {status}")


class _WasbFactory(UnderFileSystemFactory):
    def __init__(self, scheme):
        self.scheme = scheme

    def create(self, uri, conf=None, properties=None):
        u = WasbUnderFileSystem(uri, conf, properties)
        u.scheme = self.scheme
        return u


register_factory(_WasbFactory("wasb"))
register_factory(_WasbFactory("wasbs"))
