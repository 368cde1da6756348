"""S3-compatible UFS over plain HTTP with AWS Signature V4 (no boto3 in this image).

Parity target: underfs/s3a/src/main/java/alluxio/underfs/s3a/S3AUnderFileSystem.java (key
mapping, folder suffix, ranged GET streams, multi-object delete, copy-based rename) and
S3ALowLevelOutputStream.java (multipart upload for large objects).  Works against any
S3-compatible endpoint — including this project's own S3 REST proxy (alluxio_amd/proxy), which
is how it is exercised in tests.  GCS/OSS/COS/Kodo S3-interop endpoints use the same class via
their schemes (``gs://``, ``oss://``, ``cosn://``, ``kodo://``) with an explicit endpoint.
"""
from __future__ import annotations

import datetime
import hashlib
import hmac
import urllib.parse
import xml.etree.ElementTree as ET

from .object_store import ObjectMeta, ObjectUnderFileSystem
from .registry import UnderFileSystemFactory, register_factory

_EMPTY_SHA = hashlib.sha256(b"").hexdigest()


def _sign(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


# HTTP statuses an S3 client retries (AWS SDK PredefinedRetryPolicies: throttling and 5xx)
RETRYABLE_STATUS = frozenset((429, 500, 502, 503, 504))


class S3Client:
    """Signed S3 calls over a pooled ``requests`` session, with the reference client's limits
    (S3AUnderFileSystem.java:150-191): ``socket_timeout`` bounds each wait on the socket,
    ``request_timeout`` one call with all its attempts (0 = none), and a call failing with a
    connection error, a timeout, 5xx or 429 (SlowDown) is retried ``max_retries`` times with capped
    exponential back-off (AWS SDK default: 3)."""

    def __init__(self, endpoint: str, access_key: str = "", secret_key: str = "",
                 region: str = "us-east-1", timeout: float = 60.0, socket_timeout: float = 50.0,
                 connect_timeout: float = 10.0, max_retries: int = 3, backoff_base: float = 0.05,
                 backoff_max: float = 2.0):
        import requests
        self.endpoint = endpoint.rstrip("/")
        self.access_key, self.secret_key, self.region = access_key, secret_key, region
        self.session = requests.Session()
        self.timeout = timeout                  # request timeout (all attempts)
        self.socket_timeout = socket_timeout
        self.connect_timeout = min(connect_timeout, socket_timeout) if socket_timeout else connect_timeout
        self.max_retries = max(0, int(max_retries))
        self.backoff_base, self.backoff_max = backoff_base, backoff_max
        self.retries = 0                        # attempts beyond the first, over the client's life

    def _headers(self, method, path, query: dict, payload_hash: str, extra=None) -> dict:
        host = urllib.parse.urlsplit(self.endpoint).netloc
        now = datetime.datetime.now(datetime.timezone.utc)
        amz_date = now.strftime("%Y%m%dT%H%M%SZ")
        date = now.strftime("%Y%m%d")
        headers = {"host": host, "x-amz-date": amz_date, "x-amz-content-sha256": payload_hash}
        if extra:
            headers.update({k.lower(): v for k, v in extra.items()})
        if not self.access_key:
            return headers
        canon_q = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(str(v), safe='-_.~')}"
                           for k, v in sorted(query.items()))
        signed = ";".join(sorted(headers))
        canon_h = "".join(f"{k}:{headers[k].strip()}\n" for k in sorted(headers))
        creq = "\n".join([method, urllib.parse.quote(path, safe="/-_.~"), canon_q, canon_h, signed, payload_hash])
        scope = f"{date}/{self.region}/s3/aws4_request"
        sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(creq.encode()).hexdigest()])
        k = _sign(("AWS4" + self.secret_key).encode(), date)
        k = _sign(k, self.region)
        k = _sign(k, "s3")
        k = _sign(k, "aws4_request")
        sig = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
        headers["authorization"] = (f"AWS4-HMAC-SHA256 Credential={self.access_key}/{scope}, "
                                    f"SignedHeaders={signed}, Signature={sig}")
        return headers

    def request(self, method, bucket, key="", query=None, data=b"", headers=None, ok=(200, 204, 206)):
        import random
        import time

        import requests
        query = query or {}
        path = f"/{bucket}/{key}" if key else f"/{bucket}"
        ph = hashlib.sha256(data).hexdigest() if data else _EMPTY_SHA
        url = self.endpoint + urllib.parse.quote(path, safe="/-_.~")
        deadline = time.monotonic() + self.timeout if self.timeout else None
        attempt = 0
        while True:
            h = self._headers(method, path, query, ph, headers)     # a fresh signature date per attempt
            wait = self.socket_timeout or None
            if deadline is not None:
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TimeoutError(f"S3 {method} {path}: request timeout ({self.timeout}s) exceeded")
                wait = min(wait, left) if wait else left
            err = None
            try:
                r = self.session.request(method, url, params=query or None, data=data or None, headers=h,
                                         timeout=(min(self.connect_timeout, wait) if wait else self.connect_timeout,
                                                  wait))
            except (requests.ConnectionError, requests.Timeout) as e:
                r, err = None, e
            if r is not None and r.status_code in ok:
                return r
            if r is not None and r.status_code == 404:
                raise FileNotFoundError(f"s3://{bucket}/{key}")
            retry = r is None or r.status_code in RETRYABLE_STATUS
            if not retry or attempt >= self.max_retries:
                if r is None:
                    kind = TimeoutError if isinstance(err, requests.Timeout) else ConnectionError
                    raise kind(f"S3 {method} {path} failed after {attempt} retries: {err}") from err
                raise OSError(f"S3 {method} {path} failed: {r.status_code} {r.text[:200]}")
            attempt += 1
            self.retries += 1
            cap = min(self.backoff_max, self.backoff_base * (2 ** (attempt - 1)))
            pause = cap / 2 + random.random() * cap / 2
            if deadline is not None:
                pause = min(pause, max(0.0, deadline - time.monotonic()))
            time.sleep(pause)


def _parse_size(v) -> int:
    v = str(v).strip().upper().rstrip("B")
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    if v and v[-1] in mult:
        return int(float(v[:-1]) * mult[v[-1]])
    return int(v or 0)


def _xml_text(el, tag):
    for c in el:
        if c.tag.split("}")[-1] == tag:
            return c.text or ""
    return ""


class S3UnderFileSystem(ObjectUnderFileSystem):
    scheme = "s3"
    ufs_type = "s3"
    multipart_threshold = 64 << 20
    part_size = 16 << 20

    def __init__(self, root_uri, conf=None, properties=None):
        super().__init__(root_uri, conf, properties)
        p = dict(properties or {})

        def opt(*names, default=""):
            for n in names:
                if n in p:
                    return p[n]
                if conf is not None and conf.get_raw(n) is not None:
                    return conf.get(n)
            return default
        rest = root_uri.split("://", 1)[1]
        self.bucket = rest.split("/", 1)[0]
        endpoint = opt("alluxio.underfs.s3.endpoint", "fs.s3a.endpoint", default="")
        if not endpoint:
            endpoint = "https://s3.amazonaws.com"
        if not endpoint.startswith("http"):
            endpoint = "http://" + endpoint
        from ..utils.format import parse_time_size

        def ms(*names, default):
            v = opt(*names, default=default)
            return parse_time_size(str(v)) if v not in (None, "") else 0
        # the reference client's limits (S3AUnderFileSystem.java:150-191, PropertyKey.java:946-1002)
        self.socket_timeout_ms = ms("alluxio.underfs.s3.socket.timeout", "alluxio.underfs.s3a.socket.timeout.ms",
                                    "alluxio.underfs.s3a.socket.timeout", default="50sec")
        self.request_timeout_ms = ms("alluxio.underfs.s3.request.timeout", "alluxio.underfs.s3a.request.timeout.ms",
                                     "alluxio.underfs.s3a.request.timeout", default="1min")
        retry = opt("alluxio.underfs.s3.max.error.retry", "alluxio.underfs.s3a.max.error.retry", default="")
        self.max_retries = int(retry) if str(retry).strip() else 3          # AWS SDK default
        self.connect_timeout_ms = min(10_000, self.socket_timeout_ms or 10_000)
        self.client = S3Client(endpoint, opt("s3a.accessKeyId", "aws.accessKeyId"),
                               opt("s3a.secretKey", "aws.secretKey"),
                               opt("alluxio.underfs.s3.region", default="us-east-1"),
                               timeout=self.request_timeout_ms / 1000.0,
                               socket_timeout=self.socket_timeout_ms / 1000.0,
                               connect_timeout=self.connect_timeout_ms / 1000.0, max_retries=self.max_retries)
        self.folder_suffix = opt("alluxio.underfs.s3.directory.suffix", default="/") or "/"
        # native data path (csrc/http_blob.cpp): ranged GETs received straight into the caller's
        # buffer over pooled keep-alive connections, a read split into parallel sub-ranges
        self._native = None
        self._native_on = str(opt("alluxio.underfs.s3.native.reader.enabled", default="true")).lower() == "true" \
            and endpoint.startswith("http://")
        self._parallel = max(1, min(16, int(opt("alluxio.underfs.s3.threads.max", default="8") or 8)))
        self._part = _parse_size(opt("alluxio.underfs.s3.read.part.size", default="4MB"))

    multipart = True

    def _put(self, key, data):
        """One PUT (objects written through create() larger than a part go multipart)."""
        if len(data) <= self.multipart_threshold:
            self.client.request("PUT", self.bucket, key, data=data)
            return
        w = self.create(key)
        try:
            w.write(data)
        except BaseException:
            w.cancel()
            raise
        w.close()

    def _put_single(self, key, data):
        self.client.request("PUT", self.bucket, key, data=data)

    # ---- multipart upload (the streaming writer of object_store._MultipartWriter) ------------
    def _mp_init(self, key):
        r = self.client.request("POST", self.bucket, key, query={"uploads": ""})
        return _xml_text(ET.fromstring(r.content), "UploadId")

    def _mp_put_part(self, key, upload_id, num, buf, n):
        """UploadPart of ``buf[:n]``: native PUT straight from the buffer over a pooled
        connection (GIL released), else ``requests``."""
        query = {"partNumber": num, "uploadId": upload_id}
        rd = self._native_reader()
        if rd is not None:
            import numpy as np
            path = f"/{self.bucket}/{key}"
            h = self.client._headers("PUT", path, query, "UNSIGNED-PAYLOAD")
            head = "".join(f"{k}: {v}\r\n" for k, v in h.items())
            target = urllib.parse.quote(path, safe="/-_.~") + "?" + "&".join(
                f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(str(v), safe='-_.~')}"
                for k, v in sorted(query.items()))
            addr = (buf.ctypes.data if isinstance(buf, np.ndarray) else
                    np.frombuffer(buf, dtype=np.uint8, count=n).ctypes.data) if n else 0
            code, etag = rd.put_from(target, head, addr, n)
            if code == 404:
                raise FileNotFoundError(f"s3://{self.bucket}/{key} upload {upload_id}")
            if code not in (200, 204):
                raise OSError(f"S3 UploadPart {num} of {path} failed: {code}")
            return etag
        rr = self.client.request("PUT", self.bucket, key, query=query, data=bytes(memoryview(buf)[:n]))
        return rr.headers.get("ETag", "")

    def _mp_complete(self, key, upload_id, parts):
        body = "<CompleteMultipartUpload>" + "".join(
            f"<Part><PartNumber>{n}</PartNumber><ETag>{e}</ETag></Part>" for n, e in parts) + \
            "</CompleteMultipartUpload>"
        self.client.request("POST", self.bucket, key, query={"uploadId": upload_id}, data=body.encode())

    def _mp_abort(self, key, upload_id):
        try:
            self.client.request("DELETE", self.bucket, key, query={"uploadId": upload_id})
        except FileNotFoundError:
            pass          # already completed or aborted

    def _mp_list(self, prefix):
        r = self.client.request("GET", self.bucket, query={"uploads": "", "prefix": prefix})
        out = []
        for el in ET.fromstring(r.content):
            if el.tag.split("}")[-1] != "Upload":
                continue
            t = _xml_text(el, "Initiated")
            try:
                ms = int(datetime.datetime.strptime(t[:19], "%Y-%m-%dT%H:%M:%S").replace(
                    tzinfo=datetime.timezone.utc).timestamp() * 1000)
            except ValueError:
                ms = 0
            out.append((_xml_text(el, "Key"), _xml_text(el, "UploadId"), ms))
        return out

    def _get_range(self, key, offset, length):
        if length <= 0:
            return b""
        r = self.client.request("GET", self.bucket, key, headers={"Range": f"bytes={offset}-{offset + length - 1}"})
        return r.content

    def _native_reader(self):
        if self._native is None and self._native_on:
            try:
                from ..ops.native import lib
                u = urllib.parse.urlsplit(self.client.endpoint)
                self._native = lib().HttpRangeReader(u.hostname, u.port or 80, 2 * self._parallel,
                                                     **self.http_limits())
            except Exception:  # noqa: BLE001 -- no native library: the requests path serves
                self._native_on = False
        return self._native

    def http_limits(self) -> dict:
        """Timeouts and retries of the native client (csrc/http_blob.cpp HttpOptions)."""
        return {"connect_timeout_ms": self.connect_timeout_ms, "socket_timeout_ms": self.socket_timeout_ms,
                "request_timeout_ms": self.request_timeout_ms, "max_retries": self.max_retries}

    def _get_into(self, key, offset, length, addr) -> bool:
        """Ranged GET of ``length`` bytes at ``offset`` into host memory at ``addr`` (native path);
        False when the native reader is unavailable."""
        rd = self._native_reader()
        if rd is None:
            return False
        path = f"/{self.bucket}/{key}"
        h = self.client._headers("GET", path, {}, _EMPTY_SHA)
        head = "".join(f"{k}: {v}\r\n" for k, v in h.items())
        got = rd.get_into(urllib.parse.quote(path, safe="/-_.~"), head, offset, length, addr,
                          self._parallel, self._part)
        if got == -404:
            raise FileNotFoundError(f"s3://{self.bucket}/{key}")
        if got == -2:
            raise TimeoutError(f"S3 GET {path} [{offset}, +{length}) timed out")
        if got != length:
            raise OSError(f"S3 GET {path} [{offset}, +{length}) failed after retries: {got}")
        return True

    def _head(self, key):
        try:
            r = self.client.request("HEAD", self.bucket, key)
        except FileNotFoundError:
            return None
        lm = r.headers.get("Last-Modified")
        mtime = None
        if lm:
            try:
                mtime = int(datetime.datetime.strptime(lm, "%a, %d %b %Y %H:%M:%S %Z").timestamp() * 1000)
            except ValueError:
                mtime = None
        return ObjectMeta(key, int(r.headers.get("Content-Length", 0)), r.headers.get("ETag", "").strip('"'), mtime)

    def _delete(self, keys):
        keys = [k for k in keys if k]
        for i in range(0, len(keys), 1000):
            batch = keys[i:i + 1000]
            body = "<Delete><Quiet>true</Quiet>" + "".join(f"<Object><Key>{k}</Key></Object>" for k in batch) + "</Delete>"
            try:
                self.client.request("POST", self.bucket, query={"delete": ""}, data=body.encode())
            except OSError:
                for k in batch:  # endpoints without multi-object delete
                    try:
                        self.client.request("DELETE", self.bucket, k)
                    except FileNotFoundError:
                        pass

    def _list(self, prefix, delimiter):
        objs, prefixes, token = [], [], None
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if delimiter:
                q["delimiter"] = delimiter
            if token:
                q["continuation-token"] = token
            r = self.client.request("GET", self.bucket, query=q)
            root = ET.fromstring(r.content)
            for el in root:
                tag = el.tag.split("}")[-1]
                if tag == "Contents":
                    objs.append(ObjectMeta(_xml_text(el, "Key"), int(_xml_text(el, "Size") or 0),
                                           _xml_text(el, "ETag").strip('"')))
                elif tag == "CommonPrefixes":
                    prefixes.append(_xml_text(el, "Prefix"))
            if _xml_text(root, "IsTruncated").lower() == "true":
                token = _xml_text(root, "NextContinuationToken")
            else:
                return objs, prefixes

    def _copy(self, src, dst):
        self.client.request("PUT", self.bucket, dst, headers={"x-amz-copy-source": f"/{self.bucket}/{src}"})


class _S3Factory(UnderFileSystemFactory):
    def __init__(self, scheme):
        self.scheme = scheme

    def create(self, uri, conf=None, properties=None):
        u = S3UnderFileSystem(uri, conf, properties)
        u.scheme = self.scheme
        u.ufs_type = self.scheme
        return u


for _s in ("s3", "s3a", "gs", "oss", "cosn", "kodo"):
    register_factory(_S3Factory(_s))
