"""Proxy process: S3-compatible REST API, the ``/api/v1/paths`` and ``/api/v1/streams`` REST APIs,
and a WebHDFS gateway on ``/webhdfs/v1`` for Hadoop clients (:mod:`alluxio_amd.proxy.webhdfs`).

Parity: core/server/proxy/src/main/java/alluxio/proxy/s3/S3RestServiceHandler.java:72-380
(bucket = top-level directory; GET/PUT/HEAD/DELETE object, copy via ``x-amz-copy-source``,
ranged GET, ListObjects v1/v2 with prefix/delimiter/max-keys/marker/continuation-token,
multi-object delete, multipart upload initiate/upload-part/list-parts/complete/abort with parts
staged under a hidden per-upload directory), PathsRestServiceHandler.java (``/api/v1/paths/<path>/
{create-directory, create-file, delete, download-file, exists, free, get-status, list-status,
mount, open-file, rename, set-attribute, unmount}``) and StreamsRestServiceHandler.java
(``/api/v1/streams/<id>/{read, write, close}``).  Everything goes through the regular client
``FileSystem``, so S3 PUT/GET land in (and are served from) the workers' HBM tier.
"""
from __future__ import annotations

import hashlib
import itertools
import json
import logging
import threading
import time
import uuid
import xml.etree.ElementTree as ET
from email.utils import formatdate
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, unquote, urlparse

from ..utils.exceptions import AlluxioStatusException, NotFoundException

LOG = logging.getLogger(__name__)
S3_NS = "http://s3.amazonaws.com/doc/2006-03-01/"
S3_PREFIX = "/api/v1/s3"
MULTIPART_DIR = ".alluxio_s3_api_multipart"


def _xml(root_tag: str, children) -> bytes:
    root = ET.Element(root_tag, xmlns=S3_NS)

    def add(parent, items):
        for k, v in items:
            el = ET.SubElement(parent, k)
            if isinstance(v, list):
                add(el, v)
            elif v is not None:
                el.text = str(v)
    add(root, children)
    return b'<?xml version="1.0" encoding="UTF-8"?>' + ET.tostring(root)


class S3Error(Exception):
    def __init__(self, status: int, code: str, msg: str, resource: str = ""):
        super().__init__(msg)
        self.status, self.code, self.msg, self.resource = status, code, msg, resource

    def body(self) -> bytes:
        return _xml("Error", [("Code", self.code), ("Message", self.msg), ("Resource", self.resource)])


def _etag(st) -> str:
    return hashlib.md5(f"{st.info.fileId}:{st.info.length}:{st.info.lastModificationTimeMs}".encode()).hexdigest()


def _http_date(ms: int) -> str:
    return formatdate(ms / 1000.0, usegmt=True)


def _iso(ms: int) -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%S.000Z", time.gmtime(ms / 1000.0))


class _Md5Beside:
    """The ETag MD5 of an uploaded body, computed on a helper thread while the chunks are written
    into Alluxio (hashlib drops the GIL on large updates), so a PUT takes max(MD5, write) rather
    than their sum.  MD5 itself is serial, ~0.7 GB/s per object."""

    def __init__(self):
        import queue
        self._md5 = hashlib.md5()
        self._q: queue.Queue = queue.Queue(maxsize=4)
        self._t = None

    def _run(self):
        while True:
            c = self._q.get()
            if c is None:
                return
            self._md5.update(c)

    def chunks(self, body_iter):
        self._t = threading.Thread(target=self._run, name="s3-md5", daemon=True)
        self._t.start()
        try:
            for c in body_iter:
                self._q.put(c)          # rfile.read returns a fresh bytes object per chunk
                yield c
        finally:
            self._q.put(None)

    def hexdigest(self) -> str:
        if self._t is not None:
            self._t.join()
        return self._md5.hexdigest()


class S3Handler:
    """S3 semantics over an Alluxio FileSystem client."""

    def __init__(self, fs, write_type: str = "CACHE_THROUGH"):
        self.fs = fs
        self.write_type = write_type
        self._copy_lock = threading.Lock()

    # ---- helpers ------------------------------------------------------------------------------
    def _bucket_path(self, bucket: str) -> str:
        if not bucket or "/" in bucket:
            raise S3Error(400, "InvalidBucketName", f"invalid bucket name {bucket!r}", bucket)
        return "/" + bucket

    def _check_bucket(self, bucket: str) -> str:
        p = self._bucket_path(bucket)
        try:
            if not self.fs.get_status(p).is_folder:
                raise S3Error(404, "NoSuchBucket", "The specified bucket does not exist", bucket)
        except NotFoundException:
            raise S3Error(404, "NoSuchBucket", "The specified bucket does not exist", bucket) from None
        return p

    def _write(self, path: str, chunks) -> None:
        try:
            if self.fs.exists(path):
                self.fs.delete(path)
        except AlluxioStatusException:
            pass
        with self.fs.create_file(path, write_type=self.write_type, recursive=True) as f:
            for c in chunks:
                f.write(c)

    # ---- service / bucket ---------------------------------------------------------------------
    def list_buckets(self):
        items = []
        for s in self.fs.list_status("/"):
            if s.is_folder:
                items.append(("Bucket", [("Name", s.name), ("CreationDate", _iso(s.info.creationTimeMs))]))
        return 200, {}, _xml("ListAllMyBucketsResult", [("Owner", [("ID", "alluxio"), ("DisplayName", "alluxio")]),
                                                        ("Buckets", items)])

    def create_bucket(self, bucket):
        p = self._bucket_path(bucket)
        if self.fs.exists(p):
            raise S3Error(409, "BucketAlreadyExists", "The requested bucket name is not available", bucket)
        self.fs.create_directory(p, write_type=self.write_type)
        return 200, {"Location": "/" + bucket}, b""

    def delete_bucket(self, bucket):
        p = self._check_bucket(bucket)
        kids = [s for s in self.fs.list_status(p) if s.name != MULTIPART_DIR]
        if kids:
            raise S3Error(409, "BucketNotEmpty", "The bucket you tried to delete is not empty", bucket)
        self.fs.delete(p, recursive=True)
        return 204, {}, b""

    def list_objects(self, bucket, q):
        p = self._check_bucket(bucket)
        prefix = q.get("prefix", "")
        delim = q.get("delimiter", "")
        max_keys = int(q.get("max-keys", 1000))
        v2 = q.get("list-type") == "2"
        after = q.get("continuation-token") or q.get("start-after") or q.get("marker") or ""
        entries = []
        for s in self.fs.list_status(p, recursive=True):
            key = s.path[len(p) + 1:]
            if key.split("/", 1)[0] == MULTIPART_DIR:
                continue
            if s.is_folder:
                key += "/"   # directories list as zero-byte "dir/" marker objects
            if key.startswith(prefix):
                entries.append((key, s))
        entries.sort(key=lambda e: e[0])
        contents, prefixes, seen = [], [], set()
        truncated, last = False, ""
        for key, s in entries:
            if key <= after:
                continue
            if delim:
                rest = key[len(prefix):]
                i = rest.find(delim)
                if i >= 0:
                    cp = prefix + rest[:i + len(delim)]
                    if cp not in seen:
                        if len(contents) + len(prefixes) >= max_keys:
                            truncated = True
                            break
                        seen.add(cp)
                        prefixes.append(cp)
                        last = cp
                    continue
            if len(contents) + len(prefixes) >= max_keys:
                truncated = True
                break
            contents.append(("Contents", [("Key", key), ("LastModified", _iso(s.info.lastModificationTimeMs)),
                                          ("ETag", f'"{_etag(s)}"'), ("Size", 0 if s.is_folder else s.length),
                                          ("StorageClass", "STANDARD")]))
            last = key
        body = [("Name", bucket), ("Prefix", prefix), ("MaxKeys", max_keys), ("IsTruncated", str(truncated).lower())]
        if delim:
            body.append(("Delimiter", delim))
        if v2:
            body.append(("KeyCount", len(contents) + len(prefixes)))
            if q.get("continuation-token"):
                body.append(("ContinuationToken", q["continuation-token"]))
            if truncated:
                body.append(("NextContinuationToken", last))
        else:
            body.append(("Marker", q.get("marker", "")))
            if truncated:
                body.append(("NextMarker", last))
        body += contents
        body += [("CommonPrefixes", [("Prefix", cp)]) for cp in prefixes]
        return 200, {}, _xml("ListBucketResult", body)

    def multi_delete(self, bucket, body: bytes):
        p = self._check_bucket(bucket)
        root = ET.fromstring(body)
        deleted, errors = [], []
        for obj in root.iter():
            if obj.tag.split("}")[-1] != "Object":
                continue
            key = next((c.text for c in obj if c.tag.split("}")[-1] == "Key"), None)
            if not key:
                continue
            try:
                self._delete_key(p, key)
                deleted.append(("Deleted", [("Key", key)]))
            except NotFoundException:
                deleted.append(("Deleted", [("Key", key)]))
            except AlluxioStatusException as e:
                errors.append(("Error", [("Key", key), ("Code", "InternalError"), ("Message", str(e))]))
        return 200, {}, _xml("DeleteResult", deleted + errors)

    # ---- objects ------------------------------------------------------------------------------
    def put_object(self, bucket, key, headers, body_iter):
        p = self._check_bucket(bucket)
        path = f"{p}/{key}"
        src = headers.get("x-amz-copy-source")
        if key.endswith("/"):
            self.fs.create_directory(path.rstrip("/"), recursive=True, allow_exists=True,
                                     write_type=self.write_type)
            return 200, {"ETag": '""'}, b""
        if src:
            src = unquote(src).lstrip("/")
            sb, _, sk = src.partition("/")
            sp = f"{self._check_bucket(sb)}/{sk}"
            try:
                with self.fs.open_file(sp) as fin:
                    self._write(path, iter(lambda: fin.read(8 << 20), b""))
            except NotFoundException:
                raise S3Error(404, "NoSuchKey", "The specified key does not exist.", src) from None
            st = self.fs.get_status(path)
            return 200, {}, _xml("CopyObjectResult", [("LastModified", _iso(st.info.lastModificationTimeMs)),
                                                      ("ETag", f'"{_etag(st)}"')])
        md5 = _Md5Beside()
        self._write(path, md5.chunks(body_iter))
        return 200, {"ETag": f'"{md5.hexdigest()}"'}, b""

    def _stat_object(self, bucket, key):
        p = self._check_bucket(bucket)
        try:
            st = self.fs.get_status(f"{p}/{key}".rstrip("/"))
        except NotFoundException:
            raise S3Error(404, "NoSuchKey", "The specified key does not exist.", key) from None
        if st.is_folder and not key.endswith("/"):
            raise S3Error(404, "NoSuchKey", "The specified key does not exist.", key)
        return st

    def head_object(self, bucket, key):
        st = self._stat_object(bucket, key)
        return 200, {"Content-Length": str(0 if st.is_folder else st.length), "ETag": f'"{_etag(st)}"',
                     "Last-Modified": _http_date(st.info.lastModificationTimeMs),
                     "Content-Type": "application/octet-stream"}, None

    def get_object(self, bucket, key, headers):
        st = self._stat_object(bucket, key)
        n = 0 if st.is_folder else st.length
        start, end, status = 0, n - 1, 200
        rng = headers.get("Range") or headers.get("range")
        if rng and rng.startswith("bytes=") and n > 0:
            a, _, b = rng[6:].partition("-")
            if a == "":
                start, end = max(0, n - int(b)), n - 1
            else:
                start, end = int(a), min(n - 1, int(b)) if b else n - 1
            if start >= n:
                raise S3Error(416, "InvalidRange", "The requested range is not satisfiable", key)
            status = 206
        length = max(0, end - start + 1)
        data = b""
        h = {"ETag": f'"{_etag(st)}"', "Last-Modified": _http_date(st.info.lastModificationTimeMs),
             "Content-Type": "application/octet-stream", "Accept-Ranges": "bytes"}
        if length > self.STREAM_CHUNK:
            # large objects stream through one reused buffer (native reader refills, one sendall
            # per chunk) instead of being read whole into memory first
            h["Content-Length"] = str(length)
            data = self._stream(st, start, length)
        elif length:
            with self.fs.open_file(st.path, status=st) as f:
                f.seek(start)
                data = f.read(length)
        if status == 206:
            h["Content-Range"] = f"bytes {start}-{end}/{n}"
        return status, h, data

    STREAM_CHUNK = 8 << 20

    def _stream(self, st, start: int, length: int):
        f = self.fs.open_file(st.path, status=st)
        try:
            f.seek(start)
            buf = bytearray(self.STREAM_CHUNK)
            mv = memoryview(buf)
            left = length
            while left > 0:
                n = f.readinto(mv[:min(len(buf), left)])
                if not n:
                    raise IOError(f"{st.path}: object ended {left} bytes early")
                yield mv[:n]          # written out (sendall) before the buffer is reused
                left -= n
        finally:
            f.close()

    def _delete_key(self, bucket_path, key):
        path = f"{bucket_path}/{key}".rstrip("/")
        st = self.fs.get_status(path)
        self.fs.delete(path, recursive=st.is_folder)

    def delete_object(self, bucket, key):
        p = self._check_bucket(bucket)
        try:
            self._delete_key(p, key)
        except NotFoundException:
            pass  # S3 DELETE is idempotent
        return 204, {}, b""

    # ---- multipart ----------------------------------------------------------------------------
    def _mp_dir(self, bucket_path, key, upload_id):
        return f"{bucket_path}/{MULTIPART_DIR}/{key.replace('/', '_')}_{upload_id}"

    def initiate_multipart(self, bucket, key):
        p = self._check_bucket(bucket)
        uid = uuid.uuid4().hex
        self.fs.create_directory(self._mp_dir(p, key, uid), recursive=True, write_type="MUST_CACHE")
        return 200, {}, _xml("InitiateMultipartUploadResult", [("Bucket", bucket), ("Key", key), ("UploadId", uid)])

    def upload_part(self, bucket, key, upload_id, part: int, body_iter):
        p = self._check_bucket(bucket)
        d = self._mp_dir(p, key, upload_id)
        if not self.fs.exists(d):
            raise S3Error(404, "NoSuchUpload", "The specified upload does not exist.", key)
        md5 = _Md5Beside()
        self._write(f"{d}/{part:05d}", md5.chunks(body_iter))
        return 200, {"ETag": f'"{md5.hexdigest()}"'}, b""

    def list_parts(self, bucket, key, upload_id):
        p = self._check_bucket(bucket)
        d = self._mp_dir(p, key, upload_id)
        try:
            parts = sorted(self.fs.list_status(d), key=lambda s: s.name)
        except NotFoundException:
            raise S3Error(404, "NoSuchUpload", "The specified upload does not exist.", key) from None
        items = [("Part", [("PartNumber", int(s.name)), ("LastModified", _iso(s.info.lastModificationTimeMs)),
                           ("ETag", f'"{_etag(s)}"'), ("Size", s.length)]) for s in parts]
        return 200, {}, _xml("ListPartsResult", [("Bucket", bucket), ("Key", key), ("UploadId", upload_id)] + items)

    def complete_multipart(self, bucket, key, upload_id, body: bytes):
        p = self._check_bucket(bucket)
        d = self._mp_dir(p, key, upload_id)
        if not self.fs.exists(d):
            raise S3Error(404, "NoSuchUpload", "The specified upload does not exist.", key)
        wanted = []
        if body:
            for el in ET.fromstring(body).iter():
                if el.tag.split("}")[-1] == "PartNumber":
                    wanted.append(int(el.text))
        have = {int(s.name): s for s in self.fs.list_status(d)}
        order = wanted or sorted(have)
        for n in order:
            if n not in have:
                raise S3Error(400, "InvalidPart", f"part {n} was not uploaded", key)

        def chunks():
            for n in order:
                with self.fs.open_file(have[n].path) as f:
                    while True:
                        c = f.read(8 << 20)
                        if not c:
                            break
                        yield c
        self._write(f"{p}/{key}", chunks())
        self.fs.delete(d, recursive=True)
        st = self.fs.get_status(f"{p}/{key}")
        return 200, {}, _xml("CompleteMultipartUploadResult", [("Location", f"/{bucket}/{key}"), ("Bucket", bucket),
                                                               ("Key", key), ("ETag", f'"{_etag(st)}"')])

    def abort_multipart(self, bucket, key, upload_id):
        p = self._check_bucket(bucket)
        d = self._mp_dir(p, key, upload_id)
        if not self.fs.exists(d):
            raise S3Error(404, "NoSuchUpload", "The specified upload does not exist.", key)
        self.fs.delete(d, recursive=True)
        return 204, {}, b""


class PathsStreams:
    """``/api/v1/paths`` + ``/api/v1/streams`` JSON APIs."""

    def __init__(self, fs):
        self.fs = fs
        self.streams: dict[int, object] = {}
        self._ids = itertools.count(1)
        self._lock = threading.Lock()

    def _status_json(self, s):
        i = s.info
        return {"path": i.path, "name": i.name, "length": i.length, "folder": i.folder, "completed": i.completed,
                "fileId": i.fileId, "blockSizeBytes": i.blockSizeBytes, "owner": i.owner, "group": i.group,
                "mode": i.mode, "persisted": i.persisted, "inAlluxioPercentage": i.inAlluxioPercentage,
                "lastModificationTimeMs": i.lastModificationTimeMs, "ufsPath": i.ufsPath, "pinned": i.pinned}

    def paths(self, path: str, op: str, q: dict, body: bytes):
        opts = json.loads(body) if body and body.strip().startswith(b"{") else {}
        fs = self.fs
        if op == "create-directory":
            fs.create_directory(path, recursive=opts.get("recursive", False),
                                allow_exists=opts.get("allowExists", False), write_type=opts.get("writeType"))
            return None
        if op == "create-file":
            f = fs.create_file(path, write_type=opts.get("writeType"), block_size=opts.get("blockSizeBytes"),
                               recursive=opts.get("recursive", True))
            return self._register(f)
        if op == "delete":
            fs.delete(path, recursive=opts.get("recursive", False), alluxio_only=opts.get("alluxioOnly", False))
            return None
        if op == "download-file":
            return fs.read_file(path)
        if op == "exists":
            return fs.exists(path)
        if op == "free":
            fs.free(path, recursive=opts.get("recursive", False))
            return None
        if op == "get-status":
            return self._status_json(fs.get_status(path))
        if op == "list-status":
            return [self._status_json(s) for s in fs.list_status(path, recursive=opts.get("recursive", False))]
        if op == "mount":
            fs.mount(path, q["src"], read_only=opts.get("readOnly", False), shared=opts.get("shared", False),
                     properties=opts.get("properties"))
            return None
        if op == "open-file":
            return self._register(fs.open_file(path, read_type=opts.get("readType")))
        if op == "rename":
            fs.rename(path, q["dst"])
            return None
        if op == "set-attribute":
            fs.set_attribute(path, pinned=opts.get("pinned"), ttl=opts.get("ttl"), owner=opts.get("owner"),
                             group=opts.get("group"), mode=opts.get("mode"),
                             recursive=opts.get("recursive", False))
            return None
        if op == "unmount":
            fs.unmount(path)
            return None
        raise S3Error(404, "NoSuchOperation", f"unknown paths operation {op}")

    def _register(self, stream) -> int:
        with self._lock:
            sid = next(self._ids)
            self.streams[sid] = stream
            return sid

    def stream_op(self, sid: int, op: str, body: bytes):
        with self._lock:
            s = self.streams.get(sid)
        if s is None:
            raise S3Error(404, "NoSuchStream", f"stream {sid} does not exist")
        if op == "read":
            return s.read()
        if op == "write":
            s.write(body)
            return len(body)
        if op == "close":
            s.close()
            with self._lock:
                self.streams.pop(sid, None)
            return None
        raise S3Error(404, "NoSuchOperation", f"unknown stream operation {op}")


class ProxyServer:
    def advertised_address(self) -> str:
        """host:port redirects point at: ``alluxio.proxy.web.hostname`` when configured, else the
        bound address (the machine's hostname for a wildcard bind)."""
        import socket
        conf = getattr(self.s3.fs.ctx, "conf", None)
        name = conf.get_raw("alluxio.proxy.web.hostname") if conf is not None else None
        if not name:
            name = self.httpd.server_address[0]
            if name in ("0.0.0.0", "", "::"):
                name = socket.gethostname()
        return f"{name}:{self.port}"

    def __init__(self, fs, host: str = "127.0.0.1", port: int = 0, write_type: str = "CACHE_THROUGH"):
        from .webhdfs import WebHdfsGateway
        self.s3 = S3Handler(fs, write_type)
        self.api = PathsStreams(fs)
        self.webhdfs = WebHdfsGateway(fs, write_type)
        outer = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, fmt, *args):
                LOG.debug("proxy " + fmt, *args)

            def _body_iter(self):
                if self.headers.get("Transfer-Encoding", "").lower() == "chunked":
                    while True:
                        size = int(self.rfile.readline().strip().split(b";")[0], 16)
                        if size == 0:
                            self.rfile.readline()
                            return
                        data = self.rfile.read(size)
                        self.rfile.readline()
                        yield data
                n = int(self.headers.get("Content-Length") or 0)
                while n > 0:
                    c = self.rfile.read(min(n, 8 << 20))
                    if not c:
                        return
                    n -= len(c)
                    yield c

            def _reply(self, status, headers, body):
                self.send_response(status)
                for k, v in headers.items():
                    self.send_header(k, v)
                if body is None:  # HEAD: Content-Length already describes the object
                    self.end_headers()
                    return
                if not isinstance(body, (bytes, bytearray)):   # streamed (Content-Length given)
                    self.end_headers()
                    for chunk in body:
                        self.wfile.write(chunk)
                    return
                if "Content-Type" not in headers:
                    self.send_header("Content-Type", "application/xml")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _handle(self, method):
                u = urlparse(self.path)
                q = {k: v[-1] for k, v in parse_qs(u.query, keep_blank_values=True).items()}
                path = unquote(u.path)
                if path == "/webhdfs/v1" or path.startswith("/webhdfs/v1/"):
                    # redirects name this proxy, never the client-supplied Host header (an
                    # open redirect that would send CREATE data anywhere)
                    host = outer.advertised_address()
                    target = "/" + path[len("/webhdfs/v1"):].lstrip("/")
                    status, headers, body = outer.webhdfs.handle(method, target, q, host, self._body_iter)
                    if method == "HEAD":
                        body = None
                    return self._reply(status, headers, body)
                try:
                    if path.startswith("/api/v1/paths/") or path.startswith("/api/v1/streams/"):
                        return self._rest(method, path, q)
                    if path.startswith(S3_PREFIX):
                        path = path[len(S3_PREFIX):]
                    status, headers, body = outer._s3(method, path, q, self.headers, self._body_iter)
                except S3Error as e:
                    status, headers, body = e.status, {}, e.body()
                except NotFoundException as e:
                    status, headers, body = 404, {}, S3Error(404, "NoSuchKey", str(e)).body()
                except AlluxioStatusException as e:
                    status, headers, body = 500, {}, S3Error(500, "InternalError", str(e)).body()
                except Exception as e:  # noqa: BLE001
                    LOG.exception("proxy request failed")
                    status, headers, body = 500, {}, S3Error(500, "InternalError", str(e)).body()
                if method == "HEAD":  # never a body on HEAD, even for errors
                    headers.setdefault("Content-Length", "0")
                    body = None
                self._reply(status, headers, body)

            def _rest(self, method, path, q):
                body = b"".join(self._body_iter())
                try:
                    if path.startswith("/api/v1/paths/"):
                        rest = path[len("/api/v1/paths/"):].rstrip("/")
                        target, _, op = rest.rpartition("/")
                        out = outer.api.paths("/" + target.lstrip("/"), op, q, body)
                    else:
                        sid, _, op = path[len("/api/v1/streams/"):].rstrip("/").partition("/")
                        out = outer.api.stream_op(int(sid), op, body)
                    if isinstance(out, (bytes, bytearray)):
                        self._reply(200, {"Content-Type": "application/octet-stream"}, bytes(out))
                    else:
                        self._reply(200, {"Content-Type": "application/json"}, json.dumps(out).encode())
                except (AlluxioStatusException, S3Error) as e:
                    code = 404 if isinstance(e, NotFoundException) else getattr(e, "status", 500)
                    self._reply(code, {"Content-Type": "application/json"}, json.dumps({"error": str(e)}).encode())

            def do_GET(self):
                self._handle("GET")

            def do_PUT(self):
                self._handle("PUT")

            def do_POST(self):
                self._handle("POST")

            def do_DELETE(self):
                self._handle("DELETE")

            def do_HEAD(self):
                self._handle("HEAD")

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True

    def _s3(self, method, path, q, headers, body_iter):
        parts = path.lstrip("/").split("/", 1)
        bucket = parts[0]
        key = parts[1] if len(parts) > 1 else ""
        s3 = self.s3
        if not bucket:
            if method == "GET":
                return s3.list_buckets()
            raise S3Error(405, "MethodNotAllowed", "method not allowed on service")
        if not key:
            if method == "PUT":
                return s3.create_bucket(bucket)
            if method == "DELETE":
                return s3.delete_bucket(bucket)
            if method == "GET":
                return s3.list_objects(bucket, q)
            if method == "HEAD":
                s3._check_bucket(bucket)
                return 200, {}, None
            if method == "POST" and "delete" in q:
                return s3.multi_delete(bucket, b"".join(body_iter()))
            raise S3Error(405, "MethodNotAllowed", f"{method} not allowed on a bucket")
        if method == "PUT":
            if "uploadId" in q:
                return s3.upload_part(bucket, key, q["uploadId"], int(q["partNumber"]), body_iter())
            return s3.put_object(bucket, key, headers, body_iter())
        if method == "GET":
            if "uploadId" in q:
                return s3.list_parts(bucket, key, q["uploadId"])
            return s3.get_object(bucket, key, headers)
        if method == "HEAD":
            return s3.head_object(bucket, key)
        if method == "DELETE":
            if "uploadId" in q:
                return s3.abort_multipart(bucket, key, q["uploadId"])
            return s3.delete_object(bucket, key)
        if method == "POST":
            if "uploads" in q:
                return s3.initiate_multipart(bucket, key)
            if "uploadId" in q:
                return s3.complete_multipart(bucket, key, q["uploadId"], b"".join(body_iter()))
        raise S3Error(405, "MethodNotAllowed", f"{method} not allowed on an object")

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    def start(self) -> int:
        threading.Thread(target=self.httpd.serve_forever, kwargs={"poll_interval": 0.05}, name="s3-proxy",
                         daemon=True).start()
        return self.port

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()


def main(argv=None) -> int:  # pragma: no cover - CLI entry
    import argparse
    ap = argparse.ArgumentParser(description="alluxio_amd proxy (S3 + REST)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--master", default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from ..client.file_system import FileSystem
    from ..conf import Configuration
    conf = Configuration(load_site=True)
    fs = FileSystem(conf=conf, master_address=a.master)
    port = a.port if a.port is not None else conf.get_int("alluxio.proxy.web.port")
    srv = ProxyServer(fs, a.host, port, conf.get("alluxio.proxy.s3.writetype", "CACHE_THROUGH"))
    LOG.info("proxy serving on %s:%d", a.host, srv.start())
    gw = None
    hdfs_port = conf.get_int("alluxio.proxy.hdfs.rpc.port")
    if hdfs_port >= 0:
        from .hdfs_gateway import serve
        gw = serve(fs, a.host, hdfs_port, conf.get_int("alluxio.proxy.hdfs.data.port"),
                   conf.get("alluxio.proxy.hdfs.hostname") or None)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        pass
    if gw is not None:
        gw.stop()
    srv.stop()
    return 0
