"""In-process fake storage services for UFS connector tests (no network in this image).

Each fake implements just enough of the real service's HTTP API — including its authentication —
for the connector to run its full contract against it: OpenStack Swift (tempauth + Keystone v3),
Azure Blob (SharedKey signatures are recomputed and checked) and WebHDFS (namenode redirect to a
datanode for CREATE; optional OAuth2 bearer tokens as served by ADLS Gen1).
"""
from __future__ import annotations

import json
import threading
import time
import urllib.parse
import xml.sax.saxutils as sx
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


class _Server:
    def __init__(self, handler_cls, state):
        handler_cls.state = state
        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), handler_cls)
        self.port = self.httpd.server_address[1]
        self.url = f"http://127.0.0.1:{self.port}"
        state.url = self.url
        self.t = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self.t.start()

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()


class _Base(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    state = None

    def log_message(self, *a):
        pass

    def _body(self) -> bytes:
        n = int(self.headers.get("Content-Length") or 0)
        return self.rfile.read(n) if n else b""

    def _send(self, code, body=b"", headers=None, ctype="application/octet-stream"):
        self.send_response(code)
        h = {"Content-Type": ctype}
        h.update(headers or {})
        clen = h.pop("Content-Length", None)
        for k, v in h.items():
            self.send_header(k, str(v))
        if self.command == "HEAD":
            self.send_header("Content-Length", str(clen if clen is not None else len(body)))
            self.end_headers()
            return
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _split(self):
        u = urllib.parse.urlsplit(self.path)
        q = {k: v[0] for k, v in urllib.parse.parse_qs(u.query, keep_blank_values=True).items()}
        return u.path, q

    @staticmethod
    def _range(spec, size):
        if not spec:
            return 0, size
        a, b = spec.split("=", 1)[1].split("-")
        return int(a), min(size, int(b) + 1)


# ---- Swift --------------------------------------------------------------------------------------

class SwiftState:
    def __init__(self, user="alice", tenant="proj", password="pw", container="bkt", read_acl="alice"):
        self.user, self.tenant, self.password = user, tenant, password
        self.containers = {container: {}}
        self.acl = {container: (read_acl, "")}
        self.tokens = set()
        self.auth_calls = 0
        self.lock = threading.Lock()


class _SwiftHandler(_Base):
    def _auth_ok(self):
        return self.headers.get("X-Auth-Token") in self.state.tokens

    def do_GET(self):
        path, q = self._split()
        st = self.state
        if path == "/auth/v1.0":
            st.auth_calls += 1
            if self.headers.get("X-Auth-User") == f"{st.tenant}:{st.user}" and \
                    self.headers.get("X-Auth-Key") == st.password:
                tok = f"tok{st.auth_calls}"
                st.tokens.add(tok)
                return self._send(200, headers={"X-Storage-Url": st.url + "/v1/AUTH_" + st.tenant,
                                                "X-Auth-Token": tok})
            return self._send(401)
        return self._obj("GET", path, q)

    def do_POST(self):
        path, q = self._split()
        st = self.state
        if path == "/v3/auth/tokens":
            st.auth_calls += 1
            d = json.loads(self._body())
            u = d["auth"]["identity"]["password"]["user"]
            if u["name"] != st.user or u["password"] != st.password:
                return self._send(401)
            tok = f"v3tok{st.auth_calls}"
            st.tokens.add(tok)
            body = {"token": {"catalog": [
                {"type": "identity", "endpoints": [{"interface": "public", "url": "http://x"}]},
                {"type": "object-store", "endpoints": [
                    {"interface": "public", "region": "other", "url": "http://127.0.0.1:1/v1/nope"},
                    {"interface": "public", "region": "r1", "url": st.url + "/v1/AUTH_" + st.tenant}]}]}}
            return self._send(201, json.dumps(body).encode(), {"X-Subject-Token": tok}, "application/json")
        return self._send(405)

    def do_PUT(self):
        path, q = self._split()
        return self._obj("PUT", path, q)

    def do_HEAD(self):
        path, q = self._split()
        return self._obj("HEAD", path, q)

    def do_DELETE(self):
        path, q = self._split()
        return self._obj("DELETE", path, q)

    def _obj(self, method, path, q):
        st = self.state
        if not self._auth_ok():
            self._body()
            return self._send(401)
        parts = urllib.parse.unquote(path).split("/", 4)   # '', v1, AUTH_x, container, obj
        cont = parts[3] if len(parts) > 3 else ""
        name = parts[4] if len(parts) > 4 else ""
        with st.lock:
            objs = st.containers.get(cont)
            if objs is None:
                self._body()
                return self._send(404)
            if not name:
                if method == "HEAD":
                    r, w = st.acl[cont]
                    return self._send(204, headers={"X-Container-Read": r, "X-Container-Write": w,
                                                    "Content-Length": 0})
                prefix, delim = q.get("prefix", ""), q.get("delimiter")
                marker, limit = q.get("marker", ""), int(q.get("limit", 10000))
                out, seen = [], set()
                for k in sorted(objs):
                    if not k.startswith(prefix):
                        continue
                    rest = k[len(prefix):]
                    if delim and delim in rest:
                        sd = prefix + rest.split(delim, 1)[0] + delim
                        if sd > marker and sd not in seen:
                            seen.add(sd)
                            out.append({"subdir": sd})
                    elif k > marker:
                        d, mt = objs[k]
                        out.append({"name": k, "bytes": len(d), "hash": str(hash(d) & 0xFFFF),
                                    "last_modified": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(mt))})
                    if len(out) >= limit:
                        break
                return self._send(200, json.dumps(out).encode(), ctype="application/json")
            if method == "PUT":
                src = self.headers.get("X-Copy-From")
                body = self._body()
                if src:
                    sc, so = urllib.parse.unquote(src).lstrip("/").split("/", 1)
                    if so not in st.containers[sc]:
                        return self._send(404)
                    body = st.containers[sc][so][0]
                objs[name] = (body, time.time())
                return self._send(201)
            if name not in objs:
                return self._send(404)
            d, mt = objs[name]
            if method == "DELETE":
                del objs[name]
                return self._send(204)
            hdr = {"ETag": str(hash(d) & 0xFFFF), "Last-Modified": time.strftime("%a, %d %b %Y %H:%M:%S GMT",
                                                                              time.gmtime(mt))}
            if method == "HEAD":
                hdr["Content-Length"] = len(d)
                return self._send(200, headers=hdr)
            a, b = self._range(self.headers.get("Range"), len(d))
            return self._send(206 if self.headers.get("Range") else 200, d[a:b], hdr)


def swift_server(**kw):
    st = SwiftState(**kw)
    return _Server(_SwiftHandler, st), st


# ---- Azure Blob --------------------------------------------------------------------------------

class AzureState:
    def __init__(self, account="acct", key_b64="c2VjcmV0LWtleS1mb3ItdGVzdHM=", container="cont"):
        self.account, self.key = account, key_b64
        self.blobs = {container: {}}
        self.blocks = {}
        self.bad_sigs = 0
        self.lock = threading.Lock()
        self.list_page = 3


class _AzureHandler(_Base):
    def _check(self, method, path, q):
        from alluxio_amd.underfs.wasb import shared_key_signature
        h = {k: v for k, v in self.headers.items()}
        auth = h.pop("Authorization", None)
        expect = shared_key_signature(self.state.account, self.state.key, method, path, q, h)
        if auth != expect:
            self.state.bad_sigs += 1
            return False
        return True

    def _handle(self, method):
        path, q = self._split()
        body = self._body() if method in ("PUT", "POST") else b""
        st = self.state
        if not self._check(method, path, q):
            return self._send(403)
        cont, _, name = urllib.parse.unquote(path).lstrip("/").partition("/")
        with st.lock:
            blobs = st.blobs.get(cont)
            if blobs is None:
                return self._send(404)
            if not name:
                if q.get("comp") != "list":
                    return self._send(400)
                prefix, delim, marker = q.get("prefix", ""), q.get("delimiter"), q.get("marker", "")
                items, seen = [], set()
                for k in sorted(blobs):
                    if not k.startswith(prefix):
                        continue
                    rest = k[len(prefix):]
                    if delim and delim in rest:
                        p = prefix + rest.split(delim, 1)[0] + delim
                        if p not in seen:
                            seen.add(p)
                            items.append(("p", p))
                    else:
                        items.append(("b", k))
                items = [i for i in items if i[1] > marker]
                page, more = items[:st.list_page], len(items) > st.list_page
                xs = ['<?xml version="1.0" encoding="utf-8"?><EnumerationResults><Blobs>']
                for kind, k in page:
                    if kind == "p":
                        xs.append(f"<BlobPrefix><Name>{sx.escape(k)}</Name></BlobPrefix>")
                    else:
                        d, mt = blobs[k]
                        xs.append(f"<Blob><Name>{sx.escape(k)}</Name><Properties><Content-Length>{len(d)}"
                                  f"</Content-Length><Etag>0x{hash(d) & 0xFFFF:x}</Etag><Last-Modified>"
                                  f"{time.strftime('%a, %d %b %Y %H:%M:%S GMT', time.gmtime(mt))}</Last-Modified>"
                                  f"</Properties></Blob>")
                xs.append("</Blobs>")
                xs.append(f"<NextMarker>{sx.escape(page[-1][1]) if more else ''}</NextMarker></EnumerationResults>")
                return self._send(200, "".join(xs).encode(), ctype="application/xml")
            if method == "PUT":
                comp = q.get("comp")
                if comp == "block":
                    st.blocks[(cont, name, q["blockid"])] = body
                    return self._send(201)
                if comp == "blocklist":
                    import re
                    ids = re.findall(r"<Latest>([^<]+)</Latest>", body.decode())
                    blobs[name] = (b"".join(st.blocks.pop((cont, name, i)) for i in ids), time.time())
                    return self._send(201)
                src = self.headers.get("x-ms-copy-source")
                if src:
                    sp = urllib.parse.unquote(urllib.parse.urlsplit(src).path).lstrip("/").split("/", 1)[1]
                    if sp not in blobs:
                        return self._send(404)
                    blobs[name] = (blobs[sp][0], time.time())
                    return self._send(202, headers={"x-ms-copy-status": "success"})
                if self.headers.get("x-ms-blob-type") != "BlockBlob":
                    return self._send(400)
                blobs[name] = (body, time.time())
                return self._send(201)
            if name not in blobs:
                return self._send(404)
            d, mt = blobs[name]
            if method == "DELETE":
                del blobs[name]
                return self._send(202)
            hdr = {"ETag": f"0x{hash(d) & 0xFFFF:x}",
                   "Last-Modified": time.strftime("%a, %d %b %Y %H:%M:%S GMT", time.gmtime(mt))}
            if method == "HEAD":
                hdr["Content-Length"] = len(d)
                return self._send(200, headers=hdr)
            rng = self.headers.get("x-ms-range")
            a, b = self._range(rng, len(d))
            return self._send(206 if rng else 200, d[a:b], hdr)

    def do_GET(self):
        self._handle("GET")

    def do_PUT(self):
        self._handle("PUT")

    def do_HEAD(self):
        self._handle("HEAD")

    def do_DELETE(self):
        self._handle("DELETE")


def azure_server(**kw):
    st = AzureState(**kw)
    return _Server(_AzureHandler, st), st


# ---- WebHDFS / ADL -----------------------------------------------------------------------------

class WebHdfsState:
    def __init__(self, require_token: str | None = None, client_id="cid", secret="sec"):
        self.files = {"/": {"type": "DIRECTORY", "perm": "755", "owner": "hdfs", "group": "supergroup",
                            "mtime": int(time.time() * 1000)}}
        self.require_token = require_token
        self.client_id, self.secret = client_id, secret
        self.token_requests = 0
        self.lock = threading.Lock()


class _WebHdfsHandler(_Base):
    def _auth(self):
        t = self.state.require_token
        return t is None or self.headers.get("Authorization") == f"Bearer {t}"

    def _json(self, code, obj):
        return self._send(code, json.dumps(obj).encode(), ctype="application/json")

    def _fs(self, name, e):
        d = {"pathSuffix": name, "type": e["type"], "permission": e["perm"], "owner": e["owner"],
             "group": e["group"], "modificationTime": e["mtime"], "length": len(e.get("data", b"")),
             "blockSize": 128 << 20}
        return d

    def _handle(self, method):
        path, q = self._split()
        st = self.state
        body = self._body() if method in ("PUT", "POST") else b""
        if path == "/oauth2/token":
            f = urllib.parse.parse_qs(body.decode())
            st.token_requests += 1
            if f.get("client_id") == [st.client_id] and f.get("client_secret") == [st.secret]:
                return self._json(200, {"access_token": st.require_token, "expires_in": 3600})
            return self._json(401, {})
        if path.startswith("/dn/"):
            p = "/" + urllib.parse.unquote(path[len("/dn/"):]).lstrip("/")
            with st.lock:
                st.files[p] = {"type": "FILE", "data": body, "perm": q.get("permission", "644"), "owner": "u",
                               "group": "g", "mtime": int(time.time() * 1000)}
            return self._send(201)
        if not self._auth():
            return self._send(401)
        p = "/" + urllib.parse.unquote(path[len("/webhdfs/v1"):]).strip("/")
        p = p if p != "" else "/"
        op = q.get("op")
        with st.lock:
            e = st.files.get(p)
            parent = p.rsplit("/", 1)[0] or "/"
            if op == "GETFILESTATUS":
                if e is None:
                    return self._json(404, {"RemoteException": {"exception": "FileNotFoundException"}})
                return self._json(200, {"FileStatus": self._fs("", e)})
            if op == "LISTSTATUS":
                pre = p.rstrip("/") + "/"
                kids = [(k[len(pre):], v) for k, v in sorted(st.files.items())
                        if k.startswith(pre) and "/" not in k[len(pre):] and k != p]
                return self._json(200, {"FileStatuses": {"FileStatus": [self._fs(n, v) for n, v in kids]}})
            if op == "MKDIRS":
                parts = p.strip("/").split("/")
                for i in range(1, len(parts) + 1):
                    d = "/" + "/".join(parts[:i])
                    st.files.setdefault(d, {"type": "DIRECTORY", "perm": q.get("permission", "755"), "owner": "u",
                                            "group": "g", "mtime": int(time.time() * 1000)})
                return self._json(200, {"boolean": True})
            if op == "CREATE":
                if parent not in st.files:
                    return self._json(404, {})
                if q.get("write") == "true":
                    st.files[p] = {"type": "FILE", "data": body, "perm": q.get("permission", "644"), "owner": "u",
                                   "group": "g", "mtime": int(time.time() * 1000)}
                    return self._send(201)
                loc = f"{st.url}/dn{urllib.parse.quote(p)}?permission={q.get('permission', '644')}"
                return self._send(307, headers={"Location": loc})
            if op == "OPEN":
                if e is None or e["type"] != "FILE":
                    return self._json(404, {})
                off = int(q.get("offset", 0))
                ln = int(q.get("length", len(e["data"]) - off))
                return self._send(200, e["data"][off:off + ln])
            if op == "DELETE":
                if e is None:
                    return self._json(200, {"boolean": False})
                pre = p.rstrip("/") + "/"
                kids = [k for k in st.files if k.startswith(pre)]
                if kids and q.get("recursive") != "true":
                    return self._json(403, {})
                for k in kids + [p]:
                    st.files.pop(k, None)
                return self._json(200, {"boolean": True})
            if op == "RENAME":
                dst = q["destination"]
                if e is None or dst in st.files:
                    return self._json(200, {"boolean": False})
                pre = p.rstrip("/") + "/"
                for k in [k for k in st.files if k == p or k.startswith(pre)]:
                    st.files[dst + k[len(p):]] = st.files.pop(k)
                return self._json(200, {"boolean": True})
            if op == "SETPERMISSION":
                e["perm"] = q["permission"]
                return self._send(200)
            if op == "SETOWNER":
                e["owner"] = q.get("owner", e["owner"])
                e["group"] = q.get("group", e["group"])
                return self._send(200)
            if op == "GETCONTENTSUMMARY":
                pre = p.rstrip("/") + "/"
                used = sum(len(v.get("data", b"")) for k, v in st.files.items() if k.startswith(pre))
                return self._json(200, {"ContentSummary": {"length": used, "spaceConsumed": used,
                                                           "spaceQuota": 1 << 30}})
        return self._json(400, {})

    def do_GET(self):
        self._handle("GET")

    def do_PUT(self):
        self._handle("PUT")

    def do_POST(self):
        self._handle("POST")

    def do_DELETE(self):
        self._handle("DELETE")


def webhdfs_server(**kw):
    st = WebHdfsState(**kw)
    return _Server(_WebHdfsHandler, st), st
