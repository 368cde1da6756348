"""OpenStack Swift UFS (``swift://<container>/<path>``).

Parity: underfs/swift/src/main/java/alluxio/underfs/swift/SwiftUnderFileSystem.java:59-520
(container = bucket, ``/`` folder markers, auth methods tempauth / swiftauth / keystone (v2) /
keystonev3 from ``fs.swift.*``, ``fs.swift.simulation`` in-memory mode, container read/write
ACLs mapped to an Alluxio mode for the account owner, copy via ``X-Copy-From``, prefix listing
with ``delimiter``), SwiftInputStream (ranged GET per chunk) and KeystoneV3Access (token from
``X-Subject-Token``, object-store endpoint from the catalog, preferred region).  The reference
goes through the JOSS client library; this speaks the Swift v1 HTTP API directly.
"""
from __future__ import annotations

import datetime
import threading
import time
import urllib.parse

from .object_store import ObjectMeta, ObjectUnderFileSystem
from .registry import UnderFileSystemFactory, register_factory


class SwiftAuthError(PermissionError):
    pass


class SwiftClient:
    """Authenticated Swift v1 API client; re-authenticates once on 401."""

    def __init__(self, auth_url: str, user: str = "", tenant: str = "", password: str = "",
                 method: str | None = None, region: str | None = None, timeout: float = 60.0):
        import requests
        self.auth_url = auth_url.rstrip("/")
        self.user, self.tenant, self.password = user, tenant, password
        self.method = (method or "tempauth").lower()
        self.region = region
        self.timeout = timeout
        self.session = requests.Session()
        self.storage_url = None
        self.token = None
        self._lock = threading.Lock()

    # ---- authentication ---------------------------------------------------------------------
    def authenticate(self) -> None:
        m = self.method
        if m in ("tempauth", "swiftauth"):
            # both expect "tenant:user" in X-Auth-User (SwiftUnderFileSystem swaps for JOSS)
            r = self.session.get(self.auth_url, headers={"X-Auth-User": f"{self.tenant}:{self.user}",
                                                         "X-Auth-Key": self.password}, timeout=self.timeout)
            if r.status_code >= 400:
                raise SwiftAuthError(f"swift {m} authentication failed: HTTP {r.status_code}")
            self.storage_url, self.token = r.headers["X-Storage-Url"], r.headers["X-Auth-Token"]
        elif m == "keystone":
            body = {"auth": {"passwordCredentials": {"username": self.user, "password": self.password},
                             "tenantName": self.tenant}}
            r = self.session.post(self.auth_url + "/tokens", json=body, timeout=self.timeout)
            if r.status_code >= 400:
                raise SwiftAuthError(f"keystone v2 authentication failed: HTTP {r.status_code}")
            acc = r.json()["access"]
            self.token = acc["token"]["id"]
            self.storage_url = self._endpoint(
                [e for s in acc.get("serviceCatalog", []) if s.get("type") == "object-store"
                 for e in s.get("endpoints", [])], url_key="publicURL")
        elif m == "keystonev3":
            body = {"auth": {
                "identity": {"methods": ["password"], "password": {"user": {
                    "name": self.user, "domain": {"id": "default"}, "password": self.password}}},
                "scope": {"project": {"name": self.tenant, "domain": {"id": "default"}}}}}
            r = self.session.post(self.auth_url + "/auth/tokens", json=body, timeout=self.timeout)
            if r.status_code >= 400:
                raise SwiftAuthError(f"keystone v3 authentication failed: HTTP {r.status_code}")
            self.token = r.headers["X-Subject-Token"]
            cat = r.json()["token"].get("catalog", [])
            self.storage_url = self._endpoint(
                [e for s in cat if s.get("type") == "object-store" for e in s.get("endpoints", [])
                 if e.get("interface", "public") == "public"], url_key="url")
        else:
            raise SwiftAuthError(f"unknown fs.swift.auth.method {self.method!r}")

    def _endpoint(self, endpoints, url_key: str) -> str:
        if not endpoints:
            raise SwiftAuthError("no object-store endpoint in the service catalog")
        if self.region:
            for e in endpoints:
                if e.get("region") == self.region or e.get("region_id") == self.region:
                    return e[url_key]
        return endpoints[0][url_key]

    # ---- requests ---------------------------------------------------------------------------
    def request(self, method, container, obj="", params=None, data=b"", headers=None, ok=(200, 201, 202, 204, 206)):
        with self._lock:
            if self.token is None:
                self.authenticate()
        for attempt in (0, 1):
            url = f"{self.storage_url}/{urllib.parse.quote(container)}"
            if obj:
                url += "/" + urllib.parse.quote(obj)
            h = {"X-Auth-Token": self.token}
            h.update(headers or {})
            r = self.session.request(method, url, params=params, data=data, headers=h, timeout=self.timeout)
            if r.status_code == 401 and attempt == 0:
                with self._lock:
                    self.authenticate()
                continue
            if r.status_code == 404:
                raise FileNotFoundError(f"{container}/{obj}")
            if r.status_code not in ok:
                raise OSError(f"swift {method} {container}/{obj}: HTTP {r.status_code} {r.text[:200]}")
            return r
        raise SwiftAuthError("swift token rejected after re-authentication")


class _SimulatedSwift:
    """``fs.swift.simulation``: an in-memory container (JOSS mock mode)."""

    def __init__(self):
        self.objects: dict[str, bytes] = {}
        self.mtimes: dict[str, int] = {}      # last-modified ms, as a real container reports it
        self.lock = threading.Lock()


_SIM: dict[str, _SimulatedSwift] = {}


def _parse_ts(s: str | None) -> int | None:
    if not s:
        return None
    for fmt in ("%Y-%m-%dT%H:%M:%S.%f", "%Y-%m-%dT%H:%M:%S", "%a, %d %b %Y %H:%M:%S %Z"):
        try:
            return int(datetime.datetime.strptime(s, fmt).replace(tzinfo=datetime.timezone.utc).timestamp() * 1000)
        except ValueError:
            continue
    return None


class SwiftUnderFileSystem(ObjectUnderFileSystem):
    scheme = "swift"
    ufs_type = "swift"
    list_limit = 10_000

    def __init__(self, root_uri, conf=None, properties=None):
        super().__init__(root_uri, conf, properties)
        p = dict(properties or {})

        def opt(name, default=None):
            if name in p:
                return p[name]
            if conf is not None and conf.get_raw(name) is not None:
                return conf.get(name)
            return default
        self.container = root_uri.split("://", 1)[1].split("/", 1)[0]
        self.owner = opt("fs.swift.user", "") or ""
        self.simulation = str(opt("fs.swift.simulation", "false")).lower() == "true"
        self.client = None
        if self.simulation:
            self._sim = _SIM.setdefault(self.container, _SimulatedSwift())
            self.mode = 0o700
            return
        self.client = SwiftClient(opt("fs.swift.auth.url", ""), user=opt("fs.swift.user", ""),
                                  tenant=opt("fs.swift.tenant", ""), password=opt("fs.swift.password", ""),
                                  method=opt("fs.swift.auth.method"), region=opt("fs.swift.region"))
        r = self.client.request("HEAD", self.container)   # the container must exist
        self.mode = self._acl_mode(r.headers)

    def _acl_mode(self, h) -> int:
        """Container ACLs -> mode bits for the account owner (SwiftUnderFileSystem ctor)."""
        def acl(name):
            return [a.strip() for a in (h.get(name) or "").split(",") if a.strip()]
        mode = 0
        read, write = acl("X-Container-Read"), acl("X-Container-Write")
        if self.owner in read or "*" in read or ".r:*" in read:
            mode |= 0o500
        if self.owner in write or "*" in write or ".w:*" in write:
            mode |= 0o200
        return mode or 0o700      # no ACL but access granted: the user is an admin

    # ---- primitives -------------------------------------------------------------------------
    def _put(self, key, data):
        if self.simulation:
            with self._sim.lock:
                self._sim.objects[key] = bytes(data)
                self._sim.mtimes[key] = int(time.time() * 1000)
            return
        self.client.request("PUT", self.container, key, data=data)

    def _get_range(self, key, offset, length):
        if length <= 0:
            return b""
        if self.simulation:
            with self._sim.lock:
                if key not in self._sim.objects:
                    raise FileNotFoundError(key)
                return self._sim.objects[key][offset:offset + length]
        r = self.client.request("GET", self.container, key, headers={"Range": f"bytes={offset}-{offset + length - 1}"})
        return r.content

    def _head(self, key):
        if self.simulation:
            with self._sim.lock:
                d = self._sim.objects.get(key)
                mt = self._sim.mtimes.get(key)
            return None if d is None else ObjectMeta(key, len(d), str(hash(d) & 0xFFFFFFFF), mt)
        try:
            r = self.client.request("HEAD", self.container, key)
        except FileNotFoundError:
            return None
        return ObjectMeta(key, int(r.headers.get("Content-Length", 0)), r.headers.get("ETag", "").strip('"'),
                          _parse_ts(r.headers.get("Last-Modified")))

    def _delete(self, keys):
        for k in keys:
            if not k:
                continue
            if self.simulation:
                with self._sim.lock:
                    self._sim.objects.pop(k, None)
                    self._sim.mtimes.pop(k, None)
                continue
            try:
                self.client.request("DELETE", self.container, k)
            except FileNotFoundError:
                pass

    def _list(self, prefix, delimiter):
        if self.simulation:
            with self._sim.lock:
                keys = sorted(k for k in self._sim.objects if k.startswith(prefix))
                objs, prefixes = [], set()
                for k in keys:
                    rest = k[len(prefix):]
                    if delimiter and delimiter in rest:
                        prefixes.add(prefix + rest.split(delimiter, 1)[0] + delimiter)
                    else:
                        objs.append(ObjectMeta(k, len(self._sim.objects[k]), "", self._sim.mtimes.get(k)))
            return objs, sorted(prefixes)
        objs, prefixes, marker = [], [], None
        while True:
            q = {"format": "json", "prefix": prefix, "limit": str(self.list_limit)}
            if delimiter:
                q["delimiter"] = delimiter
            if marker:
                q["marker"] = marker
            page = self.client.request("GET", self.container, params=q).json()
            for e in page:
                if "subdir" in e:
                    prefixes.append(e["subdir"])
                    marker = e["subdir"]
                else:
                    objs.append(ObjectMeta(e["name"], int(e.get("bytes", 0)), e.get("hash", ""),
                                           _parse_ts(e.get("last_modified"))))
                    marker = e["name"]
            if len(page) < self.list_limit:
                return objs, prefixes

    def _copy(self, src, dst):
        if self.simulation:
            with self._sim.lock:
                self._sim.objects[dst] = self._sim.objects[src]
                self._sim.mtimes[dst] = int(time.time() * 1000)
            return
        self.client.request("PUT", self.container, dst, data=b"",
                            headers={"X-Copy-From": f"/{self.container}/{src}", "Content-Length": "0"})

    # ---- metadata ---------------------------------------------------------------------------
    def get_status(self, path):
        st = super().get_status(path)
        if st is not None:
            st.owner = st.owner or self.owner
            st.mode = self.mode
        return st


class _SwiftFactory(UnderFileSystemFactory):
    scheme = "swift"

    def create(self, uri, conf=None, properties=None):
        return SwiftUnderFileSystem(uri, conf, properties)


register_factory(_SwiftFactory())
