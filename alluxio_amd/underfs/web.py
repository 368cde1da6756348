"""Read-only HTTP(S) UFS (reference underfs/web/.../WebUnderFileSystem.java): files are
fetched with ranged GETs, directories are parsed from HTML index pages (``<a href>`` links)."""
from __future__ import annotations

import io
import re
import urllib.parse

from .base import UfsDirectoryStatus, UfsFileStatus, UnderFileSystem
from .registry import UnderFileSystemFactory, register_factory

_HREF = re.compile(r'href="([^"?#]+)"', re.I)


class WebUnderFileSystem(UnderFileSystem):
    scheme = "http"
    ufs_type = "web"

    def __init__(self, root_uri, conf=None, properties=None):
        super().__init__(root_uri, conf, properties)
        import requests
        self.session = requests.Session()

    def _url(self, path):
        return path if "://" in path else self.root_uri.rstrip("/") + "/" + path.lstrip("/")

    def _ro(self, *a, **kw):
        raise PermissionError("web UFS is read-only")

    create = mkdirs = delete_file = delete_directory = rename_file = rename_directory = _ro

    def open(self, path, options=None):
        h = {}
        if options and options.offset:
            h["Range"] = f"bytes={options.offset}-"
        r = self.session.get(self._url(path), headers=h, timeout=60)
        if r.status_code == 404:
            raise FileNotFoundError(path)
        r.raise_for_status()
        return io.BytesIO(r.content)

    def get_status(self, path):
        url = self._url(path)
        r = self.session.head(url, timeout=30, allow_redirects=True)
        if r.status_code == 404:
            return None
        name = urllib.parse.unquote(url.rstrip("/").rsplit("/", 1)[-1])
        ctype = r.headers.get("Content-Type", "")
        if url.endswith("/") or "text/html" in ctype and "Content-Length" not in r.headers:
            return UfsDirectoryStatus(name)
        return UfsFileStatus(name, int(r.headers.get("Content-Length", 0)), r.headers.get("ETag", ""))

    def list_status(self, path, options=None):
        url = self._url(path).rstrip("/") + "/"
        r = self.session.get(url, timeout=60)
        if r.status_code != 200:
            return None
        out = []
        for href in _HREF.findall(r.text):
            if href.startswith(("/", "..", "http")):
                continue
            name = urllib.parse.unquote(href.rstrip("/"))
            out.append(UfsDirectoryStatus(name) if href.endswith("/") else UfsFileStatus(name))
        return out


class _WebFactory(UnderFileSystemFactory):
    def __init__(self, scheme):
        self.scheme = scheme

    def create(self, uri, conf=None, properties=None):
        return WebUnderFileSystem(uri, conf, properties)


register_factory(_WebFactory("http"))
register_factory(_WebFactory("https"))
