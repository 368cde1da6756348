"""``AlluxioURI`` — scheme/authority/path triple with POSIX-style path normalisation.

Parity target: core/base/src/main/java/alluxio/AlluxioURI.java (join, getParent, getDepth,
isAncestorOf, getName, leading-slash normalisation).  Alluxio paths are always absolute; the
scheme is ``alluxio`` and the authority names the master (``host:19998``) or a zookeeper /
embedded-journal ensemble.
"""
from __future__ import annotations

import posixpath
from urllib.parse import urlsplit

SEPARATOR = "/"
ROOT = "/"
SCHEME = "alluxio"


def _is_normal(path: str) -> bool:
    """Already canonical: absolute, no empty / ``.`` / ``..`` components, no trailing slash."""
    if path == ROOT:
        return True
    if path[0] != SEPARATOR or path[-1] == SEPARATOR or "//" in path:
        return False
    return "/." not in path or all(c not in (".", "..") for c in path.split(SEPARATOR))


def normalize_path(path: str) -> str:
    if not path:
        return ROOT
    if _is_normal(path):           # the common case on every RPC: no normpath work
        return path
    if not path.startswith(SEPARATOR):
        path = SEPARATOR + path
    out = posixpath.normpath(path)
    if out.startswith("//"):
        out = "/" + out.lstrip("/")
    return out


class AlluxioURI:
    __slots__ = ("scheme", "authority", "path", "query")

    def __init__(self, uri: str = "/", scheme: str | None = None, authority: str | None = None):
        if "://" in uri:
            parts = urlsplit(uri)
            self.scheme = parts.scheme or None
            self.authority = parts.netloc or None
            self.path = parts.path or ROOT
            self.query = parts.query or None
        else:
            self.scheme = scheme
            self.authority = authority
            self.path = uri
            self.query = None
        # Object-store and local UFS URIs keep their path as given; alluxio paths normalise.
        if self.scheme in (None, SCHEME, "file"):
            self.path = normalize_path(self.path)

    # --- path algebra -------------------------------------------------------------------------
    def join(self, suffix: str) -> "AlluxioURI":
        if not suffix:
            return self
        base = self.path.rstrip(SEPARATOR)
        new = base + SEPARATOR + suffix.lstrip(SEPARATOR)
        return AlluxioURI._raw(self.scheme, self.authority, new)

    def get_parent(self) -> "AlluxioURI | None":
        if self.path == ROOT:
            return None
        parent = posixpath.dirname(self.path.rstrip(SEPARATOR)) or ROOT
        return AlluxioURI._raw(self.scheme, self.authority, parent)

    def get_name(self) -> str:
        if self.path == ROOT:
            return ""
        return posixpath.basename(self.path.rstrip(SEPARATOR))

    def get_depth(self) -> int:
        if self.path == ROOT:
            return 0
        return self.path.rstrip(SEPARATOR).count(SEPARATOR)

    def components(self) -> list[str]:
        return [c for c in self.path.split(SEPARATOR) if c]

    def is_root(self) -> bool:
        return self.path == ROOT

    def is_ancestor_of(self, other: "AlluxioURI") -> bool:
        if self.path == ROOT:
            return True
        a = self.path.rstrip(SEPARATOR) + SEPARATOR
        return other.path == self.path or other.path.startswith(a)

    def has_scheme(self) -> bool:
        return bool(self.scheme)

    @staticmethod
    def _raw(scheme, authority, path) -> "AlluxioURI":
        u = AlluxioURI.__new__(AlluxioURI)
        u.scheme, u.authority, u.path, u.query = scheme, authority, path, None
        return u

    def __str__(self) -> str:
        if self.scheme:
            return f"{self.scheme}://{self.authority or ''}{self.path}"
        return self.path

    def __repr__(self) -> str:
        return f"AlluxioURI({str(self)!r})"

    def __eq__(self, other) -> bool:
        if isinstance(other, str):
            other = AlluxioURI(other)
        return isinstance(other, AlluxioURI) and str(self) == str(other)

    def __hash__(self) -> int:
        return hash(str(self))


def as_uri(path) -> AlluxioURI:
    return path if isinstance(path, AlluxioURI) else AlluxioURI(str(path))


def path_components(path: str) -> list[str]:
    p = normalize_path(path)
    return p.split(SEPARATOR)[1:] if p != ROOT else []


def join_path(*parts: str) -> str:
    out = SEPARATOR.join(p.strip(SEPARATOR) for p in parts if p and p != SEPARATOR)
    return normalize_path(out)
