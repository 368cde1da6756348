"""Mount table: Alluxio path prefixes -> UFS URIs.

Parity: core/server/master/src/main/java/alluxio/master/file/meta/MountTable.java (add/delete/
update mount points journaled as AddMountPointEntry / DeleteMountPointEntry, longest-prefix
``resolve`` to (UFS URI, mount id), ``reverseResolve`` from a UFS URI, nested-mount and
read-only checks) plus the master's UfsManager (mount id -> UFS client cache).
"""
from __future__ import annotations

import threading

from ..proto import pb
from ..underfs import registry as ufs_registry
from ..utils.exceptions import AccessControlException, InvalidPathException, NotFoundException
from ..utils.uri import normalize_path

ROOT_MOUNT_ID = 1


class MountInfo:
    __slots__ = ("alluxio_path", "ufs_uri", "mount_id", "read_only", "shared", "properties")

    def __init__(self, alluxio_path, ufs_uri, mount_id, read_only=False, shared=False, properties=None):
        self.alluxio_path = alluxio_path
        self.ufs_uri = ufs_uri
        self.mount_id = mount_id
        self.read_only = read_only
        self.shared = shared
        self.properties = dict(properties or {})

    def to_entry(self):
        return pb.journal.JournalEntry(add_mount_point=pb.journal.AddMountPointEntry(
            alluxio_path=self.alluxio_path, ufs_path=self.ufs_uri, readOnly=self.read_only,
            shared=self.shared, mount_id=self.mount_id,
            properties=[pb.journal.StringPairEntry(key=k, value=v) for k, v in sorted(self.properties.items())]))

    def to_proto(self, ufs=None):
        m = pb.file.MountPointInfo(ufsUri=self.ufs_uri, ufsType=getattr(ufs, "ufs_type", ""),
                                   readOnly=self.read_only, shared=self.shared)
        for k, v in self.properties.items():
            m.properties[k] = v
        return m


class Resolution:
    __slots__ = ("uri", "ufs", "mount_id", "mount", "shared")

    def __init__(self, uri, ufs, mount_id, mount):
        self.uri, self.ufs, self.mount_id, self.mount = uri, ufs, mount_id, mount
        self.shared = mount.shared


class UfsManager:
    """Caches one UFS client per mount id."""

    def __init__(self, conf=None, metrics=None):
        self.conf = conf
        self.metrics = metrics
        self._lock = threading.Lock()
        self._ufs: dict[int, object] = {}
        self._info: dict[int, tuple[str, dict]] = {}

    def add_mount(self, mount_id: int, uri: str, properties: dict | None = None):
        with self._lock:
            self._info[mount_id] = (uri, dict(properties or {}))
            u = ufs_registry.create(uri, self.conf, properties)
            self._ufs[mount_id] = u
            return u

    def remove_mount(self, mount_id: int) -> None:
        with self._lock:
            u = self._ufs.pop(mount_id, None)
            self._info.pop(mount_id, None)
        if u is not None:
            try:
                u.close()
            except Exception:  # noqa: BLE001
                pass

    def get(self, mount_id: int):
        with self._lock:
            u = self._ufs.get(mount_id)
        if u is None:
            raise NotFoundException(f"mount id {mount_id} not found")
        return u

    def info(self, mount_id: int):
        with self._lock:
            return self._info.get(mount_id)


class MountTable:
    def __init__(self, ufs_manager: UfsManager):
        self._lock = threading.RLock()
        self._mounts: dict[str, MountInfo] = {}
        self.epoch = 0          # bumped on every mount-table change (cached FileInfo.ufsPath)
        self.epoch_listeners: list = []
        self.ufs_manager = ufs_manager

    def _bump_epoch(self) -> None:
        self.epoch += 1
        for cb in self.epoch_listeners:
            cb()

    def reset(self) -> None:
        with self._lock:
            self._bump_epoch()
            for m in self._mounts.values():
                self.ufs_manager.remove_mount(m.mount_id)
            self._mounts = {}

    # ---- state changes (called from journal application) ------------------------------------
    def apply_add(self, info: MountInfo) -> None:
        with self._lock:
            self._bump_epoch()
            # copy-on-write: readers use the dict they loaded without taking the lock
            m = dict(self._mounts)
            m[info.alluxio_path] = info
            self._mounts = m
            self.ufs_manager.add_mount(info.mount_id, info.ufs_uri, info.properties)

    def apply_delete(self, alluxio_path: str) -> MountInfo | None:
        with self._lock:
            self._bump_epoch()
            m = dict(self._mounts)
            info = m.pop(alluxio_path, None)
            self._mounts = m
        if info is not None:
            self.ufs_manager.remove_mount(info.mount_id)
        return info

    # ---- queries ----------------------------------------------------------------------------
    def mount_point_for(self, path: str) -> str | None:
        """Deepest mount point at or above ``path``: one dict probe per path level, lock-free
        (``_mounts`` is replaced, never mutated)."""
        mounts = self._mounts
        p = normalize_path(path)
        while True:
            if p in mounts:
                return p
            if p == "/":
                return None
            p = p[:p.rfind("/")] or "/"

    def is_mount_point(self, path: str) -> bool:
        with self._lock:
            return normalize_path(path) in self._mounts

    def get(self, path: str) -> MountInfo | None:
        with self._lock:
            return self._mounts.get(normalize_path(path))

    def by_id(self, mount_id: int) -> MountInfo | None:
        with self._lock:
            for m in self._mounts.values():
                if m.mount_id == mount_id:
                    return m
        return None

    def resolve(self, path: str) -> Resolution:
        path = normalize_path(path)
        mounts = self._mounts
        mp = self.mount_point_for(path)
        info = mounts.get(mp) if mp is not None else None
        if info is None:
            info = self._mounts.get(mp) if mp is not None else None
        if info is None:
            raise InvalidPathException(f"no mount point for {path}")
        rel = path[len(mp):] if mp != "/" else path
        rel = rel.lstrip("/")
        base = info.ufs_uri.rstrip("/")
        uri = base + ("/" + rel if rel else "") if base else "/" + rel
        return Resolution(uri, self.ufs_manager.get(info.mount_id), info.mount_id, info)

    def reverse_resolve(self, ufs_uri: str) -> str | None:
        with self._lock:
            best = None
            for mp, info in self._mounts.items():
                base = info.ufs_uri.rstrip("/")
                if ufs_uri == base or ufs_uri.startswith(base + "/"):
                    if best is None or len(base) > len(best[1]):
                        best = (mp, base)
        if best is None:
            return None
        mp, base = best
        rest = ufs_uri[len(base):]
        return normalize_path(mp.rstrip("/") + rest)

    def check_under_write_mount(self, path: str) -> None:
        mp = self.mount_point_for(path)
        if mp is not None and self._mounts[mp].read_only:
            raise AccessControlException(f"cannot modify {path}: mount point {mp} is read-only")

    def mounts(self) -> dict[str, MountInfo]:
        with self._lock:
            return dict(self._mounts)

    def validate_new_mount(self, alluxio_path: str, ufs_uri: str) -> None:
        alluxio_path = normalize_path(alluxio_path)
        with self._lock:
            if alluxio_path in self._mounts:
                raise InvalidPathException(f"mount point {alluxio_path} already exists")
            for mp, info in self._mounts.items():
                if mp != "/" and (alluxio_path.startswith(mp.rstrip("/") + "/")):
                    raise InvalidPathException(f"mount point {alluxio_path} is a prefix of/under mount {mp}")
                base = info.ufs_uri.rstrip("/")
                u = ufs_uri.rstrip("/")
                if u and base and (u == base or u.startswith(base + "/") or base.startswith(u + "/")) and mp != "/":
                    raise InvalidPathException(f"ufs path {ufs_uri} overlaps existing mount {mp} ({info.ufs_uri})")
