"""Under-file-system SPI.

Parity: core/common/src/main/java/alluxio/underfs/UnderFileSystem.java:183-749 (create/open/
delete/rename/listStatus/getStatus/mkdirs/getFileLocations/fingerprint/space/mode/owner/active
sync), UfsStatus/UfsFileStatus/UfsDirectoryStatus, Fingerprint.java (content + metadata
fingerprint used by metadata sync), UnderFileSystemWithLogging (metrics/logging wrapper).
"""
from __future__ import annotations

import abc
import dataclasses
import enum
import io
import logging
import time

LOG = logging.getLogger(__name__)


class UfsMode(enum.IntEnum):
    NO_ACCESS = 0
    READ_ONLY = 1
    READ_WRITE = 2


class SpaceType(enum.Enum):
    SPACE_TOTAL = 0
    SPACE_FREE = 1
    SPACE_USED = 2


@dataclasses.dataclass
class UfsStatus:
    name: str
    is_directory: bool
    owner: str = ""
    group: str = ""
    mode: int = 0o755
    last_modified_ms: int | None = None
    xattr: dict | None = None

    @property
    def is_file(self) -> bool:
        return not self.is_directory


@dataclasses.dataclass
class UfsFileStatus(UfsStatus):
    content_length: int = 0
    content_hash: str = ""
    block_size: int = 64 << 20

    def __init__(self, name, content_length=0, content_hash="", last_modified_ms=None, owner="",
                 group="", mode=0o644, block_size=64 << 20, xattr=None):
        # plain attribute stores (no dataclass super().__init__): listings build millions of these
        self.name = name
        self.is_directory = False
        self.owner = owner
        self.group = group
        self.mode = mode
        self.last_modified_ms = last_modified_ms
        self.xattr = xattr
        self.content_length = content_length
        self.content_hash = content_hash
        self.block_size = block_size


@dataclasses.dataclass
class UfsDirectoryStatus(UfsStatus):
    def __init__(self, name, owner="", group="", mode=0o755, last_modified_ms=None, xattr=None):
        super().__init__(name, True, owner, group, mode, last_modified_ms, xattr)


@dataclasses.dataclass
class CreateOptions:
    create_parent: bool = True
    ensure_atomic: bool = False
    owner: str = ""
    group: str = ""
    mode: int = 0o644


@dataclasses.dataclass
class DeleteOptions:
    recursive: bool = False


@dataclasses.dataclass
class ListOptions:
    recursive: bool = False


@dataclasses.dataclass
class MkdirsOptions:
    create_parent: bool = True
    owner: str = ""
    group: str = ""
    mode: int = 0o755


@dataclasses.dataclass
class OpenOptions:
    offset: int = 0
    length: int | None = None
    recover_failed_open: bool = False


class Fingerprint:
    """``TYPE|UFS|OWNER|GROUP|MODE|CONTENT_HASH`` tag string (reference Fingerprint.java)."""

    TAGS = ("TYPE", "UFS", "OWNER", "GROUP", "MODE", "CONTENT_HASH")
    INVALID = "INVALID_UFS_FINGERPRINT"

    def __init__(self, values: dict):
        self.values = values

    @staticmethod
    def create(ufs_type: str, status: UfsStatus) -> "Fingerprint":
        ch = status.content_hash if isinstance(status, UfsFileStatus) else "_"
        return Fingerprint({"TYPE": "DIRECTORY" if status.is_directory else "FILE", "UFS": ufs_type,
                            "OWNER": status.owner or "_", "GROUP": status.group or "_",
                            "MODE": str(status.mode), "CONTENT_HASH": ch or "_"})

    def serialize(self) -> str:
        return " ".join(f"{t}|{self.values.get(t, '_')}" for t in self.TAGS)

    @staticmethod
    def parse(s: str) -> "Fingerprint | None":
        if not s or s == Fingerprint.INVALID:
            return None
        vals = {}
        for tok in s.split(" "):
            if "|" in tok:
                k, v = tok.split("|", 1)
                vals[k] = v
        return Fingerprint(vals)

    def matches_content(self, other: "Fingerprint") -> bool:
        return other is not None and self.values.get("CONTENT_HASH") == other.values.get("CONTENT_HASH") \
            and self.values.get("TYPE") == other.values.get("TYPE")

    def matches_metadata(self, other: "Fingerprint") -> bool:
        return other is not None and all(self.values.get(t) == other.values.get(t)
                                         for t in ("OWNER", "GROUP", "MODE"))


class UnderFileSystem(abc.ABC):
    """Base class: subclasses implement the primitive operations; helpers are shared."""

    scheme = ""
    ufs_type = ""

    def __init__(self, root_uri: str, conf=None, properties: dict | None = None):
        self.root_uri = root_uri
        self.conf = conf
        self.properties = dict(properties or {})

    # ---- lifecycle ---------------------------------------------------------------------------
    def close(self) -> None:
        pass

    def cleanup(self) -> None:
        pass

    def connect_from_master(self, hostname: str) -> None:
        pass

    def connect_from_worker(self, hostname: str) -> None:
        pass

    # ---- primitives --------------------------------------------------------------------------
    @abc.abstractmethod
    def create(self, path: str, options: CreateOptions | None = None) -> io.RawIOBase: ...

    @abc.abstractmethod
    def open(self, path: str, options: OpenOptions | None = None) -> io.RawIOBase: ...

    @abc.abstractmethod
    def delete_file(self, path: str) -> bool: ...

    @abc.abstractmethod
    def delete_directory(self, path: str, options: DeleteOptions | None = None) -> bool: ...

    @abc.abstractmethod
    def get_status(self, path: str) -> UfsStatus | None: ...

    @abc.abstractmethod
    def list_status(self, path: str, options: ListOptions | None = None) -> list[UfsStatus] | None: ...

    @abc.abstractmethod
    def mkdirs(self, path: str, options: MkdirsOptions | None = None) -> bool: ...

    @abc.abstractmethod
    def rename_file(self, src: str, dst: str) -> bool: ...

    @abc.abstractmethod
    def rename_directory(self, src: str, dst: str) -> bool: ...

    # ---- derived -----------------------------------------------------------------------------
    def create_nonexisting_file(self, path: str, options: CreateOptions | None = None):
        return self.create(path, options)

    def delete_existing_file(self, path: str) -> bool:
        return self.delete_file(path)

    def delete_existing_directory(self, path: str, options: DeleteOptions | None = None) -> bool:
        return self.delete_directory(path, options)

    def open_existing_file(self, path: str, options: OpenOptions | None = None):
        return self.open(path, options)

    def rename_renamable_file(self, src: str, dst: str) -> bool:
        return self.rename_file(src, dst)

    def rename_renamable_directory(self, src: str, dst: str) -> bool:
        return self.rename_directory(src, dst)

    def exists(self, path: str) -> bool:
        return self.get_status(path) is not None

    def is_file(self, path: str) -> bool:
        st = self.get_status(path)
        return st is not None and not st.is_directory

    def is_directory(self, path: str) -> bool:
        st = self.get_status(path)
        return st is not None and st.is_directory

    def is_existing_directory(self, path: str) -> bool:
        return self.is_directory(path)

    def get_file_status(self, path: str) -> UfsFileStatus:
        st = self.get_status(path)
        if st is None or st.is_directory:
            raise FileNotFoundError(path)
        return st  # type: ignore[return-value]

    get_existing_file_status = get_file_status

    def get_directory_status(self, path: str) -> UfsDirectoryStatus:
        st = self.get_status(path)
        if st is None or not st.is_directory:
            raise FileNotFoundError(path)
        return st  # type: ignore[return-value]

    get_existing_directory_status = get_directory_status

    def get_existing_status(self, path: str):
        return self.get_status(path)

    def get_block_size_byte(self, path: str) -> int:
        st = self.get_file_status(path)
        return st.block_size

    def get_file_locations(self, path: str, options=None) -> list[str]:
        return []

    def get_fingerprint(self, path: str) -> str:
        try:
            st = self.get_status(path)
        except Exception:  # noqa: BLE001
            return Fingerprint.INVALID
        if st is None:
            return Fingerprint.INVALID
        return Fingerprint.create(self.ufs_type, st).serialize()

    def get_space(self, path: str, space_type: SpaceType) -> int:
        return -1

    def get_operation_mode(self, physical_state: dict[str, UfsMode]) -> UfsMode:
        return physical_state.get(self.root_uri, UfsMode.READ_WRITE)

    def get_physical_stores(self) -> list[str]:
        return [self.root_uri]

    def is_object_storage(self) -> bool:
        return False

    def is_seekable(self) -> bool:
        return True

    def supports_flush(self) -> bool:
        return True

    def supports_active_sync(self) -> bool:
        return False

    def active_sync_changes(self, since_txid: int):
        """UFS change feed for active sync: (changed URIs, new txid).  Only UFSes whose
        ``supports_active_sync`` is true implement it (HDFS inotify)."""
        raise NotImplementedError

    def set_owner(self, path: str, owner: str, group: str) -> None:
        pass

    def set_mode(self, path: str, mode: int) -> None:
        pass

    def set_acl_entries(self, path: str, entries) -> None:
        pass

    def get_acl_pair(self, path: str):
        return None

    def resolve_uri(self, base: str, alluxio_path: str) -> str:
        return base.rstrip("/") + "/" + alluxio_path.lstrip("/")

    def list_recursive(self, path: str) -> list[UfsStatus]:
        return self.list_status(path, ListOptions(recursive=True)) or []

    # convenience for tests/tools
    def read_all(self, path: str) -> bytes:
        with self.open(path) as f:
            return f.read()

    def write_all(self, path: str, data: bytes) -> None:
        with self.create(path) as f:
            f.write(data)


class UnderFileSystemWithLogging(UnderFileSystem):
    """Wrapper that times every call and counts failures (reference UnderFileSystemWithLogging)."""

    def __init__(self, inner: UnderFileSystem, metrics=None):
        super().__init__(inner.root_uri, inner.conf, inner.properties)
        self._inner = inner
        self.scheme = inner.scheme
        self.ufs_type = inner.ufs_type
        self._metrics = metrics

    def _call(self, name, *a, **kw):
        t0 = time.perf_counter()
        try:
            return getattr(self._inner, name)(*a, **kw)
        except Exception:
            if self._metrics is not None:
                self._metrics.counter(f"UfsOpFailures.{name}").inc()
            raise
        finally:
            if self._metrics is not None:
                self._metrics.timer(f"UfsOp.{name}").update(time.perf_counter() - t0)

    def __getattr__(self, item):
        return getattr(self._inner, item)

    def create(self, path, options=None):
        return self._call("create", path, options)

    def open(self, path, options=None):
        return self._call("open", path, options)

    def delete_file(self, path):
        return self._call("delete_file", path)

    def delete_directory(self, path, options=None):
        return self._call("delete_directory", path, options)

    def get_status(self, path):
        return self._call("get_status", path)

    def list_status(self, path, options=None):
        return self._call("list_status", path, options)

    def mkdirs(self, path, options=None):
        return self._call("mkdirs", path, options)

    def rename_file(self, src, dst):
        return self._call("rename_file", src, dst)

    def rename_directory(self, src, dst):
        return self._call("rename_directory", src, dst)

    def get_fingerprint(self, path):
        return self._call("get_fingerprint", path)

    def is_object_storage(self):
        return self._inner.is_object_storage()
