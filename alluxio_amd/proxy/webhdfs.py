"""WebHDFS REST gateway: Hadoop-ecosystem clients reach the Alluxio namespace over ``webhdfs://``.

The reference gives Hadoop clients the ``alluxio://`` scheme through its Java client
(core/client/hdfs/src/main/java/alluxio/hadoop/AbstractFileSystem.java:152,447-460,622-629:
``create``, ``open``, ``getFileStatus``, ``listStatus``, ``mkdirs``, ``rename``, ``delete``,
``setOwner``/``setPermission``, ``getContentSummary``, ``getFileChecksum``).  No JVM exists here to
host that class, so the proxy speaks the WebHDFS REST protocol (Hadoop's ``WebHdfsFileSystem`` and
``curl``/``requests`` clients) on ``/webhdfs/v1``:

* namenode-style two-step writes: ``PUT ?op=CREATE`` answers ``307`` with a ``Location`` back to
  this gateway (``&datanode=true``), the client then PUTs the bytes there -- written with the
  proxy's write type, so they land in the workers' cache tier;
* ``GET ?op=OPEN&offset=&length=`` answers ``307`` to itself and streams the range from the
  Alluxio client (``noredirect=true`` returns the location as JSON instead, like Hadoop);
* ``GETFILESTATUS``, ``LISTSTATUS``, ``LISTSTATUS_BATCH`` (``startAfter``), ``GETCONTENTSUMMARY``,
  ``GETFILECHECKSUM`` (``COMPOSITE-CRC32C``: the CRC32C of the whole file, Hadoop's composite
  checksum format), ``GETHOMEDIRECTORY``, ``MKDIRS``, ``RENAME``, ``DELETE``, ``SETPERMISSION``,
  ``SETOWNER``, ``SETTIMES`` (accepted, no settable times as in the reference's FUSE/HDFS client);
* ``APPEND``/``TRUNCATE``/``CONCAT`` answer ``UnsupportedOperationException``: Alluxio files are
  write-once (AbstractFileSystem.append throws the same);
* errors are ``RemoteException`` JSON with the Java exception name and the matching HTTP status.
"""
from __future__ import annotations

import json
import posixpath
import urllib.parse

from ..utils.exceptions import (AlreadyExistsException, AlluxioStatusException, InvalidArgumentException,
                                NotFoundException, PermissionDeniedException)

PREFIX = "/webhdfs/v1"
CHUNK = 8 << 20


class WebHdfsError(Exception):
    def __init__(self, status: int, exception: str, java_class: str, message: str):
        super().__init__(message)
        self.status, self.exception, self.java_class, self.message = status, exception, java_class, message

    def body(self) -> bytes:
        return json.dumps({"RemoteException": {"exception": self.exception, "javaClassName": self.java_class,
                                               "message": self.message}}).encode()


def _translate(e: Exception, path: str) -> WebHdfsError:
    if isinstance(e, WebHdfsError):
        return e
    if isinstance(e, NotFoundException):
        return WebHdfsError(404, "FileNotFoundException", "java.io.FileNotFoundException", f"File does not exist: {path}")
    if isinstance(e, AlreadyExistsException):
        return WebHdfsError(403, "FileAlreadyExistsException", "org.apache.hadoop.fs.FileAlreadyExistsException",
                            str(e))
    if isinstance(e, PermissionDeniedException):
        return WebHdfsError(403, "AccessControlException", "org.apache.hadoop.security.AccessControlException", str(e))
    if isinstance(e, (InvalidArgumentException, ValueError)):
        return WebHdfsError(400, "IllegalArgumentException", "java.lang.IllegalArgumentException", str(e))
    if isinstance(e, AlluxioStatusException) and "DirectoryNotEmpty" in type(e).__name__:
        return WebHdfsError(403, "PathIsNotEmptyDirectoryException",
                            "org.apache.hadoop.fs.PathIsNotEmptyDirectoryException", str(e))
    return WebHdfsError(500, "IOException", "java.io.IOException", str(e))


def _bool(v, default=False) -> bool:
    if v is None:
        return default
    return str(v).lower() in ("true", "1", "yes")


class WebHdfsGateway:
    """WebHDFS semantics over an Alluxio :class:`FileSystem` client."""

    def __init__(self, fs, write_type: str = "CACHE_THROUGH"):
        self.fs = fs
        self.write_type = write_type

    # ---- JSON shapes ------------------------------------------------------------------------
    @staticmethod
    def file_status(info, suffix: str | None = None) -> dict:
        folder = bool(info.folder)
        return {"accessTime": int(info.lastAccessTimeMs or info.lastModificationTimeMs or 0),
                "blockSize": 0 if folder else int(info.blockSizeBytes or 0),
                "childrenNum": 0,
                "fileId": int(info.fileId),
                "group": info.group or "",
                "length": 0 if folder else int(info.length),
                "modificationTime": int(info.lastModificationTimeMs or 0),
                "owner": info.owner or "",
                "pathSuffix": info.name if suffix is None else suffix,
                "permission": format(int(info.mode) & 0o7777, "o"),
                "replication": 0 if folder else max(1, int(getattr(info, "replicationMin", 0) or 1)),
                "storagePolicy": 0,
                "type": "DIRECTORY" if folder else "FILE"}

    # ---- dispatch ---------------------------------------------------------------------------
    def handle(self, method: str, path: str, q: dict, host: str, body_iter):
        """-> (status, headers, body bytes | iterator of bytes)."""
        op = (q.get("op") or "").upper()
        try:
            return self._dispatch(method, op, path, q, host, body_iter)
        except Exception as e:  # noqa: BLE001 - every failure is a RemoteException
            err = _translate(e, path)
            return err.status, {"Content-Type": "application/json"}, err.body()

    def _json(self, obj, status: int = 200):
        return status, {"Content-Type": "application/json"}, json.dumps(obj).encode()

    def _redirect(self, path: str, q: dict, host: str, noredirect: bool):
        q2 = dict(q)
        q2.pop("noredirect", None)
        q2["datanode"] = "true"
        loc = f"http://{host}{PREFIX}{urllib.parse.quote(path)}?{urllib.parse.urlencode(q2)}"
        if noredirect:
            return self._json({"Location": loc})
        return 307, {"Location": loc, "Content-Type": "application/octet-stream"}, b""

    def _dispatch(self, method, op, path, q, host, body_iter):
        fs = self.fs
        if method == "GET":
            if op == "GETFILESTATUS":
                st = fs.get_status(path)
                return self._json({"FileStatus": self.file_status(st.info, "")})
            if op == "LISTSTATUS":
                st = fs.get_status(path)
                if not st.info.folder:
                    return self._json({"FileStatuses": {"FileStatus": [self.file_status(st.info, "")]}})
                kids = sorted(fs.list_status(path), key=lambda s: s.info.name)
                return self._json({"FileStatuses": {"FileStatus": [self.file_status(k.info) for k in kids]}})
            if op == "LISTSTATUS_BATCH":
                kids = sorted(fs.list_status(path), key=lambda s: s.info.name)
                after = q.get("startAfter", "")
                if after:
                    kids = [k for k in kids if k.info.name > after]
                limit = 1000
                part = kids[:limit]
                return self._json({"DirectoryListing": {
                    "partialListing": {"FileStatuses": {"FileStatus": [self.file_status(k.info) for k in part]}},
                    "remainingEntries": max(0, len(kids) - limit)}})
            if op == "GETCONTENTSUMMARY":
                return self._json({"ContentSummary": self._summary(path)})
            if op == "GETFILECHECKSUM":
                return self._json({"FileChecksum": self._checksum(path)})
            if op == "GETHOMEDIRECTORY":
                user = q.get("user.name") or "alluxio"
                return self._json({"Path": f"/user/{user}"})
            if op == "OPEN":
                if not _bool(q.get("datanode")):
                    fs.get_status(path)                       # 404 before redirecting
                    return self._redirect(path, q, host, _bool(q.get("noredirect")))
                return self._open(path, q)
        elif method == "PUT":
            if op == "CREATE":
                if not _bool(q.get("datanode")):
                    if fs.exists(path) and not _bool(q.get("overwrite")):
                        raise WebHdfsError(403, "FileAlreadyExistsException",
                                           "org.apache.hadoop.fs.FileAlreadyExistsException", f"{path} already exists")
                    return self._redirect(path, q, host, _bool(q.get("noredirect")))
                return self._create(path, q, host, body_iter)
            if op == "MKDIRS":
                if fs.exists(path):
                    return self._json({"boolean": bool(fs.get_status(path).info.folder)})
                kw = {}
                if q.get("permission"):
                    kw["mode"] = int(q["permission"], 8)
                fs.create_directory(path, recursive=True, allow_exists=True, **kw)
                return self._json({"boolean": True})
            if op == "RENAME":
                dst = q.get("destination")
                if not dst:
                    raise WebHdfsError(400, "IllegalArgumentException", "java.lang.IllegalArgumentException",
                                       "RENAME needs destination")
                if not fs.exists(path) or fs.exists(dst):
                    return self._json({"boolean": False})
                parent = posixpath.dirname(dst.rstrip("/")) or "/"
                if not fs.exists(parent):
                    return self._json({"boolean": False})
                fs.rename(path, dst)
                return self._json({"boolean": True})
            if op == "SETPERMISSION":
                fs.set_attribute(path, mode=int(q.get("permission", "755"), 8))
                return 200, {"Content-Length": "0"}, b""
            if op == "SETOWNER":
                fs.set_attribute(path, owner=q.get("owner") or None, group=q.get("group") or None)
                return 200, {"Content-Length": "0"}, b""
            if op == "SETTIMES":
                fs.get_status(path)
                return 200, {"Content-Length": "0"}, b""
            if op == "TRUNCATE":
                raise WebHdfsError(403, "UnsupportedOperationException", "java.lang.UnsupportedOperationException",
                                   "Alluxio files are write-once: truncate is not supported")
        elif method == "POST":
            if op in ("APPEND", "CONCAT", "TRUNCATE"):
                raise WebHdfsError(403, "UnsupportedOperationException", "java.lang.UnsupportedOperationException",
                                   f"Alluxio files are write-once: {op.lower()} is not supported")
        elif method == "DELETE":
            if op == "DELETE":
                if not fs.exists(path):
                    return self._json({"boolean": False})
                st = fs.get_status(path)
                rec = _bool(q.get("recursive"))
                if st.info.folder and not rec and fs.list_status(path):
                    raise WebHdfsError(403, "PathIsNotEmptyDirectoryException",
                                       "org.apache.hadoop.fs.PathIsNotEmptyDirectoryException",
                                       f"{path} is non empty': Directory is not empty")
                if path.rstrip("/") in ("", "/"):
                    return self._json({"boolean": False})
                fs.delete(path, recursive=rec)
                return self._json({"boolean": True})
        raise WebHdfsError(400, "IllegalArgumentException", "java.lang.IllegalArgumentException",
                           f"Invalid value for webhdfs parameter \"op\": {op or '(none)'} for {method}")

    # ---- data ops ---------------------------------------------------------------------------
    def _open(self, path, q):
        st = self.fs.get_status(path)
        if st.info.folder:
            raise WebHdfsError(404, "FileNotFoundException", "java.io.FileNotFoundException", f"{path} is a directory")
        size = int(st.info.length)
        off = int(q.get("offset") or 0)
        if off < 0 or off > size:
            raise WebHdfsError(400, "IOException", "java.io.IOException", f"Offset={off} out of the range [0, {size}]")
        n = size - off if q.get("length") in (None, "") else min(int(q["length"]), size - off)
        f = self.fs.open_file(path)

        def chunks():
            try:
                f.seek(off)
                left = n
                while left > 0:
                    b = f.read(min(CHUNK, left))
                    if not b:
                        break
                    left -= len(b)
                    yield bytes(b)
            finally:
                f.close()
        return 200, {"Content-Type": "application/octet-stream", "Content-Length": str(n)}, chunks()

    def _create(self, path, q, host, body_iter):
        fs = self.fs
        if fs.exists(path):
            if not _bool(q.get("overwrite")):
                raise WebHdfsError(403, "FileAlreadyExistsException",
                                   "org.apache.hadoop.fs.FileAlreadyExistsException", f"{path} already exists")
            if fs.get_status(path).info.folder:
                raise WebHdfsError(403, "FileAlreadyExistsException",
                                   "org.apache.hadoop.fs.FileAlreadyExistsException", f"{path} is a directory")
            fs.delete(path)
        kw = {"write_type": self.write_type}
        if q.get("permission"):
            kw["mode"] = int(q["permission"], 8)
        if q.get("blocksize"):
            kw["block_size"] = int(q["blocksize"])
        parent = posixpath.dirname(path.rstrip("/")) or "/"
        if not fs.exists(parent):
            fs.create_directory(parent, recursive=True, allow_exists=True)
        out = fs.create_file(path, **kw)
        try:
            for chunk in body_iter():
                out.write(chunk)
        except BaseException:
            out.cancel() if hasattr(out, "cancel") else out.close()
            raise
        out.close()
        return 201, {"Location": f"webhdfs://{host}{urllib.parse.quote(path)}", "Content-Length": "0"}, b""

    def _summary(self, path) -> dict:
        st = self.fs.get_status(path)
        if not st.info.folder:
            n = int(st.info.length)
            return {"directoryCount": 0, "fileCount": 1, "length": n, "quota": -1, "spaceConsumed": n,
                    "spaceQuota": -1}
        dirs, files, length = 1, 0, 0
        for s in self.fs.list_status(path, recursive=True):
            if s.info.folder:
                dirs += 1
            else:
                files += 1
                length += int(s.info.length)
        return {"directoryCount": dirs, "fileCount": files, "length": length, "quota": -1,
                "spaceConsumed": length, "spaceQuota": -1}

    def _checksum(self, path) -> dict:
        """Hadoop's composite CRC file checksum (COMPOSITE-CRC32C, 4 bytes): the CRC32C of the file's
        bytes, independent of block and chunk sizes -- comparable across stores."""
        from ..ops.native import lib
        st = self.fs.get_status(path)
        if st.info.folder:
            raise WebHdfsError(404, "FileNotFoundException", "java.io.FileNotFoundException", f"{path} is a directory")
        crc_fn = lib().crc32c
        crc = 0
        with self.fs.open_file(path) as f:
            while True:
                b = f.read(CHUNK)
                if not b:
                    break
                crc = crc_fn(bytes(b), crc)            # chained: CRC32C of the concatenation
        return {"algorithm": "COMPOSITE-CRC32C", "bytes": format(crc, "08x"), "length": 4}
