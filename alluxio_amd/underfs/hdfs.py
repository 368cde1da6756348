"""HDFS UFS via ``pyarrow.fs.HadoopFileSystem`` (reference underfs/hdfs/.../HdfsUnderFileSystem.java).

libhdfs/JVM are not present in this image, so the factory only claims ``hdfs://`` URIs when
pyarrow can actually connect; otherwise ``create`` raises a clear error.  All operations map
one-to-one onto pyarrow's filesystem API.
"""
from __future__ import annotations

from .base import UfsDirectoryStatus, UfsFileStatus, UnderFileSystem
from .registry import UnderFileSystemFactory, register_factory


class HdfsUnderFileSystem(UnderFileSystem):
    scheme = "hdfs"
    ufs_type = "hdfs"

    def __init__(self, root_uri, conf=None, properties=None):
        super().__init__(root_uri, conf, properties)
        try:
            from pyarrow import fs as pafs
        except Exception as e:  # noqa: BLE001
            raise RuntimeError("pyarrow is required for hdfs:// UFS") from e
        self._pafs = pafs
        try:
            self.fs, _ = pafs.FileSystem.from_uri(root_uri)
        except Exception as e:  # noqa: BLE001
            raise RuntimeError(f"cannot connect to {root_uri}: {e} (libhdfs/JVM missing?)") from e

    def _p(self, path):
        if "://" in path:
            path = "/" + path.split("://", 1)[1].split("/", 1)[1]
        return path

    def create(self, path, options=None):
        return self.fs.open_output_stream(self._p(path))

    def open(self, path, options=None):
        f = self.fs.open_input_file(self._p(path))
        if options and options.offset:
            f.seek(options.offset)
        return f

    def _info(self, p):
        info = self.fs.get_file_info(p)
        return info if info.type != self._pafs.FileType.NotFound else None

    def delete_file(self, path):
        if self._info(self._p(path)) is None:
            return False
        self.fs.delete_file(self._p(path))
        return True

    def delete_directory(self, path, options=None):
        p = self._p(path)
        if self._info(p) is None:
            return False
        if options and options.recursive:
            self.fs.delete_dir(p)
        else:
            if self.fs.get_file_info(self._pafs.FileSelector(p)):
                return False
            self.fs.delete_dir(p)
        return True

    def get_status(self, path):
        info = self._info(self._p(path))
        if info is None:
            return None
        mt = int(info.mtime.timestamp() * 1000) if info.mtime else None
        if info.type == self._pafs.FileType.Directory:
            return UfsDirectoryStatus(info.base_name, last_modified_ms=mt)
        return UfsFileStatus(info.base_name, info.size, f"{info.size}:{mt}", mt)

    def list_status(self, path, options=None):
        p = self._p(path)
        if self._info(p) is None:
            return None
        sel = self._pafs.FileSelector(p, recursive=bool(options and options.recursive))
        out = []
        for info in self.fs.get_file_info(sel):
            rel = info.path[len(p.rstrip("/")) + 1:]
            mt = int(info.mtime.timestamp() * 1000) if info.mtime else None
            out.append(UfsDirectoryStatus(rel, last_modified_ms=mt) if info.type == self._pafs.FileType.Directory
                       else UfsFileStatus(rel, info.size, f"{info.size}:{mt}", mt))
        return out

    def mkdirs(self, path, options=None):
        p = self._p(path)
        if self._info(p) is not None:
            return False
        self.fs.create_dir(p, recursive=True)
        return True

    def rename_file(self, src, dst):
        self.fs.move(self._p(src), self._p(dst))
        return True

    rename_directory = rename_file


class _HdfsFactory(UnderFileSystemFactory):
    scheme = "hdfs"

    def create(self, uri, conf=None, properties=None):
        return HdfsUnderFileSystem(uri, conf, properties)


register_factory(_HdfsFactory())
