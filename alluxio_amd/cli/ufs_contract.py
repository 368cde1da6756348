"""``alluxio runUfsTests --path <ufs-uri>``: the under-storage contract test runner.

Parity: integration/tools/validation/src/main/java/alluxio/cli/UnderFileSystemContractTest.java
(runner: one fresh test directory per operation, cleanup after each, pass/fail summary, exit code),
UnderFileSystemCommonOperations.java (the common operation list: create / open / delete / exists /
status / list / mkdirs / object common prefixes / rename, each with its large-directory variant)
and S3ASpecificOperations.java (multipart streams: empty, less than one part, several parts).

The operations drive only the public :class:`underfs.base.UnderFileSystem` API, so the same run
checks any connector registered with :mod:`underfs.registry` (local, S3 family, WebHDFS, Swift,
WASB, Ozone, web, ...) against the semantics the master and workers rely on.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
import traceback
import uuid

from ..underfs import registry
from ..underfs.base import CreateOptions, DeleteOptions, ListOptions, MkdirsOptions, OpenOptions

LARGE_FILE_SIZE = 20 << 20      # the reference writes 20 MB-ish "large" files
LARGE_DIR_FILES = 100           # files per large-directory operation (reference: 100 children)
TEST_BYTES = b"contract-test-bytes-0123456789"


class ContractFailure(AssertionError):
    pass


def _check(cond: bool, msg: str) -> None:
    if not cond:
        raise ContractFailure(msg)


def _join(base: str, *parts: str) -> str:
    return "/".join([base.rstrip("/")] + [p.strip("/") for p in parts])


def _write(ufs, path: str, data: bytes, **opts) -> None:
    with ufs.create(path, CreateOptions(**opts) if opts else None) as f:
        if data:
            f.write(data)


def _read(ufs, path: str, offset: int = 0) -> bytes:
    with ufs.open(path, OpenOptions(offset=offset)) as f:
        out = bytearray()
        while True:
            b = f.read(1 << 20)
            if not b:
                return bytes(out)
            out += b


def _pattern(n: int) -> bytes:
    """Deterministic non-trivial content (the reference writes an int sequence)."""
    block = bytes(range(256)) * 4096
    reps, rem = divmod(n, len(block))
    return block * reps + block[:rem]


def _names(statuses) -> set[str]:
    return {s.name.rstrip("/") for s in (statuses or [])}


class CommonOperations:
    """One method per reference operation; ``self.dir`` is a fresh directory per test."""

    def __init__(self, ufs, test_dir: str):
        self.ufs = ufs
        self.dir = test_dir

    def p(self, *parts: str) -> str:
        return _join(self.dir, *parts)

    # ---- create / open -----------------------------------------------------------------------
    def create_atomic_test(self):
        path = self.p("createAtomic")
        f = self.ufs.create(path, CreateOptions(ensure_atomic=True))
        f.write(TEST_BYTES)
        _check(not self.ufs.is_file(path), "atomic create is visible before close")
        f.close()
        _check(self.ufs.is_file(path), "atomic create is not visible after close")

    def create_empty_test(self):
        path = self.p("createEmpty")
        _write(self.ufs, path, b"")
        _check(self.ufs.is_file(path), "empty file was not created")
        _check(self.ufs.get_file_status(path).content_length == 0, "empty file has non-zero length")

    def create_no_parent_test(self):
        path = self.p("testDir", "createNoParent")
        try:
            f = self.ufs.create(path, CreateOptions(create_parent=False))
            f.write(TEST_BYTES)
            f.close()
        except Exception:  # noqa: BLE001 - the expected outcome on file systems with directories
            return
        # object stores have no real parents: the object exists without one (reference accepts it)
        _check(self.ufs.is_object_storage(), "create without parent succeeded on a non-object store")

    def create_parent_test(self):
        path = self.p("testDir", "createParent")
        _write(self.ufs, path, TEST_BYTES, create_parent=True)
        _check(self.ufs.is_file(path), "file with created parent does not exist")

    def create_open_test(self):
        path = self.p("createOpen")
        _write(self.ufs, path, TEST_BYTES)
        _check(_read(self.ufs, path) == TEST_BYTES, "read bytes differ from written bytes")

    def create_open_empty_test(self):
        path = self.p("createOpenEmpty")
        _write(self.ufs, path, b"")
        _check(_read(self.ufs, path) == b"", "empty file read returned bytes")

    def create_open_at_position_test(self):
        path = self.p("createOpenAtPosition")
        data = _pattern(1 << 16)
        _write(self.ufs, path, data)
        for off in (0, 1, 4095, 1 << 15, len(data) - 1):
            _check(_read(self.ufs, path, off) == data[off:], f"read at offset {off} differs")

    def create_open_large_test(self):
        path = self.p("createOpenLarge")
        data = _pattern(LARGE_FILE_SIZE)
        _write(self.ufs, path, data)
        got = _read(self.ufs, path)
        _check(len(got) == len(data) and got == data, "large file contents differ")

    def create_open_existing_large_file_test(self):
        path = self.p("createOpenExistingLarge")
        data = _pattern(LARGE_FILE_SIZE)
        _write(self.ufs, path, data)
        with self.ufs.open_existing_file(path) as f:
            head = f.read(1 << 20)
        _check(head == data[:len(head)] and len(head) > 0, "open_existing_file read differs")

    # ---- delete ------------------------------------------------------------------------------
    def delete_file_test(self):
        path = self.p("deleteFile")
        _write(self.ufs, path, TEST_BYTES)
        _check(self.ufs.delete_file(path), "delete_file returned false")
        _check(not self.ufs.is_file(path), "deleted file still exists")

    def delete_dir_test(self):
        d = self.p("deleteDir")
        child = _join(d, "child")
        self.ufs.mkdirs(child, MkdirsOptions(create_parent=True))
        _write(self.ufs, _join(d, "file"), TEST_BYTES)
        _write(self.ufs, _join(child, "file"), TEST_BYTES)
        _check(not self.ufs.delete_directory(d, DeleteOptions(recursive=False)),
               "non-recursive delete of a non-empty directory succeeded")
        _check(self.ufs.is_directory(d), "directory vanished after a refused delete")
        _check(self.ufs.delete_directory(d, DeleteOptions(recursive=True)), "recursive delete failed")
        _check(not self.ufs.exists(d) and not self.ufs.exists(_join(child, "file")),
               "recursively deleted paths still exist")

    def delete_large_directory_test(self):
        d = self.p("deleteLargeDir")
        paths = self._large_directory(d)
        _check(self.ufs.delete_directory(d, DeleteOptions(recursive=True)), "large directory delete failed")
        for p in paths[:: max(1, len(paths) // 10)]:
            _check(not self.ufs.exists(p), f"{p} still exists after delete")

    def create_delete_file_conjuction_test(self):
        path = self.p("createDeleteConj")
        _write(self.ufs, path, TEST_BYTES)
        _check(self.ufs.delete_existing_file(path), "delete_existing_file failed")
        _write(self.ufs, path, TEST_BYTES + b"2")
        _check(_read(self.ufs, path) == TEST_BYTES + b"2", "re-created file has stale contents")

    def create_then_delete_existing_directory_test(self):
        d = self.p("createThenDeleteDir")
        self.ufs.mkdirs(d)
        _check(self.ufs.delete_existing_directory(d, DeleteOptions()), "delete_existing_directory failed")
        _check(not self.ufs.is_directory(d), "deleted directory still exists")

    # ---- exists / status ---------------------------------------------------------------------
    def exists_test(self):
        f, d = self.p("existsFile"), self.p("existsDir")
        _check(not self.ufs.exists(f) and not self.ufs.exists(d), "paths exist before creation")
        _write(self.ufs, f, TEST_BYTES)
        self.ufs.mkdirs(d)
        _check(self.ufs.exists(f) and self.ufs.exists(d), "created paths do not exist")

    def get_directory_status_test(self):
        d = self.p("dirStatus")
        self.ufs.mkdirs(d)
        st = self.ufs.get_status(d)
        _check(st is not None and st.is_directory, "directory status is not a directory")

    def create_then_get_existing_directory_status_test(self):
        d = self.p("dirStatusExisting")
        self.ufs.mkdirs(d)
        _check(self.ufs.get_existing_status(d).is_directory, "existing directory status wrong")
        _check(self.ufs.get_directory_status(d).is_directory, "get_directory_status wrong")

    def get_file_size_test(self):
        path = self.p("fileSize")
        data = _pattern(12345)
        _write(self.ufs, path, data)
        _check(self.ufs.get_file_status(path).content_length == len(data), "file size differs")

    def create_then_get_existing_file_status_test(self):
        path = self.p("fileStatusExisting")
        _write(self.ufs, path, TEST_BYTES)
        st = self.ufs.get_existing_status(path)
        _check(st.is_file and st.content_length == len(TEST_BYTES), "existing file status wrong")

    def get_file_status_test(self):
        path = self.p("fileStatus")
        _write(self.ufs, path, TEST_BYTES)
        st = self.ufs.get_file_status(path)
        _check(st.is_file and st.content_length == len(TEST_BYTES), "file status wrong")

    def create_then_get_existing_status_test(self):
        path = self.p("statusExisting")
        _write(self.ufs, path, TEST_BYTES)
        _check(self.ufs.get_existing_status(path).is_file, "existing status of a file is not a file")

    def get_mod_time_test(self):
        path = self.p("modTime")
        t0 = int(time.time() * 1000)
        _write(self.ufs, path, TEST_BYTES)
        m = self.ufs.get_file_status(path).last_modified_ms
        t1 = int(time.time() * 1000)
        # object stores report second granularity: allow a few seconds of slack either way
        _check(m is not None and t0 - 5000 <= m <= t1 + 5000, f"mod time {m} outside [{t0}, {t1}]")

    def get_non_existing_directory_status_test(self):
        self._expect_missing(self.p("missingDir") + "/")

    def get_non_existing_file_status_test(self):
        self._expect_missing(self.p("missingFile"))

    def get_non_existing_path_status_test(self):
        self._expect_missing(self.p("missing", "deep", "path"))

    def _expect_missing(self, path: str) -> None:
        _check(self.ufs.get_status(path.rstrip("/")) is None, f"{path} has a status")
        _check(not self.ufs.exists(path.rstrip("/")), f"{path} exists")

    def is_file_test(self):
        f, d = self.p("isFile"), self.p("isFileDir")
        _check(not self.ufs.is_file(f), "missing path is a file")
        _write(self.ufs, f, TEST_BYTES)
        self.ufs.mkdirs(d)
        _check(self.ufs.is_file(f) and not self.ufs.is_file(d), "is_file wrong")
        _check(self.ufs.is_directory(d) and not self.ufs.is_directory(f), "is_directory wrong")

    # ---- list --------------------------------------------------------------------------------
    def list_status_test(self):
        d = self.p("list")
        self.ufs.mkdirs(_join(d, "sub"))
        _write(self.ufs, _join(d, "a"), TEST_BYTES)
        _write(self.ufs, _join(d, "b"), TEST_BYTES)
        _write(self.ufs, _join(d, "sub", "c"), TEST_BYTES)
        got = self.ufs.list_status(d)
        _check(_names(got) == {"a", "b", "sub"}, f"listing {sorted(_names(got))}")
        by = {s.name.rstrip("/"): s for s in got}
        _check(by["sub"].is_directory and by["a"].is_file, "listing kinds wrong")

    def list_status_empty_test(self):
        d = self.p("listEmpty")
        self.ufs.mkdirs(d)
        _check(self.ufs.list_status(d) == [], "empty directory listing is not empty")

    def list_status_file_test(self):
        path = self.p("listFile")
        _write(self.ufs, path, TEST_BYTES)
        _check(self.ufs.list_status(path) is None, "listing a file did not return None")

    def list_large_directory_test(self):
        d = self.p("listLarge")
        paths = self._large_directory(d)
        got = self.ufs.list_status(d)
        _check(_names(got) == {os.path.basename(p) for p in paths}, "large listing incomplete")

    def list_status_recursive_test(self):
        d = self.p("listRecursive")
        for sub in ("x/y/z", "x/w", "v"):
            self.ufs.mkdirs(_join(d, sub), MkdirsOptions(create_parent=True))
        for f in ("x/f1", "x/y/f2", "x/y/z/f3", "v/f4", "f5"):
            _write(self.ufs, _join(d, f), TEST_BYTES)
        got = self.ufs.list_status(d, ListOptions(recursive=True))
        want = {"x", "x/y", "x/y/z", "x/w", "v", "x/f1", "x/y/f2", "x/y/z/f3", "v/f4", "f5"}
        _check(_names(got) == want, f"recursive listing {sorted(_names(got))}")

    def mkdirs_test(self):
        d = self.p("mkdirs", "a", "b")
        _check(not self.ufs.mkdirs(d, MkdirsOptions(create_parent=False)) or self.ufs.is_object_storage(),
               "mkdirs without parents succeeded on a non-object store")
        _check(self.ufs.mkdirs(d, MkdirsOptions(create_parent=True)), "mkdirs with parents failed")
        _check(self.ufs.is_directory(d) and self.ufs.is_directory(self.p("mkdirs", "a")), "mkdirs missing dirs")

    # ---- object stores: common prefixes count as directories -----------------------------------
    def _object_only(self) -> bool:
        return self.ufs.is_object_storage()

    def object_common_prefixes_is_directory_test(self):
        if not self._object_only():
            return
        _write(self.ufs, self.p("prefix", "child"), TEST_BYTES)
        _check(self.ufs.is_directory(self.p("prefix")), "common prefix is not a directory")

    def object_common_prefixes_list_status_non_recursive_test(self):
        if not self._object_only():
            return
        for f in ("a/x", "a/y", "b/z", "c"):
            _write(self.ufs, self.p("cp", f), TEST_BYTES)
        _check(_names(self.ufs.list_status(self.p("cp"))) == {"a", "b", "c"}, "prefix listing wrong")

    def object_common_prefixes_list_status_recursive_test(self):
        if not self._object_only():
            return
        for f in ("a/x", "a/b/y"):
            _write(self.ufs, self.p("cpr", f), TEST_BYTES)
        got = _names(self.ufs.list_status(self.p("cpr"), ListOptions(recursive=True)))
        _check(got == {"a", "a/x", "a/b", "a/b/y"}, f"recursive prefix listing {sorted(got)}")

    def object_nested_dirs_list_status_recursive_test(self):
        if not self._object_only():
            return
        self.ufs.mkdirs(self.p("nested", "d1", "d2"), MkdirsOptions(create_parent=True))
        _write(self.ufs, self.p("nested", "d1", "d2", "f"), TEST_BYTES)
        got = _names(self.ufs.list_status(self.p("nested"), ListOptions(recursive=True)))
        _check(got == {"d1", "d1/d2", "d1/d2/f"}, f"nested listing {sorted(got)}")

    # ---- rename ------------------------------------------------------------------------------
    def rename_file_test(self):
        src, dst = self.p("renameSrc"), self.p("renameDst")
        _write(self.ufs, src, TEST_BYTES)
        _check(self.ufs.rename_file(src, dst), "rename_file failed")
        _check(not self.ufs.exists(src) and _read(self.ufs, dst) == TEST_BYTES, "renamed file wrong")

    def rename_renamable_file_test(self):
        src, dst = self.p("renamableSrc"), self.p("renamableDst")
        _write(self.ufs, src, TEST_BYTES)
        _check(self.ufs.rename_renamable_file(src, dst), "rename_renamable_file failed")
        _check(self.ufs.is_file(dst) and not self.ufs.is_file(src), "renamed file wrong")

    def rename_directory_test(self):
        src, dst = self.p("renameDirSrc"), self.p("renameDirDst")
        _write(self.ufs, _join(src, "f1"), TEST_BYTES, create_parent=True)
        _write(self.ufs, _join(src, "f2"), TEST_BYTES, create_parent=True)
        _check(self.ufs.rename_directory(src, dst), "rename_directory failed")
        _check(not self.ufs.exists(src), "source directory still exists")
        _check(_names(self.ufs.list_status(dst)) == {"f1", "f2"}, "renamed directory contents wrong")

    def rename_directory_deep_test(self):
        src, dst = self.p("deepSrc"), self.p("deepDst")
        for f in ("f", "a/f", "a/b/f"):
            _write(self.ufs, _join(src, f), TEST_BYTES, create_parent=True)
        _check(self.ufs.rename_directory(src, dst), "deep rename failed")
        for f in ("f", "a/f", "a/b/f"):
            _check(_read(self.ufs, _join(dst, f)) == TEST_BYTES, f"{f} missing after deep rename")
            _check(not self.ufs.exists(_join(src, f)), f"{f} left behind by deep rename")

    def rename_renamable_directory_test(self):
        src, dst = self.p("renamableDirSrc"), self.p("renamableDirDst")
        _write(self.ufs, _join(src, "a", "f"), TEST_BYTES, create_parent=True)
        _check(self.ufs.rename_renamable_directory(src, dst), "rename_renamable_directory failed")
        _check(self.ufs.is_file(_join(dst, "a", "f")), "renamed directory contents wrong")

    def rename_large_directory_test(self):
        src, dst = self.p("renameLargeSrc"), self.p("renameLargeDst")
        paths = self._large_directory(src)
        _check(self.ufs.rename_directory(src, dst), "large directory rename failed")
        got = _names(self.ufs.list_status(dst))
        _check(got == {os.path.basename(p) for p in paths}, "large directory rename lost children")

    # ---- helpers -----------------------------------------------------------------------------
    def _large_directory(self, d: str) -> list[str]:
        self.ufs.mkdirs(d, MkdirsOptions(create_parent=True))
        paths = []
        for i in range(LARGE_DIR_FILES):
            p = _join(d, f"file{i}")
            _write(self.ufs, p, b"" if i % 2 else TEST_BYTES)
            paths.append(p)
        return paths


class S3ASpecificOperations:
    """Multipart-upload streams of the S3 connectors (reference: S3ASpecificOperations)."""

    def __init__(self, ufs, test_dir: str):
        self.ufs = ufs
        self.dir = test_dir

    @staticmethod
    def applies(ufs) -> bool:
        return hasattr(ufs, "multipart_threshold")

    def _with_part_size(self, size: int):
        old = self.ufs.multipart_threshold
        self.ufs.multipart_threshold = size
        return old

    def create_empty_file_test(self):
        path = _join(self.dir, "mpEmpty")
        old = self._with_part_size(1 << 20)
        try:
            _write(self.ufs, path, b"")
        finally:
            self.ufs.multipart_threshold = old
        _check(self.ufs.get_file_status(path).content_length == 0, "multipart empty file not empty")

    def create_file_less_than_one_part_test(self):
        path = _join(self.dir, "mpSmall")
        data = _pattern((1 << 20) - 7)
        old = self._with_part_size(1 << 20)
        try:
            _write(self.ufs, path, data)
        finally:
            self.ufs.multipart_threshold = old
        _check(_read(self.ufs, path) == data, "sub-part multipart file differs")

    def create_multipart_file_test(self):
        path = _join(self.dir, "mpLarge")
        data = _pattern((5 << 20) * 2 + 12345)
        old = self._with_part_size(5 << 20)
        try:
            _write(self.ufs, path, data)
        finally:
            self.ufs.multipart_threshold = old
        _check(_read(self.ufs, path) == data, "multipart file differs")


def _tests(cls) -> list[str]:
    return [n for n in vars(cls) if n.endswith("_test") and callable(getattr(cls, n))]


def run(path: str, test: str | None = None, properties: dict | None = None, out=None,
        large_file_size: int | None = None) -> dict:
    """Run the contract operations against the UFS at ``path``; returns the summary dict."""
    global LARGE_FILE_SIZE
    out = out or sys.stdout
    if large_file_size is not None:
        LARGE_FILE_SIZE = large_file_size
    ufs = registry.create(path, properties=properties or {})
    root = _join(path, f"alluxio-ufs-contract-{uuid.uuid4().hex[:12]}")
    suites = [(CommonOperations, _tests(CommonOperations))]
    if S3ASpecificOperations.applies(ufs):
        suites.append((S3ASpecificOperations, _tests(S3ASpecificOperations)))
    passed, failed = [], []
    try:
        for cls, names in suites:
            for name in names:
                if test and test != name:
                    continue
                d = _join(root, name)
                ufs.mkdirs(d, MkdirsOptions(create_parent=True))
                print(f"Running test: {cls.__name__}#{name}...", file=out)
                t0 = time.perf_counter()
                try:
                    getattr(cls(ufs, d), name)()
                    passed.append(name)
                    print(f"Passed the test! time: {(time.perf_counter() - t0) * 1e3:.0f}ms", file=out)
                except Exception as e:  # noqa: BLE001 - a failing operation is a result, not a crash
                    failed.append({"test": name, "error": f"{type(e).__name__}: {e}"})
                    print(f"Test {name} failed: {type(e).__name__}: {e}", file=out)
                    if not isinstance(e, ContractFailure):
                        traceback.print_exc(file=out)
                finally:
                    try:
                        ufs.delete_directory(d, DeleteOptions(recursive=True))
                    except Exception:  # noqa: BLE001
                        pass
    finally:
        try:
            ufs.delete_directory(root, DeleteOptions(recursive=True))
        except Exception:  # noqa: BLE001
            pass
    print(f"Tests completed with {len(passed)} passed and {len(failed)} failed.", file=out)
    return {"ufs": path, "passed": passed, "failed": failed}


def main(argv=None, out=None) -> int:
    ap = argparse.ArgumentParser(prog="alluxio runUfsTests",
                                 description="Test the under storage against Alluxio's UFS contract")
    ap.add_argument("--path", required=True, help="UFS URI to test in (a scratch directory)")
    ap.add_argument("--test", default=None, help="run only this operation (e.g. create_open_test)")
    ap.add_argument("--large-file-size", default=None, type=int, help="bytes of the 'large' files")
    ap.add_argument("-D", dest="props", action="append", default=[], help="key=value UFS property")
    a = ap.parse_args(argv)
    props = dict(kv.split("=", 1) for kv in a.props)
    res = run(a.path, a.test, props, out, a.large_file_size)
    return 0 if not res["failed"] else 1
