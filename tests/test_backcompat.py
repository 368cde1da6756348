"""Backwards compatibility with journals and backups written by the Java masters.

Reference: tests/src/main/java/alluxio/master/backcompat/BackwardsCompatibilityJournalGenerator.java
(OPS list :60-71; a 1-master cluster applies every op, takes a backup, then copies the UFS journal to
tests/src/test/resources/old_journals/{journal,backup}-<version>) and the ops' ``check`` methods in
tests/src/main/java/alluxio/master/backcompat/ops/*.java.  The fixtures under
``tests/fixtures/old_journals`` are the reference's own 1.8.0 artifacts (length-delimited
JournalEntry protobufs; the backup is the same stream gzip'ed), read with our protobuf parser only.

Each op's checks are replayed here against our master: once from the UFS journal directory (the Java
``_format_<ms>`` markers, no ``checkpoints/`` dir, no TableMaster dir, 1.x ``rename.dst_path``
entries) and once through ``alluxio.master.journal.init.from.backup``; each time the master is then
restarted on what it wrote to prove the replayed state is durable.  SetAcl is skipped as in the
reference (``supportsVersion >= 1.9``).
"""
import os
import shutil
from pathlib import Path

import pytest

from alluxio_amd.conf import Configuration
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.utils.exceptions import FileDoesNotExistException

FIXTURES = Path(__file__).parent / "fixtures" / "old_journals"
TTL = (2 ** 63 - 1) // 2          # Long.MAX_VALUE / 2
DELETE, FREE = 0, 1               # PTtlAction


def _start(journal_dir, root_ufs, backup=None):
    c = Configuration(load_site=False)
    c.set("alluxio.master.journal.type", "UFS")
    c.set("alluxio.master.journal.folder", str(journal_dir))
    c.set("alluxio.web.server.enabled", "false")
    if backup:
        c.set("alluxio.master.journal.init.from.backup", str(backup))
    m = AlluxioMasterProcess(c, port=0, enable_grpc=False, root_ufs=str(root_ufs))
    m.start(start_heartbeats=False)
    return m


def _exists(fs, p):
    try:
        fs.get_status(p)
        return True
    except FileDoesNotExistException:
        return False


def check_create_directory(fs):
    for d in ("/createDirectory", "/createDirectory/a", "/createDirectory/a/b", "/createDirectoryRecursive/a/b",
              "/createDirectoryMode/a", "/createDirectoryTtl/a", "/createDirectoryCommonTtl/a",
              "/createDirectoryThrough/a", "/createDirectoryAllOpts/a"):
        assert _exists(fs, d), d
    assert fs.get_status("/createDirectoryMode/a").mode == 0o713            # u=rwx,g=x,o=wx
    for d in ("/createDirectoryTtl/a", "/createDirectoryCommonTtl/a", "/createDirectoryAllOpts/a"):
        st = fs.get_status(d)
        assert (st.ttl, st.ttlAction) == (TTL, DELETE), d
    assert fs.get_status("/createDirectoryThrough/a").persisted
    st = fs.get_status("/createDirectoryAllOpts/a")
    assert st.mode == 0o713 and st.persisted


def check_create_file(fs):
    for f in ("/createFile", "/createFileNested/a", "/createFileThrough/a", "/createFileTtl/a"):
        assert _exists(fs, f), f
    assert fs.get_status("/createFileMode/a").mode == 0o610                 # u=rw,g=x
    assert fs.get_status("/createFileThrough/a").persisted
    st = fs.get_status("/createFileTtl/a")
    assert (st.ttl, st.ttlAction) == (TTL, FREE)
    st = fs.get_status("/createFile")
    assert st.completed and st.length == 4 and len(st.blockIds) == 1


def check_mount(fs):
    assert fs.get_status("/mount").mountPoint
    assert not _exists(fs, "/unmount")


def check_async_persist(fs):
    assert fs.get_status("/asyncPersist").persisted
    assert fs.get_status("/asyncPersistDir/nested").persisted
    assert fs.get_status("/asyncPersistDir").persisted


def check_delete(fs):
    for p in ("/pathToDelete", "/deleteFile/a", "/deleteRecursive/a/b"):
        assert not _exists(fs, p), p
    assert _exists(fs, "/deleteFile")
    assert not _exists(fs, "/deleteRecursive/a")
    assert _exists(fs, "/deleteRecursive")


def check_persist_file(fs):
    for p in ("/fileToPersist", "/persistFileDir/a", "/persistFileDir"):
        assert fs.get_status(p).persisted, p


def check_persist_directory(fs):
    assert fs.get_status("/dirToPersist").persisted
    assert fs.get_status("/dirToPersist/innerFile").persisted


def check_rename(fs):
    assert not _exists(fs, "/fileToRename")
    assert _exists(fs, "/fileRenameTarget")
    assert not _exists(fs, "/renameDir/a")
    assert _exists(fs, "/renameDir/c")
    assert _exists(fs, "/renameDir/c/b")


CHECKS = [check_create_directory, check_create_file, check_mount, check_async_persist, check_delete,
          check_persist_file, check_persist_directory, check_rename]


def _check_all(m):
    for check in CHECKS:
        check(m.fs_master)
    # BlockMaster: container id generator and the surviving blocks (3 of 14 were deleted)
    bm = m.block_master
    assert bm._next_container >= 1000
    assert len(bm._blocks) == 11


@pytest.fixture
def mount_dir():
    # the Mount op recorded this UFS path (Mount.java LOCAL_FS_MOUNT_DIR)
    os.makedirs("/tmp/alluxioTest/mount", exist_ok=True)


@pytest.mark.parametrize("source", ["journal", "backup"])
def test_replay_1_8_0(tmp_path, mount_dir, source):
    jdir = tmp_path / "journal"
    backup = None
    if source == "journal":
        shutil.copytree(FIXTURES / "journal-1.8.0", jdir)
    else:
        backup = FIXTURES / "backup-1.8.0"
    m = _start(jdir, tmp_path / "ufs", backup)
    try:
        _check_all(m)
        # new namespace ops append to the old journal
        m.fs_master.create_directory("/afterUpgrade")
    finally:
        m.stop()
    m = _start(jdir, tmp_path / "ufs")     # restart on what was written (no backup key)
    try:
        _check_all(m)
        assert _exists(m.fs_master, "/afterUpgrade")
    finally:
        m.stop()


def test_fresh_format_writes_java_marker(tmp_path):
    """A journal we format carries the ``_format_<ms>`` marker Java masters look for
    (UfsJournal.isFormatted), so a Java tool accepts it as formatted."""
    m = _start(tmp_path / "j", tmp_path / "ufs")
    m.stop()
    for master in ("BlockMaster", "FileSystemMaster", "MetaMaster"):
        names = os.listdir(tmp_path / "j" / master / "v1")
        assert any(n.startswith("_format_") for n in names), (master, names)
