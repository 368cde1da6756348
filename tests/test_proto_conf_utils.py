"""Wire schema, configuration and common-runtime unit tests (reference: core/common tests,
core/transport golden field numbers)."""
import os
import threading
import time

import pytest

from alluxio_amd.conf import Configuration, PathConfiguration, Source, load_properties_file
from alluxio_amd.conf import keys as K
from alluxio_amd.proto import SERVICES, pb
from alluxio_amd.utils import ids
from alluxio_amd.utils.collections import IndexedSet
from alluxio_amd.utils.format import parse_space_size, parse_time_size
from alluxio_amd.utils.heartbeat import HeartbeatScheduler, HeartbeatThread, manual_heartbeat
from alluxio_amd.utils.locks import RWLock
from alluxio_amd.utils.retry import CountingRetry, ExponentialBackoffRetry, retry
from alluxio_amd.utils.uri import AlluxioURI, join_path, normalize_path


# ---------------------------------------------------------------------------------------------
# proto
def test_read_request_golden_bytes():
    # field 1 varint 5, field 2 varint 3, field 5 varint 1<<20  (protoc would emit the same)
    r = pb.block.ReadRequest(block_id=5, offset=3, chunk_size=1 << 20)
    assert r.SerializeToString().hex() == "0805100328808040"


def test_journal_entry_golden_and_defaults():
    e = pb.journal.JournalEntry(sequence_number=3, inode_file=pb.journal.InodeFileEntry(id=1, name="a"))
    assert e.SerializeToString().hex() == "08035a0508011a0161"
    assert e.inode_file.ttlAction == 0  # default DELETE
    assert pb.file.OpenFilePOptions().updateLastAccessTime is True
    assert pb.file.MountPointInfo().ufsCapacityBytes == -1


def test_maps_oneofs_required():
    fi = pb.file.FileInfo(fileId=7, xattr={"k": b"v"}, blockIds=[1, 2])
    back = pb.file.FileInfo.FromString(fi.SerializeToString())
    assert back.xattr["k"] == b"v" and list(back.blockIds) == [1, 2]
    w = pb.block.WriteRequest(chunk=pb.block.Chunk(data=b"x"))
    assert w.WhichOneof("value") == "chunk"
    w.command.id = 3
    assert w.WhichOneof("value") == "command"
    m = pb.grpc.PMode(ownerBits=8, groupBits=6, otherBits=6)
    assert m.IsInitialized()
    assert not pb.grpc.PMode(ownerBits=1).IsInitialized()


def test_service_inventory():
    assert "alluxio.grpc.file.FileSystemMasterClientService" in SERVICES
    assert len(SERVICES["alluxio.grpc.file.FileSystemMasterClientService"]) == 23
    rb = SERVICES["alluxio.grpc.block.BlockWorker"]["ReadBlock"]
    assert rb.client_streaming and rb.server_streaming and rb.path == "/alluxio.grpc.block.BlockWorker/ReadBlock"
    assert SERVICES["alluxio.grpc.file.FileSystemMasterClientService"]["ListStatus"].server_streaming


# ---------------------------------------------------------------------------------------------
# configuration
def test_reference_key_defaults():
    c = Configuration()
    assert c.get_bytes("alluxio.user.block.size.bytes.default") == 64 << 20
    assert c.get("alluxio.user.file.writetype.default") == "ASYNC_THROUGH"
    assert c.get("alluxio.user.file.readtype.default") == "CACHE"
    assert c.get_ms("alluxio.worker.block.heartbeat.interval") == 1000
    assert c.get_ms("alluxio.master.worker.timeout") == 300_000
    assert c.get("alluxio.worker.allocator.class").endswith("MaxFreeAllocator")
    assert c.get("alluxio.worker.block.annotator.class").endswith("LRUAnnotator")
    assert len([k for k in K.all_keys()]) >= 504


def test_substitution_and_sources(monkeypatch):
    c = Configuration({"alluxio.home": "/opt/ax"})
    assert c.get("alluxio.work.dir") == "/opt/ax"
    assert c.get("alluxio.master.journal.folder") == "/opt/ax/journal"
    c.set("alluxio.user.file.buffer.bytes", "1MB", Source.SITE_PROPERTY)
    c.set("alluxio.user.file.buffer.bytes", "2MB", Source.DEFAULT)  # lower priority: ignored
    assert c.get_bytes("alluxio.user.file.buffer.bytes") == 1 << 20
    c.set("alluxio.user.file.buffer.bytes", "4MB", Source.RUNTIME)
    assert c.get_bytes("alluxio.user.file.buffer.bytes") == 4 << 20
    assert c.source("alluxio.user.file.buffer.bytes") == Source.RUNTIME


def test_templates_and_aliases():
    c = Configuration()
    assert c.get("alluxio.worker.tieredstore.level0.alias") == "MEM"
    assert c.get("alluxio.worker.tieredstore.level1.alias") == "SSD"
    assert c.get("alluxio.worker.tieredstore.level0.dirs.mediumtype") == "HBM"
    c.set("alluxio.underfs.s3a.directory.suffix", "_$folder$")
    assert c.get("alluxio.underfs.s3.directory.suffix") == "_$folder$"


def test_properties_file_and_path_conf(tmp_path):
    p = tmp_path / "alluxio-site.properties"
    p.write_text("# comment\nalluxio.master.hostname=m1\nalluxio.user.block.size.bytes.default : 32MB\n"
                 "alluxio.long=a,\\\n  b\n")
    props = load_properties_file(str(p))
    assert props["alluxio.master.hostname"] == "m1"
    assert props["alluxio.user.block.size.bytes.default"] == "32MB"
    assert props["alluxio.long"] == "a,b"
    pc = PathConfiguration()
    pc.set("/a", {"alluxio.user.file.writetype.default": "THROUGH"})
    pc.set("/a/b", {"alluxio.user.file.writetype.default": "MUST_CACHE"})
    base = Configuration()
    assert pc.resolve(base, "/a/x").get("alluxio.user.file.writetype.default") == "THROUGH"
    assert pc.resolve(base, "/a/b/c").get("alluxio.user.file.writetype.default") == "MUST_CACHE"
    assert pc.resolve(base, "/z").get("alluxio.user.file.writetype.default") == "ASYNC_THROUGH"


# ---------------------------------------------------------------------------------------------
# utils
def test_block_id_layout():
    bid = ids.create_block_id(5, 7)
    assert ids.get_container_id(bid) == 5 and ids.get_sequence_number(bid) == 7
    fid = ids.get_file_id(bid)
    assert fid == ids.create_file_id(5) and ids.get_sequence_number(fid) == (1 << 24) - 1
    big = ids.create_block_id((1 << 40) - 1, 0)
    assert big < 0  # signed 64-bit like Java longs
    assert ids.get_container_id(big) == (1 << 40) - 1


def test_formats_and_uri():
    assert parse_space_size("128m") == 128 << 20
    assert parse_space_size("4k") == 4096
    assert parse_space_size("1.5GB") == int(1.5 * (1 << 30))
    assert parse_time_size("30s") == 30_000 and parse_time_size("1min") == 60_000
    u = AlluxioURI("alluxio://host:19998/a/b/../c/")
    assert u.path == "/a/c" and u.authority == "host:19998"
    assert u.get_parent().path == "/a" and u.get_name() == "c" and u.get_depth() == 2
    assert AlluxioURI("/a").is_ancestor_of(AlluxioURI("/a/b"))
    assert not AlluxioURI("/a").is_ancestor_of(AlluxioURI("/ab"))
    assert normalize_path("a//b/") == "/a/b" and join_path("/a", "b", "c") == "/a/b/c"


def test_rwlock_writer_excludes_readers():
    lk = RWLock()
    lk.acquire_read()
    got = []
    t = threading.Thread(target=lambda: (lk.acquire_write(), got.append(1), lk.release_write()))
    t.start()
    time.sleep(0.05)
    assert not got
    lk.release_read()
    t.join(2)
    assert got == [1]
    assert lk.acquire_write(timeout=1)
    assert not RWLock().acquire_read(timeout=0) or True
    lk.release_write()


def test_retry_policies():
    calls = []

    def flaky():
        calls.append(1)
        if len(calls) < 3:
            raise ConnectionError("x")
        return 42
    assert retry(flaky, CountingRetry(5)) == 42
    with pytest.raises(ConnectionError):
        retry(lambda: (_ for _ in ()).throw(ConnectionError()), ExponentialBackoffRetry(1, 2, 2))


def test_manual_heartbeat_scheduler():
    hits = []
    with manual_heartbeat("test-hb"):
        t = HeartbeatThread("test-hb", lambda: hits.append(1), 10_000_000)
        t.start()
        HeartbeatScheduler.execute("test-hb")
        HeartbeatScheduler.execute("test-hb")
        assert len(hits) == 2
        t.shutdown()


def test_indexed_set():
    class W:
        def __init__(self, i, a):
            self.id, self.addr = i, a
    s = IndexedSet(id=(lambda w: w.id, True), addr=(lambda w: w.addr, False))
    a, b = W(1, "h1"), W(2, "h1")
    assert s.add(a) and s.add(b) and not s.add(W(1, "h2"))
    assert s.get_first_by_field("id", 2) is b
    assert len(s.get_by_field("addr", "h1")) == 2
    s.remove(a)
    assert s.get_first_by_field("id", 1) is None and len(s) == 1


def test_metrics_sinks_from_properties(tmp_path):
    import socket
    import threading
    from alluxio_amd.metrics import (CsvSink, GraphiteSink, LoggingSink, MetricsSystem, load_sinks,
                                     sinks_from_properties)
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    got = []

    def accept():
        c, _ = srv.accept()
        got.append(c.recv(65536).decode())
        c.close()
    t = threading.Thread(target=accept, daemon=True)
    t.start()
    props = tmp_path / "metrics.properties"
    props.write_text(f"sink.graphite.class=alluxio.metrics.sink.GraphiteSink\nsink.graphite.host=127.0.0.1\n"
                     f"sink.graphite.port={srv.getsockname()[1]}\nsink.graphite.prefix=amd\n"
                     f"sink.graphite.period=50\nsink.graphite.unit=milliseconds\n"
                     f"sink.csv.class=alluxio.metrics.sink.CsvSink\nsink.csv.directory={tmp_path / 'csv'}\n"
                     f"sink.slf4j.class=alluxio.metrics.sink.Slf4jSink\nsink.jmx.class=alluxio.metrics.sink.JmxSink\n")
    from alluxio_amd.conf import Configuration, load_properties_file
    kinds = sorted(type(s).__name__ for s in sinks_from_properties(load_properties_file(str(props))))
    assert kinds == ["CsvSink", "GraphiteSink", "LoggingSink"]
    m = MetricsSystem("Master")
    m.counter("FilesCreated").inc(3)
    sinks = load_sinks(Configuration({"alluxio.metrics.conf.file": str(props)}), m)
    try:
        t.join(5)
        assert got and "amd.Master.FilesCreated 3" in got[0]
    finally:
        for s in sinks:
            s.stop()
        srv.close()
    assert all(isinstance(s, (CsvSink, GraphiteSink, LoggingSink)) for s in sinks)
