"""Native framed-RPC front end of the master (rpc/native.py, csrc/frame_rpc.cpp): round trips,
the epoch-versioned native reply cache, and group-commit replies deferred to the journal flush
(reference behaviour being matched: DefaultFileSystemMaster RPCs return only after
``JournalContext.close()`` flushed their entries, MasterJournalContext.java:35-93)."""
import threading
import time

import pytest

from alluxio_amd.conf import Configuration
from alluxio_amd.journal.system import AsyncJournalWriter, deferred_flush
from alluxio_amd.master.process import AlluxioMasterProcess
from alluxio_amd.proto import pb
from alluxio_amd.rpc import Channel
from alluxio_amd.utils import exceptions as ex

FS = "alluxio.grpc.file.FileSystemMasterClientService"


@pytest.fixture
def master(tmp_path):
    conf = Configuration({"alluxio.master.journal.folder": str(tmp_path / "journal"),
                          "alluxio.master.journal.type": "UFS",
                          "alluxio.master.web.port": "0",
                          "alluxio.security.authorization.permission.enabled": "false"})
    m = AlluxioMasterProcess(conf, host="127.0.0.1", port=0, root_ufs=str(tmp_path / "ufs"))
    addr = m.start(start_heartbeats=False)
    ch = Channel(addr, force_grpc=True)
    stub = ch.stub(FS)
    yield m, stub
    m.stop()


def _status(stub, path, **common):
    req = pb.file.GetStatusPRequest(path=path)
    for k, v in common.items():
        setattr(req.options.commonOptions, k, v)
    return stub.GetStatus(req).fileInfo


def _create(stub, path):
    req = pb.file.CreateFilePRequest(path=path)
    req.options.writeType = 1  # MUST_CACHE
    stub.CreateFile(req)
    stub.CompleteFile(pb.file.CompleteFilePRequest(path=path))


def test_native_channel_is_used(master):
    m, stub = master
    assert m.native_rpc is not None
    before = m.native_rpc.server.requests
    stub.CreateDirectory(pb.file.CreateDirectoryPRequest(path="/d"))
    _create(stub, "/d/f")
    assert m.native_rpc.server.requests >= before + 3
    names = [fi.name for r in stub.ListStatus(pb.file.ListStatusPRequest(path="/d")) for fi in r.fileInfos]
    assert names == ["f"]


def test_reply_cache_hits_and_invalidates(master):
    m, stub = master
    srv = m.native_rpc.server
    _create(stub, "/f")
    a = _status(stub, "/f")
    hits = srv.cache_hits
    b = _status(stub, "/f")
    assert srv.cache_hits == hits + 1 and a == b
    # a namespace mutation bumps the epoch: the next reply is recomputed and shows the change
    req = pb.file.SetAttributePRequest(path="/f")
    req.options.pinned = True
    stub.SetAttribute(req)
    c = _status(stub, "/f")
    assert c.pinned and not a.pinned
    assert srv.cache_hits == hits + 1
    assert _status(stub, "/f").pinned and srv.cache_hits == hits + 2
    # a block-location change (no namespace entry) also invalidates
    ep = srv.epoch()
    m.block_master._bump_epoch()
    assert srv.epoch() == ep + 1
    _status(stub, "/f")
    assert srv.cache_hits == hits + 2
    # listings are cached too, and a create in the directory invalidates them
    ls = lambda: [fi.name for r in stub.ListStatus(pb.file.ListStatusPRequest(path="/")) for fi in r.fileInfos]
    assert ls() == ["f"]       # first listing loads the root's UFS children (a mutation)
    assert ls() == ["f"]       # computed and cached
    h = srv.cache_hits
    assert ls() == ["f"] and srv.cache_hits == h + 1
    _create(stub, "/g")
    assert ls() == ["f", "g"]


def test_sync_requests_bypass_cache(master):
    m, stub = master
    srv = m.native_rpc.server
    _create(stub, "/f")
    _status(stub, "/f", syncIntervalMs=0)
    h = srv.cache_hits
    _status(stub, "/f", syncIntervalMs=0)
    assert srv.cache_hits == h


def test_not_found_cached_until_created(master):
    """A ONCE lookup of a missing path is answered from the reply cache the second time (the
    UFS absent-path cache makes it stable), and the cached NOT_FOUND dies with the next
    namespace change: creating the path serves the real status."""
    m, stub = master
    srv = m.native_rpc.server
    for _ in range(2):
        with pytest.raises(ex.NotFoundException):
            _status(stub, "/missing", syncIntervalMs=-1)
    assert srv.cache_hits == 1
    _create(stub, "/missing")
    _status(stub, "/missing", syncIntervalMs=-1)
    # lookups that ask for a UFS sync are never cached, errors included
    h = srv.cache_hits
    for _ in range(2):
        with pytest.raises(ex.NotFoundException):
            _status(stub, "/missing2", syncIntervalMs=0)
    assert srv.cache_hits == h


def test_lose_primacy_invalidates(master):
    m, stub = master
    _create(stub, "/f")
    _status(stub, "/f")
    ep = m.native_rpc.server.epoch()
    h = m.native_rpc.server.cache_hits
    m.lose_primacy()
    assert m.native_rpc.server.epoch() > ep
    try:                       # (a non-HA master has no standby gate; an HA one refuses)
        _status(stub, "/f")
    except ex.UnavailableException:
        pass
    assert m.native_rpc.server.cache_hits == h


def test_mutation_reply_waits_for_flush(master):
    m, stub = master
    fsj = m.journal.writers["FileSystemMaster"] if hasattr(m.journal, "writers") else None
    _create(stub, "/x")
    # durable by the time the reply arrived: every appended entry has been flushed
    if fsj is not None:
        assert fsj._flushed == fsj._appended
    # a concurrent burst: all replies arrive, in batches answered by group commit
    errs = []

    def worker(i):
        try:
            for j in range(10):
                _create(stub, f"/b{i}-{j}")
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errs
    names = {fi.name for r in stub.ListStatus(pb.file.ListStatusPRequest(path="/")) for fi in r.fileInfos}
    assert len(names) == 81


class _SlowWriter:
    def __init__(self, delay=0.0, fail=False):
        self.delay, self.fail, self.written = delay, fail, []

    def write(self, e):
        self.written.append(e)

    def flush(self):
        time.sleep(self.delay)
        if self.fail:
            raise IOError("disk gone")

    def close(self):
        pass


def test_flush_async_orders_callbacks():
    w = AsyncJournalWriter(_SlowWriter(0.01), batch_ms=1)
    done = []
    ev = threading.Event()
    for i in range(5):
        c = w.append(i)
        w.flush_async(c, lambda e, i=i: (done.append((i, e)), len(done) == 5 and ev.set()))
    assert ev.wait(5)
    assert [d[0] for d in done] == list(range(5)) and all(d[1] is None for d in done)
    # already durable: fires inline
    got = []
    w.flush_async(3, got.append)
    assert got == [None]
    w.close()


def test_flush_async_reports_failure():
    w = AsyncJournalWriter(_SlowWriter(fail=True), batch_ms=1)
    res = []
    ev = threading.Event()
    c = w.append("e")
    w.flush_async(c, lambda e: (res.append(e), ev.set()))
    assert ev.wait(5)
    assert isinstance(res[0], ex.UnavailableException)


def test_deferred_flush_context_collects_counters():
    from alluxio_amd.journal.system import JournalContext
    w = AsyncJournalWriter(_SlowWriter(), batch_ms=1)
    with deferred_flush() as d:
        ctx = JournalContext(w)
        ctx.append("a")
        ctx.append("b")
        ctx.close()              # does not block
        assert d.pending == {w: 2}
    ev = threading.Event()
    w.flush_async(2, lambda e: ev.set())
    assert ev.wait(5)
    w.close()


def test_control_char_user_names_are_refused(master):
    """"\x01..." / "\x02..." caller strings mark gRPC-connection and internal native-stream
    requests inside the server: a framed-RPC client may not authenticate under such a name."""
    from alluxio_amd.ops.native import lib
    m, _ = master
    path = f"/{FS}/GetStatus"
    req = pb.file.GetStatusPRequest(path="/").SerializeToString()
    for name in ("\x02internal", "\x01cid"):
        c = lib().FrameRpcClient("127.0.0.1", m.native_rpc.port, f"SIMPLE\0{name}\0".encode(), 5000)
        try:
            with pytest.raises(Exception):
                status, msg, _ = c.call(path, req, 5000)
                if status:
                    raise RuntimeError(msg)
        finally:
            c.close()
    ok = lib().FrameRpcClient("127.0.0.1", m.native_rpc.port, b"SIMPLE\0alice\0", 5000)
    try:
        status, _, _ = ok.call(path, req, 5000)
        assert status == 0
    finally:
        ok.close()
