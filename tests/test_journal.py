"""UFS journal format, writer rotation/recovery, checkpoints and replay (reference
UfsJournalLogWriterTest / UfsJournalReaderTest / UfsJournalCheckpointThreadTest)."""
import io
import os

from alluxio_amd.journal import format as fmt
from alluxio_amd.journal.system import Journaled, UfsJournalSystem
from alluxio_amd.journal.ufs_journal import UfsJournal, UfsJournalLogWriter
from alluxio_amd.proto import pb


def _entry(i):
    return pb.journal.JournalEntry(block_info=pb.journal.BlockInfoEntry(block_id=i, length=i * 10))


def test_delimited_roundtrip_and_torn_tail():
    b = io.BytesIO()
    for i in range(5):
        fmt.write_delimited(b, _entry(i))
    raw = b.getvalue()
    assert [e.block_info.block_id for e in fmt.iter_delimited(io.BytesIO(raw))] == list(range(5))
    torn = raw[:-3]
    assert [e.block_info.block_id for e in fmt.iter_delimited(io.BytesIO(torn))] == list(range(4))
    assert fmt.encode_file_name(0x10, fmt.UNKNOWN_SEQUENCE_NUMBER) == "0x10-0x7fffffffffffffff"
    assert fmt.decode_file_name("0x1f-0x20") == (31, 32)
    assert fmt.decode_file_name("junk") is None


def test_writer_rotation_completion_and_reader(tmp_path):
    j = UfsJournal(str(tmp_path), "BlockMaster", max_log_bytes=200)
    j.format()
    w = UfsJournalLogWriter(j, 0, fsync=False)
    for i in range(50):
        w.write(_entry(i))
    w.flush()
    logs = j.logs()
    assert len(logs) >= 3 and logs[-1].is_incomplete and all(not l.is_incomplete for l in logs[:-1])
    assert [e.sequence_number for e in j.iter_log_entries(0)] == list(range(50))
    w.close()
    assert not j.current_log()
    assert j.next_sequence_number() == 50
    # crash recovery: an incomplete log with a torn tail is completed at the last good entry
    w2 = UfsJournalLogWriter(j, 50, fsync=False)
    w2.write(_entry(50))
    w2.flush()
    with open(j.current_log().path, "ab") as f:
        f.write(b"\x40\x01\x02")  # torn record
    nxt = j.next_sequence_number()
    assert nxt == 51
    w3 = UfsJournalLogWriter(j, nxt, fsync=False)
    w3.write(_entry(51))
    w3.close()
    assert [e.sequence_number for e in j.iter_log_entries(45)] == list(range(45, 52))


def test_checkpoint_and_gc(tmp_path):
    j = UfsJournal(str(tmp_path), "M", max_log_bytes=100)
    j.format()
    w = UfsJournalLogWriter(j, 0, fsync=False)
    for i in range(30):
        w.write(_entry(i))
    w.close()
    j.write_checkpoint(30, fmt.CheckpointType.JOURNAL_ENTRY, fmt.entries_to_bytes([_entry(99)]))
    removed = j.gc()
    assert removed > 0 and not j.logs()
    ctype, payload, end = j.read_checkpoint()
    assert ctype == fmt.CheckpointType.JOURNAL_ENTRY and end == 30
    assert fmt.bytes_to_entries(payload)[0].block_info.block_id == 99


class _Counter(Journaled):
    journal_name = "Counter"

    def __init__(self):
        self.values = []

    def process_journal_entry(self, e):
        if e.HasField("block_info"):
            self.values.append(e.block_info.block_id)
            return True
        return False

    def reset_state(self):
        self.values = []

    def journal_entries(self):
        for v in self.values:
            yield _entry(v)


def test_journal_system_replay_checkpoint_and_standby(tmp_path):
    js = UfsJournalSystem(str(tmp_path), flush_batch_ms=0, fsync=False)
    c = _Counter()
    js.register(c)
    js.format()
    js.start()
    js.gain_primacy()
    for i in range(10):
        ctx = js.create_context("Counter")
        e = _entry(i)
        c.process_journal_entry(e)
        ctx.append(e)
        ctx.close()
    js.checkpoint()
    for i in range(10, 15):
        with js.create_context("Counter") as ctx:
            e = _entry(i)
            c.process_journal_entry(e)
            ctx.append(e)
    js.stop()
    # replay into a fresh component: checkpoint + tail logs
    js2 = UfsJournalSystem(str(tmp_path), flush_batch_ms=0, fsync=False)
    c2 = _Counter()
    js2.register(c2)
    js2.start()
    assert c2.values == list(range(15))
    js2.stop()
    assert os.listdir(tmp_path / "Counter" / "v1" / "checkpoints") == ["0x0-0xa"]


def test_upgrade_v0_journal(tmp_path):
    """A 1.x (v0) journal is upgraded in place and replays into a working master."""
    from alluxio_amd.cli.main import main as cli
    from alluxio_amd.journal.upgrade import write_v0_journal
    from alluxio_amd.proto import pb
    import io

    def e(sn, cid):
        return pb.journal.JournalEntry(sequence_number=sn, block_container_id_generator=
                                       pb.journal.BlockContainerIdGeneratorEntry(next_container_id=cid))
    root = str(tmp_path / "journal")
    write_v0_journal(root, "BlockMaster", [e(0, 5)], [[e(1, 6), e(2, 7)], [e(3, 8)]], current=[e(4, 9)])
    conf_env = {"ALLUXIO_OPTS": f"-Dalluxio.master.journal.folder={root}"}
    import os
    old = {k: os.environ.get(k) for k in conf_env}
    os.environ.update(conf_env)
    try:
        out = io.StringIO()
        assert cli(["upgradeJournal", "-journalDirectoryV0", root], out) == 0
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert "BlockMaster: upgraded 3 log(s)" in out.getvalue()
    from alluxio_amd.journal.ufs_journal import UfsJournal
    j = UfsJournal(root, "BlockMaster")
    assert [(f.start, f.end) for f in j.logs()] == [(1, 3), (3, 4), (4, 5)]
    ctype, payload, end = j.read_checkpoint()
    assert end == 1 and [x.block_container_id_generator.next_container_id
                         for x in j.iter_log_entries(end)] == [6, 7, 8, 9]
    # a block master replays it
    from alluxio_amd.journal.system import UfsJournalSystem
    from alluxio_amd.master.block_master import BlockMaster
    from alluxio_amd.conf import Configuration
    js = UfsJournalSystem(root)
    bm = BlockMaster(Configuration(), js)
    js.register(bm)
    js.start()
    assert bm._container_limit == 9
    js.stop()


def test_compound_checkpoint_kryo_golden_bytes():
    """COMPOUND checkpoints use the reference's Kryo chunked layout (JournalUtils.writeToCheckpoint,
    CompoundCheckpointFormat): bytes derived by hand from Kryo's OutputChunked/writeString."""
    import io
    import struct

    from alluxio_amd.journal import format as fmt
    b = io.BytesIO()
    fmt.write_compound(b, [("Noop", b"")])
    # CheckpointOutputStream(COMPOUND) = 8-byte BE 1; chunk of 12 bytes: "NOOP" as Kryo ASCII
    # (last byte | 0x80) + the component's CheckpointType JOURNAL_ENTRY (8-byte BE 0); end marker 0
    assert b.getvalue() == struct.pack(">q", 1) + b"\x0c" + b"NOO\xd0" + b"\x00" * 8 + b"\x00"
    # 64 KB OutputChunked buffer: a 70000-byte body spans a full 65536-byte chunk and a tail
    body = bytes(range(256)) * 273 + b"xy"          # 69890 bytes
    b = io.BytesIO()
    fmt.write_compound(b, [("FileSystemMaster", body)])
    raw = b.getvalue()
    name = fmt.kryo_string("FILE_SYSTEM_MASTER")
    assert name == b"FILE_SYSTEM_MASTE" + bytes([ord("R") | 0x80])
    payload = name + b"\x00" * 8 + body
    assert raw[8:11] == b"\x80\x80\x04"                      # varint 65536
    assert raw[11:11 + 65536] == payload[:65536]
    rest = len(payload) - 65536
    assert raw[11 + 65536:] == fmt.kryo_varint(rest) + payload[65536:] + b"\x00"
    [(name, cp)] = fmt.read_compound(io.BytesIO(raw))
    assert name == "FileSystemMaster" and cp.type == fmt.CheckpointType.JOURNAL_ENTRY and cp.body == body
    # Kryo strings: null, empty, 1 char and >= 64 chars take the UTF-8 length form
    assert fmt.kryo_string(None) == b"\x80" and fmt.kryo_string("") == b"\x81"
    assert fmt.kryo_string("A") == b"\x82A"
    s64 = "a" * 64
    assert fmt.kryo_string(s64) == b"\xc1\x01" + s64.encode()
    for s in (None, "", "A", "NOOP", s64, "ÿ€x"):
        assert fmt.kryo_read_string(fmt.kryo_string(s) + b"tail", 0)[0] == s


def test_raft_snapshot_uses_compound(tmp_path):
    import io

    from alluxio_amd.journal import format as fmt
    from alluxio_amd.proto import pb
    entries = [pb.journal.JournalEntry(sequence_number=i, delete_file=pb.journal.DeleteFileEntry(id=i))
               for i in range(3)]
    b = io.BytesIO()
    fmt.write_compound(b, [("BlockMaster", fmt.entries_to_bytes(entries)), ("TableMaster", b"")])
    parts = fmt.read_compound(io.BytesIO(b.getvalue()))
    assert [p[0] for p in parts] == ["BlockMaster", "TableMaster"]
    assert [e.delete_file.id for e in parts[0][1].entries()] == [0, 1, 2]


def test_native_group_commit_writer_matches_python_layout(tmp_path):
    """The native writer (csrc/journal_log.cpp) produces the same segment files, byte for byte,
    as UfsJournalLogWriter: same names, same framing, sequence_number serialized first."""
    import threading

    from alluxio_amd.journal.system import NativeAsyncJournalWriter
    jp = UfsJournal(str(tmp_path / "py"), "BlockMaster", max_log_bytes=200)
    jn = UfsJournal(str(tmp_path / "nat"), "BlockMaster", max_log_bytes=200)
    jp.format()
    jn.format()
    w = UfsJournalLogWriter(jp, 7, fsync=False)
    for i in range(40):
        w.write(_entry(i))
        if i % 5 == 4:
            w.flush()             # the Python writer rotates per write, the native one per commit
    w.close()
    nw = NativeAsyncJournalWriter(jn, 7, fsync=False, batch_ms=1.0)
    fired = []
    for i in range(40):
        c = nw.append(_entry(i))
        if i % 5 == 4:
            nw.flush(c)
    done = threading.Event()
    nw.flush_async(40, lambda err: (fired.append(err), done.set()))
    assert done.wait(10) and fired == [None]
    assert nw.next_seq == 47 and nw._appended == 40
    nw.close()
    names_p = sorted(os.listdir(jp.log_dir))
    names_n = sorted(os.listdir(jn.log_dir))
    assert names_p == names_n and len(names_n) >= 2
    for n in names_n:
        with open(os.path.join(jp.log_dir, n), "rb") as a, open(os.path.join(jn.log_dir, n), "rb") as b:
            assert a.read() == b.read(), n
    assert [e.sequence_number for e in jn.iter_log_entries(7)] == list(range(7, 47))
    assert jn.next_sequence_number() == 47
    # closed: appends raise, late flush_async callbacks get the closed error
    import pytest
    from alluxio_amd.utils.exceptions import JournalClosedException
    with pytest.raises(JournalClosedException):
        nw.append(_entry(1))
    got = []
    nw.flush_async(99, got.append)
    assert isinstance(got[0], JournalClosedException)


def test_native_writer_replay_through_journal_system(tmp_path):
    """A UFS journal system on the native writer: entries survive a restart (replay), and a
    checkpoint taken at writer.next_seq lines up with the logs."""

    class Comp(Journaled):
        journal_name = "BlockMaster"

        def __init__(self):
            self.ids = []

        def process_journal_entry(self, e):
            if e.HasField("block_info"):
                self.ids.append(e.block_info.block_id)
                return True
            return False

        def reset_state(self):
            self.ids = []

        def journal_entries(self):
            return [_entry(i) for i in self.ids]

    js = UfsJournalSystem(str(tmp_path), max_log_bytes=300, fsync=False, native_writer=True)
    c = Comp()
    js.register(c)
    js.format()
    js.start()
    js.gain_primacy()
    ctx = js.create_context("BlockMaster")
    for i in range(25):
        e = _entry(i)
        c.process_journal_entry(e)
        ctx.append(e)
    ctx.close()
    assert type(js._writers["BlockMaster"]).__name__ == "NativeAsyncJournalWriter"
    assert js.sequence_numbers()["BlockMaster"] == 25
    js.stop()
    js2 = UfsJournalSystem(str(tmp_path), max_log_bytes=300, fsync=False, native_writer=True)
    c2 = Comp()
    js2.register(c2)
    js2.start()
    assert c2.ids == list(range(25))
    js2.gain_primacy()
    ctx = js2.create_context("BlockMaster")
    c2.process_journal_entry(_entry(25))
    ctx.append(_entry(25))
    ctx.close()
    js2.checkpoint()
    js2.stop()
    js3 = UfsJournalSystem(str(tmp_path), max_log_bytes=300, fsync=False)
    c3 = Comp()
    js3.register(c3)
    js3.start()
    assert c3.ids == list(range(26))
    js3.stop()


def test_native_writer_raw_entry_batch_sequence(tmp_path):
    """Natively encoded batches (RawEntryBatch) get the native writer's sequence number."""
    from alluxio_amd.journal.system import NativeAsyncJournalWriter
    from alluxio_amd.ops.native import lib
    j = UfsJournal(str(tmp_path), "BlockMaster", max_log_bytes=1 << 20)
    j.format()
    w = NativeAsyncJournalWriter(j, 3, fsync=False)
    w.append(_entry(1))
    c = w.append(fmt.RawEntryBatch(lib().encode_block_info_batch([11, 12], [5, 6]), 2))
    w.flush(c)
    w.close()
    got = list(j.iter_log_entries(3))
    assert [e.sequence_number for e in got] == [3, 4]
    assert [x.block_info.block_id for x in got[1].journal_entries] == [11, 12]
