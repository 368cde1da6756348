"""UFS journal, version v1 (one per master component).

Layout (reference UfsJournal.java:79-172)::

    <journal-root>/<MasterName>/v1/logs/0x<start>-0x<end>        completed logs (end exclusive)
    <journal-root>/<MasterName>/v1/logs/0x<start>-0x7fff...ffff   the log being written
    <journal-root>/<MasterName>/v1/checkpoints/0x0-0x<end>        snapshot of state < end
    <journal-root>/<MasterName>/v1/.tmp/<uuid>                    checkpoint being written

The writer assigns sequence numbers, rotates at ``alluxio.master.journal.log.size.bytes.max``,
completes (renames) the current log on rotation/close, and recovers from a torn tail by rescanning
the last incomplete log (UfsJournalLogWriter.java:100-209).  The reader replays the latest
checkpoint then every log entry with seq >= checkpoint end (UfsJournalReader.java).  The garbage
collector deletes logs fully covered by a newer checkpoint (UfsJournalGarbageCollector.java).
The journal directory may live on any UFS; local files get ``fsync`` on flush.
"""
from __future__ import annotations

import io
import logging
import os
import threading
import uuid

from ..utils.exceptions import JournalClosedException
from . import format as fmt

LOG = logging.getLogger(__name__)

VERSION = "v1"
FORMAT_FILE_PREFIX = "_format_"   # alluxio.master.format.file.prefix


class UfsJournalFile:
    __slots__ = ("path", "start", "end", "is_checkpoint", "is_tmp")

    def __init__(self, path, start, end, is_checkpoint=False, is_tmp=False):
        self.path, self.start, self.end = path, start, end
        self.is_checkpoint, self.is_tmp = is_checkpoint, is_tmp

    @property
    def is_incomplete(self) -> bool:
        return self.end == fmt.UNKNOWN_SEQUENCE_NUMBER

    def __repr__(self):
        return f"UfsJournalFile({os.path.basename(self.path)})"


class UfsJournal:
    def __init__(self, root: str, name: str, max_log_bytes: int = 10 << 20):
        self.root = root
        self.name = name
        self.location = os.path.join(root, name, VERSION)
        self.log_dir = os.path.join(self.location, "logs")
        self.checkpoint_dir = os.path.join(self.location, "checkpoints")
        self.tmp_dir = os.path.join(self.location, ".tmp")
        self.max_log_bytes = max_log_bytes

    # ---- format -----------------------------------------------------------------------------
    def format(self) -> None:
        """Empty the journal location and drop a ``_format_<ms>`` marker (UfsJournal.java:424-443)."""
        import shutil
        import time
        if os.path.isdir(self.location):
            shutil.rmtree(self.location)
        for d in (self.log_dir, self.checkpoint_dir, self.tmp_dir):
            os.makedirs(d, exist_ok=True)
        with open(os.path.join(self.location, f"{FORMAT_FILE_PREFIX}{int(time.time() * 1000)}"), "wb"):
            pass

    def is_formatted(self) -> bool:
        """A ``_format_*`` marker in the location (UfsJournal.java:399-414), as the Java masters
        write it; directories laid out before markers existed count as formatted as well."""
        if not os.path.isdir(self.location):
            return False
        if any(n.startswith(FORMAT_FILE_PREFIX) for n in os.listdir(self.location)):
            return True
        return os.path.isdir(self.log_dir) and os.path.isdir(self.checkpoint_dir)

    def ensure(self) -> None:
        for d in (self.log_dir, self.checkpoint_dir, self.tmp_dir):
            os.makedirs(d, exist_ok=True)

    # ---- snapshot of files ------------------------------------------------------------------
    def logs(self) -> list[UfsJournalFile]:
        out = []
        if not os.path.isdir(self.log_dir):
            return out
        for n in os.listdir(self.log_dir):
            r = fmt.decode_file_name(n)
            if r:
                out.append(UfsJournalFile(os.path.join(self.log_dir, n), r[0], r[1]))
        return sorted(out, key=lambda f: (f.start, f.end))

    def checkpoints(self) -> list[UfsJournalFile]:
        out = []
        if not os.path.isdir(self.checkpoint_dir):
            return out
        for n in os.listdir(self.checkpoint_dir):
            r = fmt.decode_file_name(n)
            if r:
                out.append(UfsJournalFile(os.path.join(self.checkpoint_dir, n), r[0], r[1], True))
        return sorted(out, key=lambda f: f.end)

    def latest_checkpoint(self) -> UfsJournalFile | None:
        cps = self.checkpoints()
        return cps[-1] if cps else None

    def current_log(self) -> UfsJournalFile | None:
        logs = self.logs()
        if logs and logs[-1].is_incomplete:
            return logs[-1]
        return None

    def next_sequence_number(self) -> int:
        """First sequence number not present in any checkpoint or log."""
        nxt = 0
        cp = self.latest_checkpoint()
        if cp:
            nxt = cp.end
        for lf in self.logs():
            if lf.is_incomplete:
                last = None
                with open(lf.path, "rb") as f:
                    for e in fmt.iter_delimited(f):
                        last = e.sequence_number
                if last is not None:
                    nxt = max(nxt, last + 1)
                else:
                    nxt = max(nxt, lf.start)
            else:
                nxt = max(nxt, lf.end)
        return nxt

    # ---- reading ----------------------------------------------------------------------------
    def read_checkpoint(self) -> tuple[fmt.CheckpointType | None, bytes, int]:
        cp = self.latest_checkpoint()
        if cp is None:
            return None, b"", 0
        with open(cp.path, "rb") as f:
            ctype = fmt.read_checkpoint_header(f)
            return ctype, f.read(), cp.end

    def iter_log_entries(self, from_seq: int):
        """Yield every log entry with ``sequence_number >= from_seq`` in order (skips dups)."""
        expect = from_seq
        for lf in self.logs():
            if not lf.is_incomplete and lf.end <= from_seq:
                continue
            with open(lf.path, "rb") as f:
                for e in fmt.iter_delimited(f):
                    if e.sequence_number < expect:
                        continue
                    if e.sequence_number > expect:
                        raise RuntimeError(f"journal gap in {lf}: expected {expect}, found "
                                           f"{e.sequence_number}")
                    expect += 1
                    yield e

    # ---- checkpoint writing -----------------------------------------------------------------
    def write_checkpoint(self, end_seq: int, ctype: fmt.CheckpointType, payload: bytes) -> str:
        self.ensure()
        tmp = os.path.join(self.tmp_dir, uuid.uuid4().hex)
        with open(tmp, "wb") as f:
            fmt.write_checkpoint_header(f, ctype)
            f.write(payload)
            f.flush()
            os.fsync(f.fileno())
        final = os.path.join(self.checkpoint_dir, fmt.encode_file_name(0, end_seq))
        os.replace(tmp, final)
        return final

    def gc(self) -> int:
        """Delete checkpoints older than the latest and logs entirely below it."""
        cp = self.latest_checkpoint()
        if cp is None:
            return 0
        n = 0
        for old in self.checkpoints()[:-1]:
            os.remove(old.path)
            n += 1
        for lf in self.logs():
            if not lf.is_incomplete and lf.end <= cp.end:
                os.remove(lf.path)
                n += 1
        for t in os.listdir(self.tmp_dir) if os.path.isdir(self.tmp_dir) else []:
            try:
                os.remove(os.path.join(self.tmp_dir, t))
            except OSError:
                pass
        return n


class UfsJournalLogWriter:
    """Appends sequence-numbered entries; rotation, completion and torn-tail recovery."""

    def __init__(self, journal: UfsJournal, next_seq: int, fsync: bool = True):
        self.journal = journal
        self.next_seq = next_seq
        self.fsync = fsync
        self._f: io.BufferedWriter | None = None
        self._cur_path: str | None = None
        self._cur_start = next_seq
        self._bytes = 0
        self._closed = False
        self._lock = threading.Lock()
        self._pending: list = []  # written but not yet flushed (for recovery)
        journal.ensure()
        cur = journal.current_log()
        if cur is not None:
            # complete the previous incomplete log at the recovered end
            self._complete(cur.path, cur.start, next_seq)

    def _complete(self, path, start, end) -> None:
        if end <= start:
            os.remove(path)
            return
        final = os.path.join(self.journal.log_dir, fmt.encode_file_name(start, end))
        os.replace(path, final)

    def _rotate(self) -> None:
        if self._f is not None:
            self._close_current()
        self._cur_start = self.next_seq
        self._cur_path = os.path.join(self.journal.log_dir,
                                      fmt.encode_file_name(self.next_seq, fmt.UNKNOWN_SEQUENCE_NUMBER))
        self._f = open(self._cur_path, "ab")
        self._bytes = 0

    def _close_current(self) -> None:
        self._f.flush()
        if self.fsync:
            os.fsync(self._f.fileno())
        self._f.close()
        self._f = None
        self._complete(self._cur_path, self._cur_start, self.next_seq)
        self._cur_path = None

    def write(self, entry) -> int:
        with self._lock:
            if self._closed:
                raise JournalClosedException("journal writer is closed")
            if self._f is None or self._bytes >= self.journal.max_log_bytes:
                self._rotate()
            entry.sequence_number = self.next_seq
            self._bytes += fmt.write_delimited(self._f, entry)
            self._pending.append(entry)
            self.next_seq += 1
            return entry.sequence_number

    def flush(self) -> None:
        with self._lock:
            if self._f is None:
                return
            self._f.flush()
            if self.fsync:
                os.fsync(self._f.fileno())
            self._pending.clear()

    def close(self) -> None:
        with self._lock:
            if self._closed:
                return
            self._closed = True
            if self._f is not None:
                self._close_current()
