"""Journal system: replay, batched asynchronous writes, checkpoints, standby tailing.

Parity: JournalSystem SPI (core/server/common/.../journal/JournalSystem.java: start/stop,
gainPrimacy/losePrimacy, checkpoint, format), ``Journaled.processJournalEntry`` /
``resetState`` / ``getJournalEntryIterator`` contract, ``JournalContext.append`` +
``close()`` waiting for flush (MasterJournalContext.java:35-93), AsyncJournalWriter.java:48-382
(queue + flush thread batching for ``alluxio.master.journal.flush.batch.time``, flush tickets),
UfsJournalCheckpointThread (standby tails logs and writes checkpoints), NoopJournalSystem.
"""
from __future__ import annotations

import heapq
import itertools
import logging
import struct
import threading
import time

from ..utils import optiming as _OPT
from ..utils.exceptions import JournalClosedException, UnavailableException
from . import format as fmt
from .ufs_journal import UfsJournal, UfsJournalLogWriter

LOG = logging.getLogger(__name__)

_DEFER = threading.local()


class deferred_flush:
    """Inside this context, ``JournalContext.close()`` does not block for durability: it records
    ``(writer, counter)`` in ``pending`` and the caller completes the RPC from a flush callback
    (``AsyncJournalWriter.flush_async``).  This is group commit without a parked thread per
    request: the RPC front end answers every mutation of a flush batch when that flush lands."""

    def __enter__(self):
        self.pending: dict = {}
        self.after: list = []      # after_durable callbacks, run once ``pending`` is durable
        self._prev = (getattr(_DEFER, "pending", None), getattr(_DEFER, "after", None))
        _DEFER.pending = self.pending
        _DEFER.after = self.after
        return self

    def __exit__(self, *exc):
        _DEFER.pending, _DEFER.after = self._prev
        return False


def after_durable(cb) -> None:
    """Run ``cb()`` once every journal entry this RPC appended so far is durable.

    In a blocking RPC the journal contexts already waited, so ``cb`` runs now.  Inside
    :class:`deferred_flush` (group-committed native RPCs) it is queued and run by the RPC front end
    after the flush lands, before the reply, and never if the flush fails -- the ordering
    ``RpcContext.close`` gives the reference: namespace entries durable first, then side effects
    such as block deletion (a crash leaves an orphaned block, never an inode with missing blocks)."""
    pending = getattr(_DEFER, "pending", None)
    if pending:
        _DEFER.after.append(cb)
    else:
        cb()


class Journaled:
    """Mixin for journaled master state."""

    journal_name = "Unnamed"

    def process_journal_entry(self, entry) -> bool:  # pragma: no cover - interface
        raise NotImplementedError

    def reset_state(self) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def journal_entries(self):  # pragma: no cover - interface
        """Iterate JournalEntry protos that recreate the current state (checkpoint content)."""
        raise NotImplementedError

    def apply_and_journal(self, ctx, entry) -> None:
        if not self.process_journal_entry(entry):
            raise RuntimeError(f"{self.journal_name} cannot apply its own entry {entry}")
        ctx.append(entry)


def _error_reply(reply, err):
    from ..utils import exceptions as ex
    se = ex.wrap(err)
    return (reply[0], int(se.status), se.message or str(se), b"")


class AsyncJournalWriter:
    """Group commit (AsyncJournalWriter.doFlush): the flush thread wakes as soon as a caller asks
    for a flush (or ``flush.batch.time`` after entries were queued without one), writes everything
    queued -- for at most one batch time per session -- and flushes once; entries arriving during
    that flush ride the next one.  Latency is one write+flush, not a fixed batch window."""

    def __init__(self, writer: UfsJournalLogWriter, batch_ms: float = 5.0, flush_timeout_s: float = 300.0):
        self.writer = writer
        self.batch = batch_ms / 1000.0
        self.flush_timeout = flush_timeout_s
        self._cond = threading.Condition()
        self._queue: list = []
        self._appended = 0       # counter of appended entries
        self._written = 0        # counter of entries handed to the writer
        self._flushed = 0        # counter of durably flushed entries
        self._requested = 0      # highest counter a caller is waiting for
        self._error: BaseException | None = None
        self._closed = False
        self._waiters: list = []   # heap of (counter, seq, callback) for flush_async
        self._seq = itertools.count()
        self._thread = threading.Thread(target=self._run, daemon=True, name="journal-flush")
        self._thread.start()

    def append(self, entry) -> int:
        with self._cond:
            if self._closed:
                raise JournalClosedException("journal is closed")
            if self._error is not None:
                raise UnavailableException(f"journal write failed: {self._error}")
            self._queue.append(entry)
            self._appended += 1
            return self._appended

    def flush(self, counter: int) -> None:
        deadline = time.monotonic() + self.flush_timeout
        with self._cond:
            if counter > self._requested:
                self._requested = counter
                self._cond.notify_all()
            while self._flushed < counter:
                if self._error is not None:
                    raise UnavailableException(f"journal flush failed: {self._error}")
                if self._closed and not self._queue and self._flushed < counter:
                    raise JournalClosedException("journal closed before flush")
                rem = deadline - time.monotonic()
                if rem <= 0:
                    raise UnavailableException("journal flush timed out")
                self._cond.wait(min(rem, 0.05))

    def flush_async(self, counter: int, cb) -> None:
        """Call ``cb(None)`` once entries up to ``counter`` are durable (``cb(exc)`` on failure);
        runs ``cb`` on the flush thread, or inline when already flushed."""
        err = None
        with self._cond:
            if self._error is not None:
                err = UnavailableException(f"journal flush failed: {self._error}")
            elif self._flushed < counter:
                if self._closed and not self._queue:
                    err = JournalClosedException("journal closed before flush")
                else:
                    heapq.heappush(self._waiters, (counter, next(self._seq), cb))
                    if counter > self._requested:
                        self._requested = counter
                        self._cond.notify_all()
                    return
        cb(err)

    def reply_when_flushed(self, counter: int, srv, reply) -> None:
        """Send the RPC ``reply`` (a native server's respond_many tuple) once entries up to
        ``counter`` are durable -- an error reply if the flush fails.  The flush thread sends every
        reply its flush released in ONE respond_many call per server (one wakeup of the server's
        I/O threads per group commit instead of one per deferred RPC)."""
        with self._cond:
            if self._error is None and self._flushed < counter and not (self._closed and not self._queue):
                heapq.heappush(self._waiters, (counter, next(self._seq), (srv, reply)))
                if counter > self._requested:
                    self._requested = counter
                    self._cond.notify_all()
                return
            err = None
            if self._error is not None:
                err = UnavailableException(f"journal flush failed: {self._error}")
            elif self._flushed < counter:
                err = JournalClosedException("journal closed before flush")
        srv.respond_many([reply if err is None else _error_reply(reply, err)])

    def _fire(self, flushed: int, err=None) -> None:
        ready = []
        replies: dict = {}
        with self._cond:
            while self._waiters and (err is not None or self._waiters[0][0] <= flushed):
                w = heapq.heappop(self._waiters)[2]
                if type(w) is tuple:
                    srv, reply = w
                    ent = replies.get(id(srv))
                    if ent is None:
                        ent = replies[id(srv)] = (srv, [])
                    ent[1].append(reply if err is None else _error_reply(reply, err))
                else:
                    ready.append(w)
        for srv, batch in replies.values():
            try:
                srv.respond_many(batch)
            except Exception:  # noqa: BLE001
                LOG.exception("journal flush replies failed")
        for cb in ready:
            try:
                cb(err)
            except Exception:  # noqa: BLE001
                LOG.exception("journal flush callback failed")

    def _run(self) -> None:
        try:
            self._run_loop()
        finally:
            with self._cond:
                closed_err = self._error
            self._fire(0, UnavailableException(f"journal flush failed: {closed_err}") if closed_err
                       else JournalClosedException("journal closed before flush"))

    def _run_loop(self) -> None:
        while True:
            with self._cond:
                # stand still until entries are queued and someone waits for them (or the batch
                # time passed since they were queued, to flush proactively)
                waited_since = None
                while True:
                    if self._closed and not self._queue:
                        return
                    if self._queue and (self._requested > self._written or self._closed):
                        break
                    if self._queue:
                        now = time.monotonic()
                        waited_since = waited_since or now
                        if now - waited_since >= self.batch:
                            break
                        self._cond.wait(self.batch - (now - waited_since))
                    else:
                        waited_since = None
                        self._cond.wait(0.1)
                batch, self._queue = self._queue, []
            try:
                t0 = time.monotonic()
                c0 = time.thread_time() if _OPT.ENABLED else 0.0
                n = 0
                for e in batch:
                    self.writer.write(e)
                    n += 1
                    if self.batch and n % 256 == 0 and time.monotonic() - t0 >= self.batch:
                        break
                if n < len(batch):       # session over: the rest goes first next time
                    with self._cond:
                        self._queue[:0] = batch[n:]
                if _OPT.ENABLED:
                    c1 = time.thread_time()
                    _OPT.add("journal_write_cpu_per_entry", (c1 - c0) / max(1, n))
                    _OPT.add("journal_entries_per_flush", n * 1e-6)
                    f0 = time.perf_counter()
                self.writer.flush()
                if _OPT.ENABLED:
                    _OPT.add("journal_fsync_wall", time.perf_counter() - f0)
                with self._cond:
                    self._written += n
                    self._flushed = flushed = self._written
                    self._cond.notify_all()
                if self._waiters:
                    c2 = time.thread_time() if _OPT.ENABLED else 0.0
                    self._fire(flushed)
                    if _OPT.ENABLED:
                        _OPT.add("journal_fire_cpu_per_entry", (time.thread_time() - c2) / max(1, n))
            except BaseException as e:  # noqa: BLE001
                LOG.exception("journal flush failed")
                with self._cond:
                    self._error = e
                    self._cond.notify_all()
                return

    def close(self) -> None:
        with self._cond:
            self._closed = True
            self._cond.notify_all()
        self._thread.join(timeout=10)
        self.writer.close()


class NativeAsyncJournalWriter:
    """AsyncJournalWriter over the native group-commit log (csrc/journal_log.cpp): same interface
    (append / flush / flush_async / reply_when_flushed / close, ``writer.next_seq``), but the flush
    loop -- framing, write, fsync, segment rotation, and the replies of the RPCs a commit releases --
    runs on a C++ thread that never takes the GIL.  Python callbacks (``flush_async``: RPCs with
    post-durable work or entries in several journals) are fired by a helper thread that waits on
    the native log with the GIL released.

    Parity: AsyncJournalWriter.java:243-295 (doFlush), :334 (flush); UfsJournalLogWriter.java:115-209.
    """

    def __init__(self, journal: UfsJournal, next_seq: int, fsync: bool = True, batch_ms: float = 5.0,
                 flush_timeout_s: float = 300.0):
        from ..ops.native import lib
        UfsJournalLogWriter(journal, next_seq, fsync=fsync)    # completes the previous incomplete log
        self._log = lib().JournalLog(journal.log_dir, next_seq, journal.max_log_bytes, fsync, batch_ms)
        self.writer = self               # ``w.writer.next_seq`` (checkpoint / sequence_numbers)
        self.flush_timeout = flush_timeout_s
        self._cb_cond = threading.Condition()
        self._cbs: list = []             # heap of (counter, seq, callback)
        self._seq = itertools.count()
        self._cb_thread: threading.Thread | None = None
        self._closed = False
        self._servers: set = set()       # servers with replies in flight (kept alive until close)
        if _OPT.ENABLED:
            _OPT.add_reporter(f"journal_commit:{journal.name}",
                              self.commit_stats)

    def commit_stats(self) -> dict:
        e, f, w, s, r, wait, mx = self._log.stats()
        return {"entries": e, "flushes": f, "entries_per_flush": round(e / max(1, f), 1),
                "write_us_per_flush": round(w / max(1, f), 1), "fsync_us_per_flush": round(s / max(1, f), 1),
                "reply_us_per_flush": round(r / max(1, f), 1),
                "append_to_durable_us_mean": round(wait / max(1, e), 1), "append_to_durable_us_max": mx}

    @property
    def next_seq(self) -> int:
        return self._log.next_seq

    @property
    def _appended(self) -> int:
        return self._log.appended

    @staticmethod
    def _raise(e: RuntimeError):
        msg = str(e)
        if msg.startswith("closed: "):
            raise JournalClosedException(msg[len("closed: "):]) from None
        raise UnavailableException(msg[len("failed: "):] if msg.startswith("failed: ") else msg) from None

    def append(self, entry) -> int:
        if type(entry) is fmt.RawEntryBatch:
            data = entry.body              # natively encoded batch body, no sequence number yet
        else:
            if entry.sequence_number:
                entry.sequence_number = 0  # the native log prepends the sequence number it assigns
            data = entry.SerializeToString()
        try:
            return self._log.append(data)
        except RuntimeError as e:
            self._raise(e)

    def flush(self, counter: int) -> None:
        try:
            if self._log.wait_flushed(counter, int(self.flush_timeout * 1000)):
                raise UnavailableException("journal flush timed out")
        except RuntimeError as e:
            self._raise(e)

    def reply_when_flushed(self, counter: int, srv, reply) -> None:
        if srv not in self._servers:
            self._servers.add(srv)
        self._log.reply_when_flushed(counter, srv, reply)

    def flush_async(self, counter: int, cb) -> None:
        with self._cb_cond:
            if not self._closed:
                heapq.heappush(self._cbs, (counter, next(self._seq), cb))
                if self._cb_thread is None:
                    self._cb_thread = threading.Thread(target=self._cb_loop, daemon=True, name="journal-callbacks")
                    self._cb_thread.start()
                self._cb_cond.notify()
                self._log.request(counter)
                return
        cb(JournalClosedException("journal closed before flush"))

    def _cb_loop(self) -> None:
        while True:
            with self._cb_cond:
                while not self._cbs and not self._closed:
                    self._cb_cond.wait(0.5)
                if not self._cbs:
                    return
                target = self._cbs[0][0]
            err = None
            try:
                if self._log.wait_flushed(target, 200):
                    continue                  # timed out: re-check (new, lower counters may have come)
            except RuntimeError as e:
                try:
                    self._raise(e)
                except Exception as ex_:  # noqa: BLE001
                    err = ex_
            flushed = self._log.flushed
            ready = []
            with self._cb_cond:
                while self._cbs and (err is not None or self._cbs[0][0] <= flushed):
                    ready.append(heapq.heappop(self._cbs)[2])
            for cb in ready:
                try:
                    cb(err)
                except Exception:  # noqa: BLE001
                    LOG.exception("journal flush callback failed")

    def close(self) -> None:
        self._log.close()                 # flushes what is queued; replies go out or fail
        with self._cb_cond:
            self._closed = True
            self._cb_cond.notify_all()
        t = self._cb_thread
        if t is not None:
            t.join(timeout=10)
        with self._cb_cond:                # callbacks whose entries never became durable
            rest, self._cbs = self._cbs, []
        flushed = self._log.flushed
        for c, _s, cb in rest:
            try:
                cb(None if c <= flushed else JournalClosedException("journal closed before flush"))
            except Exception:  # noqa: BLE001
                LOG.exception("journal flush callback failed")
        self._servers.clear()


class JournalContext:
    """Collects entries for one RPC; ``close`` blocks until they are durable."""

    def __init__(self, writer: AsyncJournalWriter | None, state_lock=None):
        self._writer = writer
        self._last = 0
        self._state_lock = state_lock

    def append(self, entry) -> None:
        if self._writer is not None:
            self._last = self._writer.append(entry)

    def close(self) -> None:
        if self._writer is not None and self._last:
            pending = getattr(_DEFER, "pending", None)
            if pending is not None and hasattr(self._writer, "flush_async"):
                w = self._writer
                pending[w] = max(pending.get(w, 0), self._last)
            else:
                self._writer.flush(self._last)

    def __enter__(self):
        if self._state_lock is not None:
            self._state_lock.acquire_shared()
        return self

    def __exit__(self, *exc):
        try:
            self.close()
        finally:
            if self._state_lock is not None:
                self._state_lock.release_shared()


class NoopJournalContext(JournalContext):
    def __init__(self, state_lock=None):
        super().__init__(None, state_lock)


class JournalSystem:
    def __init__(self):
        self._journaled: dict[str, Journaled] = {}
        self.primary = False

    def register(self, j: Journaled) -> None:
        self._journaled[j.journal_name] = j

    @property
    def journaled(self) -> dict[str, Journaled]:
        return dict(self._journaled)

    def start(self) -> None: ...

    def stop(self) -> None: ...

    def gain_primacy(self) -> None:
        self.primary = True

    def lose_primacy(self) -> None:
        self.primary = False

    def create_context(self, name: str, state_lock=None) -> JournalContext:
        return NoopJournalContext(state_lock)

    def checkpoint(self) -> None: ...

    def format(self) -> None: ...

    def is_formatted(self) -> bool:
        return True

    def is_empty(self) -> bool:
        return True

    def sequence_numbers(self) -> dict[str, int]:
        return {}

    # ---- standby journal application control (JournalSystem.suspend/catchup/resume, used by
    # the backup-worker role to take a backup at a sequence chosen by the primary) ----------------
    def suspend(self) -> None:
        raise NotImplementedError(f"{type(self).__name__} cannot suspend journal application")

    def catchup(self, sequences: dict[str, int], timeout: float = 60.0) -> None:
        raise NotImplementedError(f"{type(self).__name__} cannot catch up to given sequences")

    def resume(self) -> None:
        raise NotImplementedError(f"{type(self).__name__} cannot resume journal application")


class NoopJournalSystem(JournalSystem):
    """No persistence (tests, ephemeral masters)."""


def _native_journal_available() -> bool:
    try:
        from ..ops.native import lib
        return hasattr(lib(), "JournalLog")
    except Exception:  # noqa: BLE001 - extension not built: the Python writer
        return False


class UfsJournalSystem(JournalSystem):
    def __init__(self, root: str, max_log_bytes: int = 10 << 20, flush_batch_ms: float = 5.0,
                 checkpoint_period_entries: int = 2_000_000, fsync: bool = True, native_writer: bool = False):
        super().__init__()
        self.native_writer = native_writer
        self.root = root
        self.max_log_bytes = max_log_bytes
        self.flush_batch_ms = flush_batch_ms
        self.checkpoint_period = checkpoint_period_entries
        self.fsync = fsync
        self._journals: dict[str, UfsJournal] = {}
        self._writers: dict[str, AsyncJournalWriter] = {}
        self._applied: dict[str, int] = {}
        self._lock = threading.RLock()
        self._tail_thread = None
        self._tail_stop = threading.Event()
        self._suspended = False        # standby: tailing paused for a delegated backup

    def register(self, j: Journaled) -> None:
        super().register(j)
        self._journals[j.journal_name] = UfsJournal(self.root, j.journal_name, self.max_log_bytes)

    def format(self) -> None:
        for j in self._journals.values():
            j.format()

    def is_formatted(self) -> bool:
        """Formatted when any master's journal is: a journal written by an older release lacks the
        directories of masters added since (e.g. TableMaster in a 1.8 journal); ``start`` creates
        them empty."""
        return any(j.is_formatted() for j in self._journals.values())

    def is_empty(self) -> bool:
        return all(not j.logs() and not j.checkpoints() for j in self._journals.values())

    def start(self) -> None:
        for j in self._journals.values():
            j.ensure()
        # standby: replay what exists and keep tailing until primacy
        self._replay_all()
        self._tail_stop.clear()
        self._tail_thread = threading.Thread(target=self._tail_loop, daemon=True, name="journal-tailer")
        self._tail_thread.start()

    def _replay_all(self) -> None:
        with self._lock:
            for name, j in self._journals.items():
                comp = self._journaled[name]
                comp.reset_state()
                ctype, payload, end = j.read_checkpoint()
                applied = 0
                if ctype is not None:
                    self._apply_checkpoint(comp, ctype, payload)
                    applied = end
                for e in j.iter_log_entries(applied):
                    self._apply(comp, e)
                    applied = e.sequence_number + 1
                self._applied[name] = applied

    @staticmethod
    def _apply(comp: Journaled, e) -> None:
        if e.journal_entries:
            for sub in e.journal_entries:
                comp.process_journal_entry(sub)
        elif not comp.process_journal_entry(e):
            LOG.warning("%s ignored journal entry %s", comp.journal_name, e.WhichOneof)

    def _apply_checkpoint(self, comp, ctype, payload) -> None:
        """Restore ``comp`` from its checkpoint file: JOURNAL_ENTRY (delimited entries) or the
        typed/nested formats (e.g. the FileSystemMaster COMPOUND tree, journal/checkpoint.py)."""
        from . import checkpoint as ck
        cp = ck.parse(ck.typed(ctype, payload), fmt.CHECKPOINT_NAMES.get(comp.journal_name, comp.journal_name))
        ck.restore_journaled(comp, cp, self._apply)

    def _tail_loop(self) -> None:
        while not self._tail_stop.wait(0.5):
            if self.primary:
                return
            try:
                with self._lock:
                    if self._suspended:
                        continue
                    for name, j in self._journals.items():
                        comp = self._journaled[name]
                        start = self._applied.get(name, 0)
                        for e in j.iter_log_entries(start):
                            self._apply(comp, e)
                            self._applied[name] = e.sequence_number + 1
            except Exception:  # noqa: BLE001
                LOG.exception("journal tailing failed")

    def suspend(self) -> None:
        """Stop applying tailed entries (UfsJournalSystem.suspend)."""
        with self._lock:
            if self.primary:
                raise RuntimeError("cannot suspend the primary's journal")
            self._suspended = True

    def catchup(self, sequences: dict[str, int], timeout: float = 60.0) -> None:
        """Apply tailed entries exactly up to ``sequences`` (exclusive, per master) while
        suspended, waiting for the primary's logs to reach them (UfsJournalSystem.catchup)."""
        deadline = time.monotonic() + timeout
        while True:
            with self._lock:
                if not self._suspended:
                    raise RuntimeError("catchup needs a suspended journal")
                behind = False
                for name, target in sequences.items():
                    j, comp = self._journals.get(name), self._journaled.get(name)
                    if j is None or comp is None:
                        continue
                    start = self._applied.get(name, 0)
                    if start > target:
                        raise RuntimeError(f"{name} already applied {start} > requested {target}")
                    if start < target:
                        for e in j.iter_log_entries(start):
                            if e.sequence_number >= target:
                                break
                            self._apply(comp, e)
                            self._applied[name] = e.sequence_number + 1
                    behind = behind or self._applied.get(name, 0) < target
                if not behind:
                    return
            if time.monotonic() > deadline:
                raise TimeoutError(f"journal catch-up to {sequences} timed out")
            time.sleep(0.05)

    def resume(self) -> None:
        with self._lock:
            self._suspended = False

    def gain_primacy(self) -> None:
        self._tail_stop.set()
        if self._tail_thread is not None:
            self._tail_thread.join(timeout=5)
        with self._lock:
            # catch up fully, then become the writer
            self._suspended = False
            self._replay_all()
            for name, j in self._journals.items():
                nxt = max(self._applied.get(name, 0), j.next_sequence_number())
                if self.native_writer and _native_journal_available():
                    self._writers[name] = NativeAsyncJournalWriter(j, nxt, fsync=self.fsync,
                                                                   batch_ms=self.flush_batch_ms)
                else:
                    w = UfsJournalLogWriter(j, nxt, fsync=self.fsync)
                    self._writers[name] = AsyncJournalWriter(w, self.flush_batch_ms)
        super().gain_primacy()

    def lose_primacy(self) -> None:
        self._close_writers()
        super().lose_primacy()

    def _close_writers(self) -> None:
        for w in self._writers.values():
            w.close()
        self._writers.clear()

    def stop(self) -> None:
        self._tail_stop.set()
        self._close_writers()

    def create_context(self, name: str, state_lock=None) -> JournalContext:
        w = self._writers.get(name)
        if w is None:
            raise UnavailableException(f"journal for {name} is not writable (not primary)")
        return JournalContext(w, state_lock)

    def checkpoint(self) -> None:
        """Snapshot every component at its current sequence number and GC old files."""
        with self._lock:
            for name, j in self._journals.items():
                w = self._writers.get(name)
                comp = self._journaled[name]
                if w is not None:
                    w.flush(w._appended)
                    end = w.writer.next_seq
                else:
                    end = self._applied.get(name, 0)
                from . import checkpoint as ck
                data = ck.write_journaled(comp)        # typed stream, header included
                j.write_checkpoint(end, fmt.CheckpointType(struct.unpack(">q", data[:8])[0]), data[8:])
                j.gc()

    def sequence_numbers(self) -> dict[str, int]:
        out = {}
        for name, j in self._journals.items():
            w = self._writers.get(name)
            out[name] = w.writer.next_seq if w else self._applied.get(name, 0)
        return out
