"""Metadata backups: local and delegated-to-standby backups, status tracking, daily backups, and
the standby-master registration (MetaMasterSync) that delegation relies on.

Parity (core/server/master/src/main/java/alluxio/master/):
* backup/BackupLeaderRole.java:60-362 -- ``backup`` initiates under a lock (one backup at a time),
  delegates to a standby when ``alluxio.master.backup.delegation.enabled`` and the masters run HA
  (``allowLeader`` falls back to a local backup when no standby is registered), otherwise takes
  the backup locally under the exclusive state lock; ``runAsync`` returns ``Initiating`` at once.
* backup/BackupWorkerRole.java:60-400 -- the standby suspends journal application when asked,
  catches up to exactly the journal sequence numbers the primary read under its exclusive state
  lock, writes the backup from its own state, then resumes; a suspend not followed by a request
  within ``alluxio.master.backup.transport.timeout`` resumes on its own.
* backup/BackupTracker.java -- status of the current backup (Initiating -> Transitioning ->
  Running -> Completed / Failed) with waiters.
* meta/DailyMetadataBackup.java -- a backup every day at ``alluxio.master.daily.backup.time``
  (UTC), keeping ``alluxio.master.daily.backup.files.retained`` files.
* meta/MetaMasterSync.java -- standbys register with the primary (GetMasterId / RegisterMaster)
  and heartbeat it (re-registering on ``MetaCommand_Register``).

Transport difference: the reference runs the leader<->worker protocol over a copycat-style
messaging stream opened by the standby; here the primary calls the standby's
``BackupWorkerService`` RPCs (SuspendJournals, DelegateBackup, GetBackupStatus) at the address the
standby registered through MetaMasterSync, and polls status every
``alluxio.master.backup.heartbeat.interval``; a standby unreachable for
``alluxio.master.backup.abandon.timeout`` fails the backup.
"""
from __future__ import annotations

import datetime
import gzip
import io
import logging
import os
import threading
import time
import uuid

from ..journal import format as jfmt
from ..proto import enum_name, pb
from ..utils.exceptions import (AlluxioStatusException, FailedPreconditionException, UnavailableException)

LOG = logging.getLogger(__name__)

SVC_BACKUP_WORKER = "alluxio.grpc.meta.BackupWorkerService"
SVC_META_MASTER = "alluxio.grpc.meta.MetaMasterMasterService"
BACKUP_PREFIX = "alluxio-backup-"

S = pb.meta.BackupState
INITIATING, TRANSITIONING, RUNNING = S.values_by_name["Initiating"].number, \
    S.values_by_name["Transitioning"].number, S.values_by_name["Running"].number
COMPLETED, FAILED = S.values_by_name["Completed"].number, S.values_by_name["Failed"].number


class BackupException(FailedPreconditionException):
    pass


class BackupDelegationException(FailedPreconditionException):
    pass


def write_backup(masters, target_dir: str, host: str = "") -> tuple[str, int]:
    """Gzip'ed length-delimited JournalEntry stream of every master's state (the format
    ``alluxio.master.journal.init.from.backup`` restores, same as the Java masters')."""
    os.makedirs(target_dir, exist_ok=True)
    stamp = datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%d-%H%M%S%f")
    name = f"{BACKUP_PREFIX}{stamp}-{uuid.uuid4().hex[:6]}.gz"
    path = os.path.join(target_dir, name)
    buf = io.BytesIO()
    count = 0
    for m in masters:
        for e in m.journal_entries():
            jfmt.write_delimited(buf, e)
            count += 1
    tmp = path + ".tmp"
    with gzip.open(tmp, "wb") as f:
        f.write(buf.getvalue())
    os.replace(tmp, path)
    return path, count


class BackupTracker:
    """Status of the latest backup plus waiters (BackupTracker.java)."""

    def __init__(self):
        self._cond = threading.Condition()
        self.status = pb.meta.BackupPStatus(backupState=S.values_by_name["None"].number)
        self._history: dict[str, pb.meta.BackupPStatus] = {}

    def reset(self, host: str) -> str:
        with self._cond:
            bid = uuid.uuid4().hex
            self.status = pb.meta.BackupPStatus(backupId=bid, backupState=INITIATING, backupHost=host)
            self._history[bid] = self.status
            return bid

    def in_progress(self) -> bool:
        with self._cond:
            return self.status.backupState in (INITIATING, TRANSITIONING, RUNNING)

    def update(self, st: pb.meta.BackupPStatus) -> None:
        with self._cond:
            if st.backupId != self.status.backupId:
                return
            self.status.CopyFrom(st)
            self._cond.notify_all()

    def set_state(self, state: int, **fields) -> None:
        with self._cond:
            self.status.backupState = state
            for k, v in fields.items():
                setattr(self.status, k, v)
            self._cond.notify_all()

    def fail(self, err: BaseException | str) -> None:
        self.set_state(FAILED, backupError=str(err).encode())

    def wait_finished(self, timeout: float | None = None) -> pb.meta.BackupPStatus:
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cond:
            while self.status.backupState not in (COMPLETED, FAILED):
                rem = None if deadline is None else deadline - time.monotonic()
                if rem is not None and rem <= 0:
                    break
                self._cond.wait(0.2 if rem is None else min(rem, 0.2))
            return self.copy()

    def copy(self) -> pb.meta.BackupPStatus:
        with self._cond:
            out = pb.meta.BackupPStatus()
            out.CopyFrom(self.status)
            return out

    def get(self, backup_id: str) -> pb.meta.BackupPStatus:
        with self._cond:
            st = self._history.get(backup_id)
            if st is None:
                return pb.meta.BackupPStatus(backupId=backup_id, backupState=S.values_by_name["None"].number)
            out = pb.meta.BackupPStatus()
            out.CopyFrom(st)
            return out


class BackupLeaderRole:
    """Primary side: initiate backups locally or on a standby master."""

    def __init__(self, process):
        self.p = process                   # AlluxioMasterProcess
        self.conf = process.conf
        self.tracker = BackupTracker()
        self._initiate = threading.Lock()
        self._poller: threading.Thread | None = None

    # ---- helpers ------------------------------------------------------------------------------
    def _host(self) -> str:
        return (self.p.meta_master.master_address or "127.0.0.1:0").split(":")[0]

    def _ha(self) -> bool:
        c = self.conf
        if c.get("alluxio.master.journal.type", "UFS").upper() == "EMBEDDED":
            return len([a for a in (c.get_raw("alluxio.master.embedded.journal.addresses") or "").split(",") if a]) > 1
        return c.get("alluxio.master.ha.primary.selector", "NONE").upper() != "NONE"

    def _target_dir(self, req) -> str:
        return req.targetDirectory or self.conf.get("alluxio.master.backup.directory", "/alluxio_backups")

    def standby_addresses(self) -> list[str]:
        return [a for a in self.p.meta_master.standby_rpc_addresses() if a != self.p.meta_master.master_address]

    # ---- entry point --------------------------------------------------------------------------
    def backup(self, req: pb.meta.BackupPRequest) -> pb.meta.BackupPStatus:
        with self._initiate:
            if self.tracker.in_progress():
                raise BackupException("Backup in progress")
            delegate = self.conf.get_bool("alluxio.master.backup.delegation.enabled", "false") and self._ha()
            standbys = self.standby_addresses() if delegate else []
            if delegate and not standbys:
                if req.options.allowLeader:
                    delegate = False
                else:
                    raise BackupDelegationException("No master found to delegate backup.")
            bid = self.tracker.reset(self._host())
        if delegate:
            if not self._schedule_remote(bid, req, standbys):
                err = BackupDelegationException("Failed to delegate the backup.")
                self.tracker.fail(err)
                raise err
        else:
            threading.Thread(target=self._local, args=(req,), daemon=True, name="backup-local").start()
        if req.options.runAsync:
            return pb.meta.BackupPStatus(backupId=bid, backupState=INITIATING)
        return self.tracker.wait_finished()

    def status(self, backup_id: str) -> pb.meta.BackupPStatus:
        return self.tracker.get(backup_id)

    # ---- local --------------------------------------------------------------------------------
    def _local(self, req) -> None:
        try:
            self.tracker.set_state(RUNNING)
            with self.p.state_lock.exclusive():
                path, n = write_backup(self.p.meta_master.masters_for_backup, self._target_dir(req))
            self.tracker.set_state(COMPLETED, backupUri=path, entryCount=n)
            LOG.info("backup %s written with %d entries", path, n)
        except Exception as e:  # noqa: BLE001
            LOG.exception("local backup failed")
            self.tracker.fail(e)

    # ---- delegated ----------------------------------------------------------------------------
    def _schedule_remote(self, bid: str, req, standbys: list[str]) -> bool:
        for addr in standbys:
            try:
                stub = self.p.peer_stub(addr, SVC_BACKUP_WORKER)
                stub.SuspendJournals(pb.meta.BackupSuspendPRequest())
                with self.p.state_lock.exclusive():
                    seqs = self.p.journal.sequence_numbers()
                msg = pb.meta.BackupDelegatePRequest(backupId=bid, request=req)
                for k, v in seqs.items():
                    msg.sequences.add(master=k, sequence=v)
                stub.DelegateBackup(msg)
                LOG.info("delegated backup %s to standby %s at sequences %s", bid, addr, seqs)
                self.tracker.set_state(TRANSITIONING, backupHost=addr.split(":")[0])
                self._poller = threading.Thread(target=self._poll_remote, args=(bid, addr), daemon=True,
                                                name="backup-remote-status")
                self._poller.start()
                return True
            except Exception as e:  # noqa: BLE001
                LOG.warning("failed to delegate backup to %s: %s", addr, e)
        return False

    def _poll_remote(self, bid: str, addr: str) -> None:
        interval = self.conf.get_ms("alluxio.master.backup.heartbeat.interval", "2sec") / 1000.0
        abandon = self.conf.get_ms("alluxio.master.backup.abandon.timeout", "1min") / 1000.0
        last_ok = time.monotonic()
        stub = self.p.peer_stub(addr, SVC_BACKUP_WORKER)
        while self.tracker.in_progress():
            try:
                st = stub.GetBackupStatus(pb.meta.BackupStatusPRequest(backupId=bid))
                last_ok = time.monotonic()
                self.tracker.update(st)
                if st.backupState in (COMPLETED, FAILED):
                    return
            except Exception as e:  # noqa: BLE001
                if time.monotonic() - last_ok > abandon:
                    self.tracker.fail(f"backup worker {addr} abandoned the backup: {e}")
                    return
            time.sleep(min(interval, 0.2) if self.tracker.in_progress() else 0)


class BackupWorkerRole:
    """Standby side of a delegated backup (served as ``BackupWorkerService`` even on standbys)."""

    def __init__(self, process):
        self.p = process
        self.conf = process.conf
        self._lock = threading.Lock()
        self._statuses: dict[str, pb.meta.BackupPStatus] = {}
        self._resume_timer: threading.Timer | None = None
        self._suspended = False

    def _resume(self) -> None:
        with self._lock:
            if self._suspended:
                try:
                    self.p.journal.resume()
                finally:
                    self._suspended = False

    # ---- RPCs ---------------------------------------------------------------------------------
    def SuspendJournals(self, req, ctx):  # noqa: N802
        if self.p.primary:
            raise FailedPreconditionException("the primary master cannot act as a backup worker")
        with self._lock:
            if self._suspended:
                raise BackupException("journals already suspended for a backup")
            self.p.journal.suspend()
            self._suspended = True
            timeout = self.conf.get_ms("alluxio.master.backup.transport.timeout", "30sec") / 1000.0
            self._resume_timer = threading.Timer(timeout, self._resume)
            self._resume_timer.daemon = True
            self._resume_timer.start()
        LOG.info("journals suspended for a delegated backup")
        return pb.meta.BackupSuspendPResponse()

    def DelegateBackup(self, req, ctx):  # noqa: N802
        with self._lock:
            if self._resume_timer is not None:
                self._resume_timer.cancel()
                self._resume_timer = None
            if not self._suspended:
                raise BackupException("Journal has been resumed due to a time-out")
            st = pb.meta.BackupPStatus(backupId=req.backupId, backupState=TRANSITIONING,
                                       backupHost=(self.p.address or "").split(":")[0])
            self._statuses[req.backupId] = st
        seqs = {s.master: s.sequence for s in req.sequences}
        threading.Thread(target=self._run, args=(req, seqs), daemon=True, name="backup-worker").start()
        return pb.meta.BackupDelegatePResponse()

    def GetBackupStatus(self, req, ctx):  # noqa: N802
        with self._lock:
            st = self._statuses.get(req.backupId)
            if st is None:
                return pb.meta.BackupPStatus(backupId=req.backupId, backupState=S.values_by_name["None"].number)
            out = pb.meta.BackupPStatus()
            out.CopyFrom(st)
            return out

    def _set(self, bid: str, **fields) -> None:
        with self._lock:
            st = self._statuses[bid]
            for k, v in fields.items():
                setattr(st, k, v)

    def _run(self, req, seqs) -> None:
        bid = req.backupId
        try:
            timeout = self.conf.get_ms("alluxio.master.backup.abandon.timeout", "1min") / 1000.0
            self.p.journal.catchup(seqs, timeout)
            self._set(bid, backupState=RUNNING)
            target = req.request.targetDirectory or self.conf.get("alluxio.master.backup.directory",
                                                                  "/alluxio_backups")
            path, n = write_backup(self.p.meta_master.masters_for_backup, target)
            self._set(bid, backupState=COMPLETED, backupUri=path, entryCount=n)
            LOG.info("delegated backup %s written to %s (%d entries)", bid, path, n)
        except Exception as e:  # noqa: BLE001
            LOG.exception("delegated backup failed")
            self._set(bid, backupState=FAILED, backupError=str(e).encode())
        finally:
            self._resume()


class DailyMetadataBackup:
    """Backup once a day at ``alluxio.master.daily.backup.time`` (HH:MM, UTC), keeping the newest
    ``alluxio.master.daily.backup.files.retained`` backups in the backup directory."""

    def __init__(self, leader: BackupLeaderRole, conf):
        self.leader = leader
        self.conf = conf
        hh, _, mm = conf.get("alluxio.master.daily.backup.time", "05:00").partition(":")
        self.hour, self.minute = int(hh), int(mm or 0)
        self.retained = conf.get_int("alluxio.master.daily.backup.files.retained", "3")
        self.directory = conf.get("alluxio.master.backup.directory", "/alluxio_backups")
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None

    def seconds_until_next(self, now: datetime.datetime | None = None) -> float:
        now = now or datetime.datetime.now(datetime.timezone.utc)
        nxt = now.replace(hour=self.hour, minute=self.minute, second=0, microsecond=0)
        if nxt <= now:
            nxt += datetime.timedelta(days=1)
        return (nxt - now).total_seconds()

    def run_once(self) -> pb.meta.BackupPStatus:
        st = self.leader.backup(pb.meta.BackupPRequest(
            targetDirectory=self.directory, options=pb.meta.BackupPOptions(allowLeader=True)))
        if st.backupState == COMPLETED:
            self.delete_stale()
        else:
            LOG.warning("daily backup ended %s: %s", enum_name(S, st.backupState), st.backupError)
        return st

    def delete_stale(self) -> list[str]:
        try:
            names = sorted(n for n in os.listdir(self.directory) if n.startswith(BACKUP_PREFIX) and n.endswith(".gz"))
        except FileNotFoundError:
            return []
        stale = names[:-self.retained] if self.retained > 0 else names
        for n in stale:
            try:
                os.remove(os.path.join(self.directory, n))
            except OSError:
                pass
        return stale

    def start(self) -> None:
        self._stop = stop = threading.Event()

        def loop():
            while not stop.wait(self.seconds_until_next()):
                try:
                    self.run_once()
                except Exception:  # noqa: BLE001
                    LOG.exception("daily backup failed")
        self._thread = threading.Thread(target=loop, daemon=True, name="daily-backup")
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()


class MetaMasterSync:
    """Standby -> primary registration and heartbeat (MetaMasterSync.java)."""

    def __init__(self, process, primary_addresses):
        self.p = process
        self.primary_addresses = primary_addresses   # callable -> list of candidate addresses
        self.master_id: int | None = None

    def _stub(self):
        from ..rpc import master_channel
        addrs = [a for a in self.primary_addresses() if a and a != self.p.address]
        if not addrs:
            raise UnavailableException("no primary master address known")
        return master_channel(addrs).stub(SVC_META_MASTER)

    def heartbeat(self) -> None:
        if self.p.primary:
            self.master_id = None
            return
        try:
            stub = self._stub()
            if self.master_id is None:
                host, _, port = self.p.address.partition(":")
                self.master_id = stub.GetMasterId(pb.meta.GetMasterIdPRequest(
                    masterAddress=pb.grpc.NetAddress(host=host, rpcPort=int(port)))).masterId
                stub.RegisterMaster(pb.meta.RegisterMasterPRequest(masterId=self.master_id))
                return
            cmd = stub.MasterHeartbeat(pb.meta.MasterHeartbeatPRequest(masterId=self.master_id)).command
            if enum_name(pb.meta.MetaCommand, cmd) == "MetaCommand_Register":
                self.master_id = None
        except AlluxioStatusException as e:
            LOG.debug("standby heartbeat to the primary failed: %s", e)
            self.master_id = None
