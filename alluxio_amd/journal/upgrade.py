"""Legacy (v0) journal support and the v0 -> v1 upgrader (``alluxio upgradeJournal``).

Parity: core/server/common/src/main/java/alluxio/master/journalv0/ufs/UfsJournal.java (per-master
v0 layout: ``checkpoint.data``, ``log.out`` = current log, ``completed/log.%020d`` = finished logs,
ProtoBufJournalFormatter = varint-delimited ``JournalEntry``s), journalv0 JournalWriter
``recover`` / ``completeLogs`` (a dangling ``log.out`` becomes the next completed log) and
core/server/common/src/main/java/alluxio/master/journal/JournalUpgrader.java:114-206 (v0 checkpoint
-> ``checkpoints/0x0-0x<first log SN>``, each completed log -> ``logs/0x<start>-0x<end+1>``; no
checkpoint means nothing to upgrade).  Files are moved (renamed), as in the reference, so a v0
journal is consumed by the upgrade; back it up first.
"""
from __future__ import annotations

import logging
import os
import shutil

from . import format as fmt
from .ufs_journal import UfsJournal

LOG = logging.getLogger(__name__)

CHECKPOINT_V0 = "checkpoint.data"
CURRENT_LOG_V0 = "log.out"
COMPLETED_V0 = "completed"


def completed_log_v0(master_dir: str, n: int) -> str:
    return os.path.join(master_dir, COMPLETED_V0, f"log.{n:020d}")


def write_v0_journal(root: str, master: str, checkpoint_entries, logs, current=None) -> str:
    """Create a v0 journal (tests / migration fixtures): ``logs`` is a list of entry lists."""
    d = os.path.join(root, master)
    os.makedirs(os.path.join(d, COMPLETED_V0), exist_ok=True)
    with open(os.path.join(d, CHECKPOINT_V0), "wb") as f:
        for e in checkpoint_entries:
            fmt.write_delimited(f, e)
    for i, entries in enumerate(logs, start=1):
        with open(completed_log_v0(d, i), "wb") as f:
            for e in entries:
                fmt.write_delimited(f, e)
    if current:
        with open(os.path.join(d, CURRENT_LOG_V0), "wb") as f:
            for e in current:
                fmt.write_delimited(f, e)
    return d


def _complete_current_log(d: str) -> None:
    """journalv0 JournalWriter.completeLogs: the current log becomes the next completed log."""
    cur = os.path.join(d, CURRENT_LOG_V0)
    if not os.path.exists(cur):
        return
    if os.path.getsize(cur) == 0:
        os.remove(cur)
        return
    n = 1
    while os.path.exists(completed_log_v0(d, n)):
        n += 1
    os.makedirs(os.path.join(d, COMPLETED_V0), exist_ok=True)
    os.replace(cur, completed_log_v0(d, n))


def upgrade_master(v0_root: str, v1_root: str, master: str) -> dict:
    """Upgrade one master's journal; returns what was moved."""
    d = os.path.join(v0_root, master)
    ckpt = os.path.join(d, CHECKPOINT_V0)
    if not os.path.exists(ckpt):
        LOG.info("No checkpoint is found for %s. No upgrade is required.", master)
        return {"master": master, "upgraded": False, "logs": 0}
    _complete_current_log(d)
    j = UfsJournal(v1_root, master)
    if not j.is_formatted():
        j.format()
    j.ensure()
    n, moved, checkpoint_end = 1, 0, None
    while os.path.exists(completed_log_v0(d, n)):
        path = completed_log_v0(d, n)
        with open(path, "rb") as f:
            seqs = [e.sequence_number for e in fmt.iter_delimited(f)]
        n += 1
        if not seqs:
            os.remove(path)
            continue
        start, end = seqs[0], seqs[-1]
        if checkpoint_end is None:
            checkpoint_end = start
            _move_checkpoint(j, ckpt, start)
        dst = os.path.join(j.log_dir, fmt.encode_file_name(start, end + 1))
        shutil.move(path, dst)
        moved += 1
    if checkpoint_end is None:
        checkpoint_end = 1
        _move_checkpoint(j, ckpt, 1)
    LOG.info("Finished upgrading %s journal (%d logs).", master, moved)
    return {"master": master, "upgraded": True, "logs": moved, "checkpoint_end": checkpoint_end}


def _move_checkpoint(j: UfsJournal, ckpt_v0: str, end: int) -> None:
    # a v1 checkpoint is typed; the v0 payload is the JOURNAL_ENTRY kind (delimited entries)
    with open(ckpt_v0, "rb") as f:
        payload = f.read()
    j.write_checkpoint(end, fmt.CheckpointType.JOURNAL_ENTRY, payload)
    os.remove(ckpt_v0)


def upgrade(v0_root: str, v1_root: str, masters=None) -> list[dict]:
    masters = masters or sorted(n for n in os.listdir(v0_root) if os.path.isdir(os.path.join(v0_root, n)))
    return [upgrade_master(v0_root, v1_root, m) for m in masters]


def main(argv=None, out=None) -> int:
    import argparse
    import sys
    out = out or sys.stdout
    ap = argparse.ArgumentParser(prog="alluxio upgradeJournal",
                                 description="Upgrades journal from v0 to v1 (back up the v0 journal first).")
    ap.add_argument("-journalDirectoryV0", "--journalDirectoryV0", default=None)
    a = ap.parse_args(argv)
    from ..conf import Configuration
    conf = Configuration(load_site=True)
    v1 = conf.get("alluxio.master.journal.folder")
    if v1.startswith("file://"):
        v1 = v1[len("file://"):]
    v0 = a.journalDirectoryV0 or v1
    for r in upgrade(v0, v1):
        print(f"{r['master']}: {'upgraded ' + str(r['logs']) + ' log(s)' if r['upgraded'] else 'nothing to upgrade'}",
              file=out)
    return 0
