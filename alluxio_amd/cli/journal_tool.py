"""``alluxio readJournal`` — dump a UFS or embedded (Raft) journal as text.

Parity: core/server/master/src/main/java/alluxio/master/journal/tool/JournalTool.java (dumps
the latest checkpoint and the log entries in [start, end) of one master's journal into an
output directory: ``checkpoints/`` and ``edits.txt``) and RaftJournalDumper.java (embedded
journal: the latest snapshot + the committed Raft log, one master's entries or all of them).
"""
from __future__ import annotations

import os
import sys

from google.protobuf import text_format


def dump_journal(journal_dir: str, master: str, output_dir: str, start: int = 0, end: int = 2 ** 63 - 1,
                 out=None) -> int:
    from ..journal.ufs_journal import UfsJournal
    out = out or sys.stdout
    j = UfsJournal(journal_dir, master)
    if not j.is_formatted():
        raise FileNotFoundError(f"no journal for {master} under {journal_dir}")
    os.makedirs(output_dir, exist_ok=True)
    ctype, payload, cp_end = j.read_checkpoint()
    if ctype is not None:
        from ..journal import checkpoint as ck
        cdir = os.path.join(output_dir, "checkpoints")
        os.makedirs(cdir, exist_ok=True)
        with open(os.path.join(cdir, f"0x0-0x{cp_end:x}.{ctype.name}"), "wb") as f:
            f.write(payload)
        # human-readable outline (reference CheckpointFormat.parseToHumanReadable)
        with open(os.path.join(cdir, f"0x0-0x{cp_end:x}.txt"), "w") as f:
            f.write("\n".join(ck.describe(ck.parse(ck.typed(ctype, payload), master))) + "\n")
        print(f"Checkpoint type {ctype.name} covering [0, {cp_end}) written to {cdir}", file=out)
    n = 0
    with open(os.path.join(output_dir, "edits.txt"), "w") as f:
        for e in j.iter_log_entries(max(start, cp_end if ctype is not None and start < cp_end else start)):
            if e.sequence_number >= end:
                break
            f.write(text_format.MessageToString(e))
            f.write("\n")
            n += 1
    print(f"Dumped {n} journal entries of {master} to {output_dir}/edits.txt", file=out)
    return n


def dump_raft_journal(journal_dir: str, master: str | None, output_dir: str, start: int = 0,
                      end: int = 2 ** 63 - 1, out=None) -> int:
    """Embedded journal under ``<journal_dir>/raft``: snapshot parts + log entries (by global SN)."""
    from ..journal import format as fmt
    from ..journal.raft import KIND_JOURNAL, RaftStorage
    from ..proto import pb
    out = out or sys.stdout
    root = os.path.join(journal_dir, "raft")
    if not os.path.isdir(root):
        raise FileNotFoundError(f"no embedded journal under {journal_dir}")
    st = RaftStorage(root, fsync=False)
    os.makedirs(output_dir, exist_ok=True)
    try:
        if st.snapshot_path:
            cdir = os.path.join(output_dir, "checkpoints")
            os.makedirs(cdir, exist_ok=True)
            with open(st.snapshot_path, "rb") as f:
                hdr = fmt.read_delimited(f, pb.raft.RaftSnapshotHeader)
                from ..journal import checkpoint as ck
                for name, cp in fmt.read_compound(f):
                    if master in (None, "", name):
                        base = os.path.join(cdir, f"{name}-0x0-0x{hdr.nextSequenceNumber:x}")
                        with open(base, "wb") as g:
                            g.write(ck.typed(cp.type, cp.body))
                        with open(base + ".txt", "w") as g:
                            g.write("\n".join(ck.describe(cp)) + "\n")
            print(f"Snapshot at raft index {hdr.index} (term {hdr.term}, next SN {hdr.nextSequenceNumber}, "
                  f"peers {list(hdr.peers)}) written to {cdir}", file=out)
        n = 0
        with open(os.path.join(output_dir, "edits.txt"), "w") as f:
            for idx, term, payload in st.entries(st.base_index + 1):
                if payload[:1] != KIND_JOURNAL:
                    continue
                for ne in pb.raft.RaftCommand.FromString(payload[1:]).entries:
                    sn = ne.entry.sequence_number
                    if sn < start or sn >= end or master not in (None, "", ne.master):
                        continue
                    f.write(f"# raft index {idx} term {term} master {ne.master}\n")
                    f.write(text_format.MessageToString(ne.entry))
                    f.write("\n")
                    n += 1
    finally:
        st.close()
    print(f"Dumped {n} journal entries to {output_dir}/edits.txt", file=out)
    return n


def main(argv=None, out=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(prog="alluxio readJournal")
    ap.add_argument("-master", "--master", default="FileSystemMaster")
    ap.add_argument("-start", "--start", type=int, default=0)
    ap.add_argument("-end", "--end", type=int, default=2 ** 63 - 1)
    ap.add_argument("-inputDir", "--inputDir", default=None)
    ap.add_argument("-outputDir", "--outputDir", default=None)
    a = ap.parse_args(argv)
    from ..conf import Configuration
    conf = Configuration(load_site=True)
    jdir = a.inputDir or conf.get("alluxio.master.journal.folder")
    if jdir.startswith("file://"):
        jdir = jdir[len("file://"):]
    outdir = a.outputDir or os.path.join(os.getcwd(), f"journal_dump-{os.getpid()}")
    if os.path.isdir(os.path.join(jdir, "raft")):
        dump_raft_journal(jdir, a.master, outdir, a.start, a.end, out)
    else:
        dump_journal(jdir, a.master, outdir, a.start, a.end, out)
    return 0
