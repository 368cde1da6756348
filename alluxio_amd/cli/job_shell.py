"""``alluxio job`` — job-service shell (reference shell/src/main/java/alluxio/cli/job/JobShell.java,
command/{Cancel,Leader,List,Stat}Command.java)."""
from __future__ import annotations

import sys

from ..proto import enum_name, pb
from ..utils.exceptions import AlluxioStatusException


class JobShell:
    def __init__(self, channel=None, out=None, conf=None):
        if channel is None:
            from ..client.context import FileSystemContext
            channel = FileSystemContext(conf).master_channel()
        from ..job import JobClient
        self.jc = JobClient(channel)
        self.channel = channel
        self.out = out or sys.stdout

    def p(self, *a):
        print(*a, file=self.out)

    def run(self, argv) -> int:
        if not argv:
            self.p("Usage: alluxio job [cancel <id> | leader | ls | stat [-v] <id>]")
            return 1
        cmd, args = argv[0], argv[1:]
        try:
            if cmd == "cancel":
                self.jc.cancel(int(args[0]))
                return 0
            if cmd == "leader":
                mi = self.channel.stub("alluxio.grpc.meta.MetaMasterClientService").GetMasterInfo(
                    pb.meta.GetMasterInfoPOptions()).masterInfo
                self.p(mi.leaderMasterAddress)
                return 0
            if cmd == "ls":
                for j in sorted(self.jc.list(), key=lambda j: j.id):
                    self.p(f"{j.id:<16}{j.name:<16}{enum_name(pb.job.Status, j.status)}")
                return 0
            if cmd == "stat":
                verbose = "-v" in args
                jid = int([a for a in args if a != "-v"][0])
                info = self.jc.status(jid, detailed=verbose)
                self.p(f"ID: {info.id}")
                self.p(f"Name: {info.name}")
                self.p(f"Description: {info.description}")
                self.p(f"Status: {enum_name(pb.job.Status, info.status)}")
                if info.errorMessage:
                    self.p(f"Error: {info.errorMessage}")
                if info.result:
                    self.p(f"Result: {info.result.decode(errors='replace')}")
                if verbose:
                    for c in info.children:
                        self.p(f"Task {c.id}")
                        self.p(f"\tStatus: {enum_name(pb.job.Status, c.status)}")
                        if c.errorMessage:
                            self.p(f"\tError: {c.errorMessage}")
                return 0
        except AlluxioStatusException as e:
            self.p(str(e))
            return -1
        except (IndexError, ValueError):
            self.p(f"invalid arguments for {cmd}")
            return -1
        self.p(f"{cmd} is an unknown command.")
        return 1


def main(argv=None, out=None) -> int:
    return JobShell(out=out).run(list(sys.argv[1:] if argv is None else argv))
