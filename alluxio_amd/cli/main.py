"""``alluxio`` launcher: ``python -m alluxio_amd <command> [args]``.

Parity: bin/alluxio:201-386 (format, formatJournal, formatMasters, formatWorker, fs, fsadmin,
getConf, job, logLevel, readJournal, runClass, runTests, runUfsTests, runJournalCrashTest, upgradeJournal,
validateConf, validateEnv, version) and bin/alluxio-start.sh (master / worker / job_master /
job_worker / proxy / fuse / logserver processes).
"""
from __future__ import annotations

import os
import shutil
import sys

USAGE = """Usage: alluxio COMMAND [GENERIC_COMMAND_OPTIONS] [COMMAND_ARGS]

COMMAND is one of:
  format [-s]           Format Alluxio master and all workers (-s: only if not formatted)
  formatJournal         Format Alluxio master journal locally
  formatMasters         Format Alluxio master nodes
  formatWorker          Format Alluxio worker nodes
  bootstrapConf         Generate a config file if one doesn't exist
  fs                    Command line tool for interacting with the Alluxio filesystem.
  fsadmin               Command line tool for use by Alluxio filesystem admins.
  getConf [key]         Look up a configuration key, or print all configuration.
  job                   Command line tool for interacting with the job service.
  table                 Command line tool for interacting with the table (catalog) service.
  logLevel              Set or get log level of Alluxio servers.
  readJournal           Read an Alluxio journal file from stdin and write a human-readable version of it to stdout.
  runClass              Run the main function of a module (``pkg.module`` or ``pkg.module:function``).
  runTests              Run all end-to-end tests on an Alluxio cluster.
  runUfsTests --path P   Test an under storage against the UFS contract (UnderFileSystemContractTest).
  yarn submit|status|stop  Run the cluster as YARN applications (ResourceManager REST API).
  upgradeJournal        Upgrade an Alluxio journal from v0 to v1 (-journalDirectoryV0 <dir>).
  stress                Run a stress benchmark (master|worker|client-io|ufs-io|max-throughput).
  validateConf          Validate Alluxio conf and exit.
  validateEnv           Validate Alluxio environment.
  version               Print Alluxio version and exit.
  master | worker | proxy | fuse | logserver    Start a server process in the foreground.
"""


def _conf():
    from ..conf import Configuration
    return Configuration(load_site=True)


def _master_journal(conf):
    """The journal system with the standard masters' journals registered (names only)."""
    from ..journal.system import Journaled
    from ..master.process import build_journal_system
    j = build_journal_system(conf)
    for name in ("BlockMaster", "FileSystemMaster", "MetaMaster"):
        stub = Journaled()
        stub.journal_name = name
        j.register(stub)
    return j


def run_class(args, out=None) -> int:
    """``alluxio runClass <module[:function]> [args]`` (bin/alluxio runClass)."""
    import importlib
    if not args:
        print("Usage: alluxio runClass <module[:function]> [args...]", file=out or sys.stdout)
        return 1
    mod, _, fn = args[0].partition(":")
    target = getattr(importlib.import_module(mod), fn or "main")
    rc = target(args[1:])
    return rc if isinstance(rc, int) else 0


def format_journal(conf=None, out=None) -> None:
    conf = conf or _conf()
    _master_journal(conf).format()
    print(f"Formatted journal at {conf.get('alluxio.master.journal.folder')}", file=out or sys.stdout)


def format_worker(conf=None, out=None) -> None:
    """Delete the file-backed tier dirs' block data (reference Format.format(WORKER))."""
    conf = conf or _conf()
    from ..conf.keys import Templates
    for lvl in range(conf.get_int("alluxio.worker.tieredstore.levels")):
        for p in conf.get_list(Templates.WORKER_TIERED_STORE_LEVEL_DIRS_PATH.format(lvl)):
            if p.startswith(("hbm", "dram", "auto")):
                continue  # device/host arenas hold no state across restarts
            d = os.path.join(p, conf.get("alluxio.worker.data.folder", "alluxioworker").strip("/"))
            if os.path.isdir(d):
                shutil.rmtree(d)
            os.makedirs(d, exist_ok=True)
            print(f"Formatted worker data folder {d}", file=out or sys.stdout)


def get_conf(argv, out=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(prog="alluxio getConf")
    ap.add_argument("--master", action="store_true")
    ap.add_argument("--source", action="store_true")
    ap.add_argument("--unit", default=None, choices=["B", "KB", "MB", "GB", "TB", "MS", "S", "MIN", "HR", "DAY"])
    ap.add_argument("key", nargs="?")
    a = ap.parse_args(argv)
    out = out or sys.stdout
    if a.master:
        from ..client.context import FileSystemContext
        from ..proto import pb
        ctx = FileSystemContext()
        r = ctx.meta_config().GetConfiguration(pb.meta.GetConfigurationPOptions())
        props = {c.name: (c.value, c.source) for c in r.clusterConfigs}
    else:
        conf = _conf()
        props = {k: (conf.get(k), conf.source(k).name) for k in conf.to_map(include_defaults=True)}
    if a.key:
        if a.key not in props:
            print("", file=out)
            return 1
        v, src = props[a.key]
        if a.unit and v is not None:
            from ..utils.format import parse_space_size, parse_time_size
            div = {"B": 1, "KB": 1 << 10, "MB": 1 << 20, "GB": 1 << 30, "TB": 1 << 40}
            tdiv = {"MS": 1, "S": 1000, "MIN": 60_000, "HR": 3_600_000, "DAY": 86_400_000}
            v = parse_space_size(v) // div[a.unit] if a.unit in div else parse_time_size(v) // tdiv[a.unit]
        print(f"{v} ({src})" if a.source else ("" if v is None else v), file=out)
        return 0
    for k in sorted(props):
        v, src = props[k]
        print(f"{k}={'' if v is None else v}" + (f" ({src})" if a.source else ""), file=out)
    return 0


def log_level(argv, out=None) -> int:
    """``logLevel --logName <name> [--level <LEVEL>]`` on this process's loggers (servers expose
    the same through their web endpoint ``/api/v1/logLevel``)."""
    import argparse
    import logging
    ap = argparse.ArgumentParser(prog="alluxio logLevel")
    ap.add_argument("--logName", required=True)
    ap.add_argument("--level", default=None)
    ap.add_argument("--target", default=None)
    a = ap.parse_args(argv)
    if a.target:
        import json
        import urllib.request
        for t in a.target.split(","):
            q = f"http://{t}/api/v1/logLevel?logName={a.logName}" + (f"&level={a.level}" if a.level else "")
            with urllib.request.urlopen(urllib.request.Request(q, method="POST"), timeout=10) as r:
                print(f"{t}{json.loads(r.read())}", file=out or sys.stdout)
        return 0
    lg = logging.getLogger(a.logName)
    if a.level:
        lg.setLevel(a.level.upper())
    print(f"{a.logName} level={logging.getLevelName(lg.getEffectiveLevel())}", file=out or sys.stdout)
    return 0


def main(argv=None, out=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    out = out or sys.stdout
    if not argv:
        print(USAGE, file=out)
        return 1
    cmd, rest = argv[0], argv[1:]
    if cmd == "fs":
        from .fs_shell import main as m
        return m(rest, out)
    if cmd == "table":
        from ..table import TableShell
        return TableShell(out=out).run(rest)
    if cmd == "fsadmin":
        from .fsadmin import main as m
        return m(rest, out)
    if cmd == "job":
        from .job_shell import main as m
        return m(rest, out)
    if cmd in ("format", "formatMasters", "formatJournal", "formatWorker"):
        conf = _conf()
        if cmd == "format" and "-s" in rest:
            if _master_journal(conf).is_formatted():
                print("Journal is already formatted; skipping (-s).", file=out)
                return 0
        if cmd in ("format", "formatMasters", "formatJournal"):
            format_journal(conf, out)
        if cmd in ("format", "formatWorker"):
            format_worker(conf, out)
        return 0
    if cmd == "bootstrapConf":
        from ..conf import site_properties_path
        path = site_properties_path()
        if os.path.exists(path):
            print(f"{path} already exists", file=out)
            return 0
        master = rest[0] if rest else "localhost"
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(f"alluxio.master.hostname={master}\n")
            f.write("alluxio.worker.tieredstore.level0.alias=MEM\n")
            f.write("alluxio.worker.tieredstore.level0.dirs.path=hbm\n")
        print(f"wrote {path}", file=out)
        return 0
    if cmd == "getConf":
        return get_conf(rest, out)
    if cmd == "logLevel":
        return log_level(rest, out)
    if cmd == "readJournal":
        from .journal_tool import main as m
        return m(rest, out)
    if cmd == "runTests":
        from .test_runner import main as m
        return m(rest, out)
    if cmd == "runUfsTests":
        from .ufs_contract import main as m
        return m(rest, out)
    if cmd == "yarn":
        from ..yarn import main as m
        return m(rest, out)
    if cmd == "upgradeJournal":
        from ..journal.upgrade import main as m
        return m(rest, out)
    if cmd == "runClass":
        return run_class(rest, out)
    if cmd == "validateEnv":
        from .validate import main_env
        return main_env(rest, out)
    if cmd == "validateConf":
        from .validate import main_conf
        return main_conf(rest, out)
    if cmd == "version":
        from .. import __version__
        print(f"Alluxio (MI355X-native) version: {__version__}", file=out)
        return 0
    if cmd == "stress":
        from ..stress.__main__ import main as m
        return m(rest)
    if cmd == "master":
        from ..master.process import main as m
        return m(rest)
    if cmd == "worker":
        from ..worker.process import main as m
        return m(rest)
    if cmd == "proxy":
        from ..proxy import main as m
        return m(rest)
    if cmd == "fuse":
        from ..fuse import main as m
        return m(rest)
    if cmd == "logserver":
        from ..web.logserver import main as m
        return m(rest)
    print(f"Unknown command: {cmd}\n{USAGE}", file=out)
    return 1


if __name__ == "__main__":  # pragma: no cover
    raise SystemExit(main())
