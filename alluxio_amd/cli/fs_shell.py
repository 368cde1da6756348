"""``alluxio fs`` — the file-system shell.

Parity: shell/src/main/java/alluxio/cli/fs/FileSystemShell.java and the 47 commands under
shell/src/main/java/alluxio/cli/fs/command/ (Cat, CheckConsistency, Checksum, Chgrp, Chmod,
Chown, CopyFromLocal, CopyToLocal, Count, Cp, DistributedCp, DistributedLoad, DistributedMv, Du,
Free, GetCapacityBytes, GetFacl, GetSyncPathList, GetUsedBytes, Head, Help, Leader, Load,
LoadMetadata, Location, Ls (LsCommand.java:54-66 column layout), MasterInfo, Mkdir, Mount, Mv,
Persist, Pin, Rm, SetFacl, SetReplication, SetTtl, StartSync, Stat, StopSync, Tail, Test, Touch,
Unmount, Unpin, UnsetTtl, UpdateMount).  Commands write to ``out`` and return an exit code so
tests can drive the shell in-process.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shlex
import sys
import time

from ..proto import enum_name, pb
from ..utils.exceptions import AlluxioStatusException, NotFoundException
from ..utils.format import bytes_to_human, mode_to_string, parse_time_size

COMMANDS: dict[str, tuple] = {}


def command(name, usage, desc):
    def deco(fn):
        COMMANDS[name] = (fn, usage, desc)
        return fn
    return deco


class _Parser(argparse.ArgumentParser):
    def error(self, message):
        raise ValueError(message)


def _parser(name, usage):
    return _Parser(prog=f"alluxio fs {name}", usage=usage, add_help=False)


def _is_local(p: str) -> bool:
    return p.startswith("file://")


def _local(p: str) -> str:
    return p[len("file://"):] if p.startswith("file://") else p


def _fmt_time(ms: int) -> str:
    return time.strftime("%m-%d-%Y %H:%M:%S", time.localtime(ms / 1000.0)) + f":{ms % 1000:03d}"


def _expand(fs, path: str) -> list[str]:
    """Glob expansion over the Alluxio namespace (``*`` / ``?`` in the last components)."""
    if not any(c in path for c in "*?["):
        return [path]
    import fnmatch
    parts = path.rstrip("/").split("/")
    cur = ["/"]
    for comp in parts[1:]:
        nxt = []
        for base in cur:
            if any(c in comp for c in "*?["):
                try:
                    for s in fs.list_status(base):
                        if fnmatch.fnmatch(s.name, comp):
                            nxt.append(s.path)
                except NotFoundException:
                    pass
            else:
                nxt.append(base.rstrip("/") + "/" + comp)
        cur = nxt
    return sorted(cur)


class FileSystemShell:
    def __init__(self, fs=None, out=None, conf=None, job_client=None):
        if fs is None:
            from ..client.file_system import FileSystem
            fs = FileSystem(conf=conf)
        self.fs = fs
        self.out = out or sys.stdout
        self._job_client = job_client

    def p(self, *a):
        print(*a, file=self.out)

    def job_client(self):
        if self._job_client is None:
            from ..job import JobClient
            self._job_client = JobClient(self.fs.ctx.master_channel())
        return self._job_client

    def run(self, argv: list[str]) -> int:
        if isinstance(argv, str):
            argv = shlex.split(argv)
        if not argv:
            self.usage()
            return 1
        name, args = argv[0], argv[1:]
        ent = COMMANDS.get(name)
        if ent is None:
            self.p(f"{name} is an unknown command.")
            self.usage()
            return 1
        fn, usage, _ = ent
        try:
            return fn(self, args) or 0
        except ValueError as e:
            self.p(f"Usage: {usage}\n{e}")
            return -1
        except AlluxioStatusException as e:
            self.p(str(e))
            return -1
        except (OSError, IOError) as e:
            self.p(str(e))
            return -1

    def usage(self):
        self.p("Usage: alluxio fs [generic options]")
        for name in sorted(COMMANDS):
            self.p(f"\t [{COMMANDS[name][1]}]")


# ---- read / write -------------------------------------------------------------------------------
@command("cat", "cat <path>", "Prints the file's contents to the console.")
def _cat(sh, args):
    a = _parser("cat", "cat <path>")
    a.add_argument("path")
    ns = a.parse_args(args)
    for path in _expand(sh.fs, ns.path):
        st = sh.fs.get_status(path)
        if st.is_folder:
            sh.p(f"Path \"{path}\" must be a file.")
            return -1
        with sh.fs.open_file(path) as f:
            data = f.read()
        sh.out.write(data.decode("utf-8", errors="replace"))
    return 0


@command("head", "head -c <number> <path>", "Prints the file's first n bytes (by default, 1KB) to the console.")
def _head(sh, args):
    a = _parser("head", "head -c <number> <path>")
    a.add_argument("-c", default="1KB")
    a.add_argument("path")
    ns = a.parse_args(args)
    from ..utils.format import parse_space_size
    n = parse_space_size(ns.c)
    with sh.fs.open_file(ns.path) as f:
        sh.out.write(f.read(n).decode("utf-8", errors="replace"))
    return 0


@command("tail", "tail -c <number> <path>", "Prints the file's last n bytes (by default, 1KB) to the console.")
def _tail(sh, args):
    a = _parser("tail", "tail -c <number> <path>")
    a.add_argument("-c", default="1KB")
    a.add_argument("path")
    ns = a.parse_args(args)
    from ..utils.format import parse_space_size
    n = parse_space_size(ns.c)
    st = sh.fs.get_status(ns.path)
    with sh.fs.open_file(ns.path, status=st) as f:
        f.seek(max(0, st.length - n))
        sh.out.write(f.read().decode("utf-8", errors="replace"))
    return 0


@command("touch", "touch <path>", "Creates a 0 byte file. The file will be written to the under file system.")
def _touch(sh, args):
    a = _parser("touch", "touch <path>")
    a.add_argument("path")
    ns = a.parse_args(args)
    sh.fs.create_file(ns.path, write_type="THROUGH").close()
    sh.p(f"{ns.path} has been created")
    return 0


@command("mkdir", "mkdir <path1> [path2] ... [pathn]", "Creates the specified directories, including any parent directories that are required.")
def _mkdir(sh, args):
    if not args:
        raise ValueError("mkdir requires at least 1 argument")
    for p in args:
        sh.fs.create_directory(p, recursive=True)
        sh.p(f"Successfully created directory {p}")
    return 0


def _copy_local_to_alluxio(sh, src, dst, write_type=None, buffer=8 << 20):
    if os.path.isdir(src):
        sh.fs.create_directory(dst, recursive=True, allow_exists=True)
        n = 0
        for name in sorted(os.listdir(src)):
            n += _copy_local_to_alluxio(sh, os.path.join(src, name), dst.rstrip("/") + "/" + name, write_type)
        return n
    with open(src, "rb") as fin, sh.fs.create_file(dst, write_type=write_type) as fout:
        while True:
            b = fin.read(buffer)
            if not b:
                break
            fout.write(b)
    return 1


def _copy_alluxio_to_local(sh, src, dst, buffer=8 << 20):
    st = sh.fs.get_status(src)
    if st.is_folder:
        os.makedirs(dst, exist_ok=True)
        n = 0
        for c in sh.fs.list_status(src):
            n += _copy_alluxio_to_local(sh, c.path, os.path.join(dst, c.name))
        return n
    if os.path.isdir(dst):
        dst = os.path.join(dst, st.name)
    tmp = dst + ".alluxio_tmp"
    with sh.fs.open_file(src, status=st) as fin, open(tmp, "wb") as fout:
        while True:
            b = fin.read(buffer)
            if not b:
                break
            fout.write(b)
    os.replace(tmp, dst)
    return 1


def _copy_alluxio(sh, src, dst, recursive):
    st = sh.fs.get_status(src)
    if st.is_folder:
        if not recursive:
            raise IOError(f"{src} is a directory, to copy it please use \"cp -R <src> <dst>\"")
        sh.fs.create_directory(dst, recursive=True, allow_exists=True)
        return sum(_copy_alluxio(sh, c.path, dst.rstrip("/") + "/" + c.name, True) for c in sh.fs.list_status(src))
    try:
        if sh.fs.get_status(dst).is_folder:
            dst = dst.rstrip("/") + "/" + st.name
    except NotFoundException:
        pass
    with sh.fs.open_file(src, status=st) as fin, sh.fs.create_file(dst) as fout:
        while True:
            b = fin.read(8 << 20)
            if not b:
                break
            fout.write(b)
    return 1


@command("cp", "cp [-R] [--buffersize <bytes>] <src> <dst>", "Copies a file or a directory in the Alluxio filesystem or between local filesystem and Alluxio filesystem.")
def _cp(sh, args):
    a = _parser("cp", "cp [-R] <src> <dst>")
    a.add_argument("-R", action="store_true", dest="recursive")
    a.add_argument("--buffersize", default=None)
    a.add_argument("--thread", type=int, default=1)
    a.add_argument("src")
    a.add_argument("dst")
    ns = a.parse_args(args)
    if _is_local(ns.src) and _is_local(ns.dst):
        raise ValueError("cp between two local paths is not supported")
    if _is_local(ns.src):
        _copy_local_to_alluxio(sh, _local(ns.src), ns.dst)
        sh.p(f"Copied {ns.src} to {ns.dst}")
    elif _is_local(ns.dst):
        for src in _expand(sh.fs, ns.src):
            _copy_alluxio_to_local(sh, src, _local(ns.dst))
            sh.p(f"Copied {src} to {ns.dst}")
    else:
        for src in _expand(sh.fs, ns.src):
            _copy_alluxio(sh, src, ns.dst, ns.recursive)
            sh.p(f"Copied {src} to {ns.dst}")
    return 0


@command("copyFromLocal", "copyFromLocal [--thread <num>] [--buffersize <bytes>] <src> <remoteDst>", "Copies a file or a directory from local filesystem to Alluxio filesystem.")
def _cfl(sh, args):
    pos = [x for x in args if not x.startswith("-")]
    if len(pos) != 2:
        raise ValueError("copyFromLocal requires 2 arguments")
    return _cp(sh, ["file://" + os.path.abspath(_local(pos[0])), pos[1]])


@command("copyToLocal", "copyToLocal [--buffersize <bytes>] <src> <localDst>", "Copies a file or a directory from the Alluxio filesystem to the local filesystem.")
def _ctl(sh, args):
    pos = [x for x in args if not x.startswith("-")]
    if len(pos) != 2:
        raise ValueError("copyToLocal requires 2 arguments")
    return _cp(sh, [pos[0], "file://" + os.path.abspath(_local(pos[1]))])


@command("mv", "mv <src> <dst>", "Renames a file or directory.")
def _mv(sh, args):
    a = _parser("mv", "mv <src> <dst>")
    a.add_argument("src")
    a.add_argument("dst")
    ns = a.parse_args(args)
    dst = ns.dst
    try:
        if sh.fs.get_status(dst).is_folder:
            dst = dst.rstrip("/") + "/" + ns.src.rstrip("/").rsplit("/", 1)[-1]
    except NotFoundException:
        pass
    sh.fs.rename(ns.src, dst)
    sh.p(f"Renamed {ns.src} to {dst}")
    return 0


@command("rm", "rm [-R] [-U] [--alluxioOnly] <path>", "Removes the specified file. Specify -R to remove file or directory recursively.")
def _rm(sh, args):
    a = _parser("rm", "rm [-R] [-U] [--alluxioOnly] <path>")
    a.add_argument("-R", action="store_true", dest="recursive")
    a.add_argument("-r", action="store_true", dest="recursive2")
    a.add_argument("-U", action="store_true", dest="unchecked")
    a.add_argument("--alluxioOnly", action="store_true")
    a.add_argument("path")
    ns = a.parse_args(args)
    rec = ns.recursive or ns.recursive2
    for path in _expand(sh.fs, ns.path):
        st = sh.fs.get_status(path)
        if st.is_folder and not rec:
            raise IOError(f"{path} is a directory, to remove it, please use \"rm -R <path>\"")
        sh.fs.delete(path, recursive=rec, alluxio_only=ns.alluxioOnly, unchecked=ns.unchecked)
        sh.p(f"{path} has been removed" + (" only from Alluxio space" if ns.alluxioOnly else ""))
    return 0


# ---- listing / metadata -------------------------------------------------------------------------
def _ls_line(st, human: bool, timestamp: str = "lastModificationTime") -> str:
    i = st.info
    size = bytes_to_human(i.length) if human else str(i.length)
    if i.folder:
        size = str(len(i.blockIds)) if False else size
    ts = i.lastModificationTimeMs if timestamp == "lastModificationTime" else \
        (i.creationTimeMs if timestamp == "creationTime" else i.lastAccessTimeMs)
    perm = mode_to_string(i.mode, i.folder)
    if i.acl.entries:
        perm += "+"
    state = "" if i.folder else f"{i.inAlluxioPercentage}%"
    persist = "DIR" if i.folder else i.persistenceState
    return f"{perm:<12}{i.owner:<15}{i.group:<15}{size:>15}{persist:>16}{_fmt_time(ts):>24}{state:>5} {i.path}"


@command("ls", "ls [-d|-f|-p|-R|-h|--sort=option|--timestamp=option|-r] <path>", "Displays information for all files and directories directly under the specified path.")
def _ls(sh, args):
    a = _parser("ls", "ls [-d|-f|-p|-R|-h|--sort=option|-r] <path>")
    a.add_argument("-d", action="store_true", dest="dir_as_file")
    a.add_argument("-f", action="store_true", dest="force")
    a.add_argument("-p", action="store_true", dest="pinned")
    a.add_argument("-R", action="store_true", dest="recursive")
    a.add_argument("-h", action="store_true", dest="human")
    a.add_argument("-r", action="store_true", dest="reverse")
    a.add_argument("--sort", default=None, choices=["creationTime", "inMemoryPercentage", "lastAccessTime",
                                                   "lastModificationTime", "name", "path", "size"])
    a.add_argument("--timestamp", default="lastModificationTime",
                   choices=["creationTime", "lastAccessTime", "lastModificationTime"])
    a.add_argument("path", nargs="?", default="/")
    ns = a.parse_args(args)
    lm = "ALWAYS" if ns.force else "ONCE"
    for path in _expand(sh.fs, ns.path):
        st = sh.fs.get_status(path, load_metadata=lm)
        items = [st] if (ns.dir_as_file or not st.is_folder) else \
            sh.fs.list_status(path, recursive=ns.recursive, load_metadata=lm)
        if ns.pinned:
            items = [s for s in items if s.info.pinned]
        key = {"creationTime": lambda s: s.info.creationTimeMs, "inMemoryPercentage": lambda s: s.info.inMemoryPercentage,
               "lastAccessTime": lambda s: s.info.lastAccessTimeMs,
               "lastModificationTime": lambda s: s.info.lastModificationTimeMs,
               "name": lambda s: s.name, "path": lambda s: s.path, "size": lambda s: s.length}[ns.sort or "path"]
        items = sorted(items, key=key, reverse=ns.reverse)
        for s in items:
            sh.p(_ls_line(s, ns.human, ns.timestamp))
    return 0


@command("stat", "stat [-f <format>] <path>", "Displays info for the specified path both file and directory.")
def _stat(sh, args):
    a = _parser("stat", "stat [-f <format>] <path>")
    a.add_argument("-f", default=None, dest="format")
    a.add_argument("path")
    ns = a.parse_args(args)
    st = sh.fs.get_status(ns.path)
    i = st.info
    if ns.format:
        rep = {"%N": i.name, "%z": str(i.length), "%u": i.owner, "%g": i.group,
               "%y": _fmt_time(i.lastModificationTimeMs), "%Y": str(i.lastModificationTimeMs),
               "%b": str(len(i.blockIds)), "%i": str(i.fileId), "%r": str(i.replicationMin),
               "%F": "directory" if i.folder else "regular file"}
        s = ns.format
        for k, v in rep.items():
            s = s.replace(k, v)
        sh.p(s)
        return 0
    kind = "directory" if i.folder else "file"
    sh.p(f"{ns.path} is a {kind} path.")
    sh.p(str(i).rstrip())
    if not i.folder:
        sh.p("Containing the following blocks: ")
        for fbi in i.fileBlockInfos:
            sh.p(str(fbi.blockInfo).replace("\n", " ").strip())
    return 0


@command("count", "count [-h] <dir>", "Displays the number of files and directories matching the specified prefix.")
def _count(sh, args):
    a = _parser("count", "count [-h] <dir>")
    a.add_argument("-h", action="store_true", dest="human")
    a.add_argument("path")
    ns = a.parse_args(args)
    st = sh.fs.get_status(ns.path)
    files = dirs = size = 0
    if st.is_folder:
        dirs = 1
        for s in sh.fs.list_status(ns.path, recursive=True):
            if s.is_folder:
                dirs += 1
            else:
                files += 1
                size += s.length
    else:
        files, size = 1, st.length
    fmt = "%-25s%-25s%-15s"
    sh.p(fmt % ("File Count", "Folder Count", "Folder Size"))
    sh.p(fmt % (files, dirs, bytes_to_human(size) if ns.human else size))
    return 0


@command("du", "du [-h|-s|--memory] <path>", "Displays the total size and the in Alluxio size of the specified file or directory.")
def _du(sh, args):
    a = _parser("du", "du [-h|-s|--memory] <path>")
    a.add_argument("-h", action="store_true", dest="human")
    a.add_argument("-s", action="store_true", dest="summarize")
    a.add_argument("--memory", action="store_true")
    a.add_argument("path")
    ns = a.parse_args(args)
    st = sh.fs.get_status(ns.path)
    files = [st] if not st.is_folder else [s for s in sh.fs.list_status(ns.path, recursive=True) if not s.is_folder]
    hs = bytes_to_human if ns.human else str

    def row(size, inal, inmem, path):
        pct = f"({int(inal * 100 / size) if size else 0}%)"
        cols = f"{hs(size):<12}{hs(inal) + pct:<20}"
        if ns.memory:
            cols += f"{hs(inmem) + '(' + str(int(inmem * 100 / size) if size else 0) + '%)':<20}"
        sh.p(cols + path)
    hdr = f"{'File Size':<12}{'In Alluxio':<20}" + (f"{'In Memory':<20}" if ns.memory else "") + "Path"
    sh.p(hdr)
    tot = [0, 0, 0]
    for s in files:
        inal = s.length * s.in_alluxio_percentage // 100
        inmem = s.length * s.in_memory_percentage // 100
        tot[0] += s.length
        tot[1] += inal
        tot[2] += inmem
        if not ns.summarize:
            row(s.length, inal, inmem, s.path)
    if ns.summarize:
        row(tot[0], tot[1], tot[2], ns.path)
    return 0


@command("checksum", "checksum <Alluxio path>", "Calculates the md5 checksum of a file in the Alluxio filesystem.")
def _checksum(sh, args):
    a = _parser("checksum", "checksum [--crc32c] <Alluxio path>")
    a.add_argument("--crc32c", action="store_true")
    a.add_argument("path")
    ns = a.parse_args(args)
    h = hashlib.md5()
    crc = 0
    from ..ops.native import lib
    with sh.fs.open_file(ns.path) as f:
        while True:
            b = f.read(8 << 20)
            if not b:
                break
            h.update(b)
            if ns.crc32c:
                crc = lib().crc32c(b, crc)
    sh.p(f"md5sum: {h.hexdigest()}")
    if ns.crc32c:
        sh.p(f"crc32c: {crc:08x}")
    return 0


@command("location", "location <path>", "Displays the list of hosts storing the specified file.")
def _location(sh, args):
    a = _parser("location", "location <path>")
    a.add_argument("path")
    ns = a.parse_args(args)
    st = sh.fs.get_status(ns.path)
    sh.p(f"{ns.path} with file id {st.info.fileId} is on nodes: ")
    for fbi in st.info.fileBlockInfos:
        hosts = sorted({f"{l.workerAddress.host}:{l.workerAddress.rpcPort}" for l in fbi.blockInfo.locations})
        for h in hosts:
            sh.p(h)
    return 0


@command("test", "test [-d|-f|-e|-s|-z] <path>", "Test a property of a path, returning 0 if the property is true, or 1 otherwise.")
def _test(sh, args):
    a = _parser("test", "test [-d|-f|-e|-s|-z] <path>")
    g = a.add_mutually_exclusive_group(required=True)
    for o in ("d", "f", "e", "s", "z"):
        g.add_argument(f"-{o}", action="store_true")
    a.add_argument("path")
    ns = a.parse_args(args)
    try:
        st = sh.fs.get_status(ns.path)
    except NotFoundException:
        return 1
    if ns.e:
        return 0
    if ns.d:
        return 0 if st.is_folder else 1
    if ns.f:
        return 0 if not st.is_folder else 1
    if ns.s:
        return 0 if (sh.fs.list_status(ns.path) if st.is_folder else st.length) else 1
    if ns.z:
        return 0 if (not st.is_folder and st.length == 0) else 1
    return 1


# ---- attributes ---------------------------------------------------------------------------------
def _recursive_flag(args):
    rec = "-R" in args
    return rec, [x for x in args if x != "-R"]


@command("chmod", "chmod [-R] <mode> <path>", "Changes the permission of a file or directory specified by args.")
def _chmod(sh, args):
    rec, rest = _recursive_flag(args)
    if len(rest) != 2:
        raise ValueError("chmod requires 2 arguments")
    mode_s, path = rest
    if mode_s.isdigit():
        mode = int(mode_s, 8)
    else:
        mode = _symbolic_mode(sh.fs.get_status(path).info.mode, mode_s)
    sh.fs.set_attribute(path, mode=mode, recursive=rec)
    sh.p(f"Changed permission of {path} to {oct(mode)[2:]}")
    return 0


def _symbolic_mode(cur: int, spec: str) -> int:
    """u+x, go-w, a=r style (reference ModeParser)."""
    mode = cur
    for clause in spec.split(","):
        who = ""
        i = 0
        while i < len(clause) and clause[i] in "ugoa":
            who += clause[i]
            i += 1
        who = who or "a"
        op = clause[i]
        perms = clause[i + 1:]
        bits = (4 if "r" in perms else 0) | (2 if "w" in perms else 0) | (1 if "x" in perms else 0)
        shifts = [s for c, s in (("u", 6), ("g", 3), ("o", 0)) if c in who or "a" in who]
        for s in shifts:
            if op == "+":
                mode |= bits << s
            elif op == "-":
                mode &= ~(bits << s)
            elif op == "=":
                mode = (mode & ~(7 << s)) | (bits << s)
    return mode


@command("chown", "chown [-R] <owner>[:<group>] <path>", "Changes the owner of a file or directory specified by args.")
def _chown(sh, args):
    rec, rest = _recursive_flag(args)
    if len(rest) != 2:
        raise ValueError("chown requires 2 arguments")
    who, path = rest
    owner, _, group = who.partition(":")
    sh.fs.set_attribute(path, owner=owner, group=group or None, recursive=rec)
    sh.p(f"Changed owner of {path} to {owner}" + (f" and group to {group}" if group else ""))
    return 0


@command("chgrp", "chgrp [-R] <group> <path>", "Changes the group of a file or directory specified by args.")
def _chgrp(sh, args):
    rec, rest = _recursive_flag(args)
    if len(rest) != 2:
        raise ValueError("chgrp requires 2 arguments")
    group, path = rest
    sh.fs.set_attribute(path, group=group, recursive=rec)
    sh.p(f"Changed group of {path} to {group}")
    return 0


@command("getfacl", "getfacl <path>", "Displays the access control lists (ACLs) of files and directories.")
def _getfacl(sh, args):
    if len(args) != 1:
        raise ValueError("getfacl requires 1 argument")
    from ..security.acl import AclEntry
    i = sh.fs.get_status(args[0]).info
    sh.p(f"# file: {i.path}")
    sh.p(f"# owner: {i.owner}")
    sh.p(f"# group: {i.group}")
    m = i.mode
    sh.p(f"user::{mode_to_string(m)[1:4]}")
    for e in i.acl.entries:
        ae = AclEntry.from_pacl_entry(e)
        if ae.subject:
            sh.p(ae.to_cli())
    sh.p(f"group::{mode_to_string(m)[4:7]}")
    sh.p(f"other::{mode_to_string(m)[7:10]}")
    for e in i.defaultAcl.entries:
        sh.p(AclEntry.from_pacl_entry(e).to_cli())
    return 0


@command("setfacl", "setfacl [-d] [-R] [--set | -m | -x <acl_entries> <path>] | [-b | -k <path>]", "Sets the access control list (ACL) for a path.")
def _setfacl(sh, args):
    a = _parser("setfacl", "setfacl ...")
    a.add_argument("-R", action="store_true", dest="recursive")
    a.add_argument("-d", action="store_true", dest="default")
    a.add_argument("--set", default=None)
    a.add_argument("-m", default=None)
    a.add_argument("-x", default=None)
    a.add_argument("-b", action="store_true")
    a.add_argument("-k", action="store_true")
    a.add_argument("path")
    ns = a.parse_args(args)
    pref = "default:" if ns.default else ""
    if ns.b:
        sh.fs.set_acl(ns.path, "REMOVE_ALL", [], ns.recursive)
    elif ns.k:
        sh.fs.set_acl(ns.path, "REMOVE_DEFAULT", [], ns.recursive)
    else:
        for action, spec in (("REPLACE", ns.set), ("MODIFY", ns.m), ("REMOVE", ns.x)):
            if spec:
                entries = [pref + e if pref and not e.startswith("default:") else e for e in spec.split(",")]
                sh.fs.set_acl(ns.path, action, entries, ns.recursive)
    return 0


@command("pin", "pin <path> media1 media2 media3 ...", "Marks a file or directory as pinned.")
def _pin(sh, args):
    if not args:
        raise ValueError("pin requires at least 1 argument")
    sh.fs.set_attribute(args[0], pinned=True, pinned_media=args[1:] or None)
    sh.p(f"File '{args[0]}' was successfully pinned.")
    return 0


@command("unpin", "unpin <path>", "Unpins the given file or folder from memory (works recursively for a directory).")
def _unpin(sh, args):
    if len(args) != 1:
        raise ValueError("unpin requires 1 argument")
    sh.fs.set_attribute(args[0], pinned=False)
    sh.p(f"File '{args[0]}' was successfully unpinned.")
    return 0


@command("setTtl", "setTtl [--action delete|free] <path> <time to live>", "Sets a new TTL value for the file at path.")
def _setttl(sh, args):
    a = _parser("setTtl", "setTtl [--action delete|free] <path> <ttl>")
    a.add_argument("--action", default="delete", choices=["delete", "free"])
    a.add_argument("path")
    a.add_argument("ttl")
    ns = a.parse_args(args)
    ttl = int(ns.ttl) if ns.ttl.isdigit() else parse_time_size(ns.ttl)
    sh.fs.set_attribute(ns.path, ttl=ttl, ttl_action=ns.action.upper())
    sh.p(f"TTL of path '{ns.path}' was successfully set to {ttl} milliseconds, with expiry action set to "
         f"{ns.action.upper()}")
    return 0


@command("unsetTtl", "unsetTtl <path>", "Unsets the TTL value for the given path.")
def _unsetttl(sh, args):
    if len(args) != 1:
        raise ValueError("unsetTtl requires 1 argument")
    sh.fs.set_attribute(args[0], ttl=-1, ttl_action="DELETE")
    sh.p(f"TTL of path '{args[0]}' was successfully removed.")
    return 0


@command("setReplication", "setReplication [-R] [--max <num> | --min <num>] <path>", "Sets the minimal and maximal replication level of a file or directory.")
def _setrep(sh, args):
    a = _parser("setReplication", "setReplication [-R] [--max n] [--min n] <path>")
    a.add_argument("-R", action="store_true", dest="recursive")
    a.add_argument("--max", type=int, default=None)
    a.add_argument("--min", type=int, default=None)
    a.add_argument("path")
    ns = a.parse_args(args)
    if ns.max is None and ns.min is None:
        raise ValueError("at least one option of '--max' or '--min' must be specified")
    if ns.max is not None and ns.min is not None and ns.max != -1 and ns.max < ns.min:
        raise ValueError("max replication must be >= min replication")
    sh.fs.set_attribute(ns.path, replication_min=ns.min, replication_max=ns.max, recursive=ns.recursive)
    msg = f"Changed the replication level of {ns.path}"
    if ns.min is not None:
        msg += f"\nreplicationMin was set to {ns.min}"
    if ns.max is not None:
        msg += f"\nreplicationMax was set to {ns.max}"
    sh.p(msg)
    return 0


# ---- cache management ---------------------------------------------------------------------------
@command("free", "free [-f] <path>", "Frees the space occupied by a file or a directory in Alluxio.")
def _free(sh, args):
    a = _parser("free", "free [-f] <path>")
    a.add_argument("-f", action="store_true", dest="forced")
    a.add_argument("path")
    ns = a.parse_args(args)
    for path in _expand(sh.fs, ns.path):
        sh.fs.free(path, recursive=True, forced=ns.forced)
        sh.p(f"{path} was successfully freed from Alluxio space.")
    return 0


@command("load", "load [--local] <path>", "Loads a file or directory in Alluxio space, makes it resident in Alluxio.")
def _load(sh, args):
    a = _parser("load", "load [--local] <path>")
    a.add_argument("--local", action="store_true")
    a.add_argument("path")
    ns = a.parse_args(args)
    st = sh.fs.get_status(ns.path)
    files = [st] if not st.is_folder else [s for s in sh.fs.list_status(ns.path, recursive=True) if not s.is_folder]
    for s in files:
        if s.in_alluxio_percentage == 100 and not ns.local:
            sh.p(f"{s.path} already in Alluxio fully")
            continue
        with sh.fs.open_file(s.path, read_type="CACHE_PROMOTE", status=s) as f:
            while f.read(8 << 20):
                pass
        sh.p(f"{s.path} loaded")
    return 0


@command("persist", "persist [--wait <time>] <path> [<path> ...]", "Persists files or directories currently stored only in Alluxio to the UnderFileSystem.")
def _persist(sh, args):
    a = _parser("persist", "persist [--wait <time>] <path> ...")
    a.add_argument("--wait", default="0")
    a.add_argument("--timeout", default="20min")
    a.add_argument("paths", nargs="+")
    ns = a.parse_args(args)
    todo = []
    for p in ns.paths:
        st = sh.fs.get_status(p)
        files = [st] if not st.is_folder else [s for s in sh.fs.list_status(p, recursive=True) if not s.is_folder]
        for s in files:
            if s.is_persisted:
                sh.p(f"{s.path} is already persisted")
                continue
            sh.fs.persist(s.path, parse_time_size(ns.wait) if not ns.wait.isdigit() else int(ns.wait))
            todo.append(s.path)
    deadline = time.time() + parse_time_size(ns.timeout) / 1000.0
    for p in todo:
        while not sh.fs.get_status(p, sync_interval_ms=-1).is_persisted:
            if time.time() > deadline:
                raise IOError(f"timed out waiting for {p} to be persisted")
            time.sleep(0.05)
        sh.p(f"persisted file {p} with size {sh.fs.get_status(p).length}")
    return 0


@command("loadMetadata", "loadMetadata [-R] [-F] <path>", "Loads metadata for the given Alluxio path from the under file system.")
def _loadmeta(sh, args):
    a = _parser("loadMetadata", "loadMetadata [-R] [-F] <path>")
    a.add_argument("-R", action="store_true", dest="recursive")
    a.add_argument("-F", action="store_true", dest="force")
    a.add_argument("path")
    ns = a.parse_args(args)
    if ns.force:
        sh.fs.list_status(ns.path, recursive=ns.recursive, sync_interval_ms=0)
    else:
        sh.fs.load_metadata(ns.path, recursive=ns.recursive)
    return 0


@command("checkConsistency", "checkConsistency [-r] [-t <thread count>] <Alluxio path>", "Checks the consistency of a persisted file or directory in Alluxio.")
def _checkcons(sh, args):
    a = _parser("checkConsistency", "checkConsistency [-r] <path>")
    a.add_argument("-r", action="store_true", dest="repair")
    a.add_argument("-t", type=int, default=1)
    a.add_argument("path")
    ns = a.parse_args(args)
    bad = sh.fs.check_consistency(ns.path)
    if not bad:
        sh.p(f"{ns.path} is consistent with the under storage system.")
        return 0
    if not ns.repair:
        sh.p(f"The following files are inconsistent:")
        for p in bad:
            sh.p(p)
        return 0
    sh.p(f"{ns.path} has: {len(bad)} inconsistent files. Repairing with {ns.t} threads.")
    for p in bad:
        try:
            sh.fs.delete(p, alluxio_only=True, recursive=True)
        except NotFoundException:
            pass
        sh.fs.exists(p, load_metadata="ALWAYS")
        sh.p(f"repaired {p}")
    return 0


# ---- mounts / sync ------------------------------------------------------------------------------
@command("mount", "mount [--readonly] [--shared] [--option <key=val>] <alluxioPath> <ufsURI>", "Mounts a UFS path onto an Alluxio path.")
def _mount(sh, args):
    a = _parser("mount", "mount [--readonly] [--shared] [--option k=v] <alluxioPath> <ufsURI>")
    a.add_argument("--readonly", action="store_true")
    a.add_argument("--shared", action="store_true")
    a.add_argument("--option", action="append", default=[])
    a.add_argument("alluxio", nargs="?")
    a.add_argument("ufs", nargs="?")
    ns = a.parse_args(args)
    if ns.alluxio is None:
        for mp, info in sorted(sh.fs.get_mount_table().items()):
            flags = ("readonly, " if info.readOnly else "") + ("shared" if info.shared else "not shared")
            sh.p(f"{info.ufsUri:<40}on  {mp:<20}({info.ufsType}, capacity={info.ufsCapacityBytes}, "
                 f"used={info.ufsUsedBytes}, {flags}, properties={dict(info.properties)})")
        return 0
    props = dict(o.split("=", 1) for o in ns.option)
    sh.fs.mount(ns.alluxio, ns.ufs, read_only=ns.readonly, shared=ns.shared, properties=props)
    sh.p(f"Mounted {ns.ufs} at {ns.alluxio}")
    return 0


@command("unmount", "unmount <alluxioPath>", "Unmounts an Alluxio path.")
def _unmount(sh, args):
    if len(args) != 1:
        raise ValueError("unmount requires 1 argument")
    sh.fs.unmount(args[0])
    sh.p(f"Unmounted {args[0]}")
    return 0


@command("updateMount", "updateMount [--readonly] [--shared] [--option <key=val>] <alluxioPath>", "Updates options for a mount point while keeping the Alluxio metadata under the path.")
def _updatemount(sh, args):
    a = _parser("updateMount", "updateMount [--readonly] [--shared] [--option k=v] <alluxioPath>")
    a.add_argument("--readonly", action="store_true")
    a.add_argument("--shared", action="store_true")
    a.add_argument("--option", action="append", default=[])
    a.add_argument("alluxio")
    ns = a.parse_args(args)
    sh.fs.update_mount(ns.alluxio, read_only=ns.readonly, shared=ns.shared,
                       properties=dict(o.split("=", 1) for o in ns.option))
    sh.p(f"Updated mount point options at {ns.alluxio}")
    return 0


@command("startSync", "startSync <path>", "Starts the automatic syncing process of the specified path.")
def _startsync(sh, args):
    if len(args) != 1:
        raise ValueError("startSync requires 1 argument")
    sh.p("Starting a full sync of '" + args[0] + "'. You can check the status of the sync using getSyncPathList cmd")
    sh.fs.start_sync(args[0])
    sh.p(f"Started automatic syncing of '{args[0]}'.")
    return 0


@command("stopSync", "stopSync <path>", "Stops the automatic syncing process of the specified path.")
def _stopsync(sh, args):
    if len(args) != 1:
        raise ValueError("stopSync requires 1 argument")
    sh.fs.stop_sync(args[0])
    sh.p(f"Stopped automatic syncing of '{args[0]}'.")
    return 0


@command("getSyncPathList", "getSyncPathList", "Gets all the paths that are under active syncing right now.")
def _getsync(sh, args):
    sh.p("The following paths are under active sync")
    for p in sh.fs.get_sync_path_list():
        sh.p(p)
    return 0


# ---- cluster info -------------------------------------------------------------------------------
@command("getCapacityBytes", "getCapacityBytes", "Gets the capacity of the Alluxio file system.")
def _cap(sh, args):
    sh.p(f"Capacity Bytes: {sh.fs.capacity()[0]}")
    return 0


@command("getUsedBytes", "getUsedBytes", "Gets number of bytes used in the Alluxio file system.")
def _used(sh, args):
    sh.p(f"Used Bytes: {sh.fs.capacity()[1]}")
    return 0


def _master_info(sh):
    return sh.fs.ctx.meta_master().GetMasterInfo(pb.meta.GetMasterInfoPOptions()).masterInfo


@command("leader", "leader", "Prints the hostname of the primary master.")
def _leader(sh, args):
    sh.p(_master_info(sh).leaderMasterAddress)
    return 0


@command("masterInfo", "masterInfo", "Prints information regarding master fault tolerance such as leader address, list of master addresses, and the configured Zookeeper address.")
def _masterinfo(sh, args):
    mi = _master_info(sh)
    sh.p(f"Current leader master: {mi.leaderMasterAddress}")
    sh.p("All masters: " + str([f"{a.host}:{a.rpcPort}" for a in mi.masterAddresses] or [mi.leaderMasterAddress]))
    return 0


# ---- distributed (job service) ------------------------------------------------------------------
def _run_job(sh, cfg, async_: bool = False) -> int:
    jc = sh.job_client()
    if async_:
        jid = jc.run(cfg)
        sh.p(f"Submitted job {jid}")
        return 0
    status, result, err = jc.run_and_wait(cfg)
    if status != "COMPLETED":
        sh.p(f"Job {status}: {err}")
        return -1
    sh.p(f"Job completed: {result}")
    return 0


@command("distributedLoad", "distributedLoad [--replication <N>] [--active-jobs <N>] [--host-file <file>] [--hosts <hosts>] [--excluded-hosts <hosts>] <path>", "Loads a file or all files in a directory into Alluxio space.")
def _dload(sh, args):
    a = _parser("distributedLoad", "distributedLoad [--replication N] <path>")
    a.add_argument("--replication", type=int, default=1)
    a.add_argument("--active-jobs", type=int, default=3000)
    a.add_argument("--hosts", default="")
    a.add_argument("--excluded-hosts", default="")
    a.add_argument("--async", action="store_true", dest="async_")
    a.add_argument("path")
    ns = a.parse_args(args)
    from ..job import LoadConfig
    cfg = LoadConfig(path=ns.path, replication=ns.replication,
                     worker_set=[h for h in ns.hosts.split(",") if h],
                     excluded_worker_set=[h for h in ns.excluded_hosts.split(",") if h])
    sh.p(f"Allow up to {ns.active_jobs} active jobs")
    return _run_job(sh, cfg, ns.async_)


def _migrate(sh, args, name, delete_source):
    a = _parser(name, f"{name} <src> <dst>")
    a.add_argument("--active-jobs", type=int, default=3000)
    a.add_argument("--overwrite", action="store_true")
    a.add_argument("--async", action="store_true", dest="async_")
    a.add_argument("src")
    a.add_argument("dst")
    ns = a.parse_args(args)
    from ..job import MigrateConfig
    wt = sh.fs.ctx.conf.get("alluxio.user.file.writetype.default")
    return _run_job(sh, MigrateConfig(source=ns.src, destination=ns.dst, write_type=wt, overwrite=ns.overwrite,
                                      delete_source=delete_source), ns.async_)


@command("distributedCp", "distributedCp [--active-jobs <N>] <src> <dst>", "Copies a file or directory in parallel at file level.")
def _dcp(sh, args):
    return _migrate(sh, args, "distributedCp", False)


@command("distributedMv", "distributedMv <src> <dst>", "Moves a file or directory in parallel at file level.")
def _dmv(sh, args):
    rc = _migrate(sh, args, "distributedMv", True)
    if rc == 0:
        src = [x for x in args if not x.startswith("-")][0]
        try:
            if sh.fs.get_status(src).is_folder:
                sh.fs.delete(src, recursive=True)
        except NotFoundException:
            pass
    return rc


@command("help", "help <command>", "Prints help message for the given command. If command is not given, prints help messages for all supported commands.")
def _help(sh, args):
    names = args or sorted(COMMANDS)
    for n in names:
        ent = COMMANDS.get(n)
        if ent is None:
            sh.p(f"{n} is an unknown command.")
            return -1
        sh.p(f"{ent[1]}\n\t{ent[2]}")
    return 0


def main(argv=None, out=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    sh = FileSystemShell(out=out)
    try:
        return sh.run(argv)
    finally:
        sh.fs.close()


__all__ = ["FileSystemShell", "COMMANDS", "main", "enum_name"]
