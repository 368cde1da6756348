"""``alluxio validateEnv`` / ``validateConf``.

Parity: integration/tools/validation/src/main/java/alluxio/cli/ValidateEnv.java (named tasks
grouped by target master/worker/cluster, each returning OK / WARNING / FAILED / SKIPPED) and
shell/src/main/java/alluxio/cli/ValidateConf.java (every key set in the site properties must
be a known key).  The MI355X build swaps the ramdisk/ssh checks for the ones that matter here:
HIP device visibility, HBM tier quota vs device memory, the native extension, the RCCL
library and xGMI topology, pinned host memory, and the UFS root.
"""
from __future__ import annotations

import os
import shutil
import socket
import sys

OK, WARNING, FAILED, SKIPPED = "OK", "WARNING", "FAILED", "SKIPPED"
TASKS: dict[str, tuple] = {}


def task(name, targets, desc):
    def deco(fn):
        TASKS[name] = (fn, targets, desc)
        return fn
    return deco


@task("master.rpc.port.available", ("master",), "validate master RPC port is available")
def _master_port(conf):
    return _port_free(conf.get_int("alluxio.master.rpc.port"))


@task("worker.rpc.port.available", ("worker",), "validate worker RPC port is available")
def _worker_port(conf):
    return _port_free(conf.get_int("alluxio.worker.rpc.port"))


def _port_free(port):
    s = socket.socket()
    try:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind(("0.0.0.0", port))
        return OK, f"port {port} is available"
    except OSError as e:
        return FAILED, f"port {port} is not available: {e}"
    finally:
        s.close()


@task("native.extension", ("master", "worker"), "the HIP/C++ extension builds and loads")
def _native(conf):
    try:
        from ..ops.native import lib
        C = lib()
        return OK, f"loaded {C.__file__}"
    except Exception as e:  # noqa: BLE001
        return FAILED, f"native extension unavailable: {e}"


@task("worker.gpu.visible", ("worker",), "validate HIP devices are visible to the worker")
def _gpu(conf):
    try:
        import torch
        n = torch.cuda.device_count()
    except Exception as e:  # noqa: BLE001
        return FAILED, f"torch/HIP unavailable: {e}"
    if n == 0:
        return WARNING, "no HIP device visible; HBM tiers fall back to host DRAM"
    return OK, f"{n} HIP device(s) visible"


@task("worker.hbm.quota", ("worker",), "validate the HBM tier quota fits device memory")
def _hbm_quota(conf):
    from ..conf.keys import Templates
    from ..utils.format import parse_space_size
    try:
        import torch
        if torch.cuda.device_count() == 0:
            return SKIPPED, "no HIP device"
        total = torch.cuda.get_device_properties(0).total_memory
    except Exception as e:  # noqa: BLE001
        return SKIPPED, str(e)
    levels = conf.get_int("alluxio.worker.tieredstore.levels")
    want = 0
    for lvl in range(levels):
        paths = conf.get_list(Templates.WORKER_TIERED_STORE_LEVEL_DIRS_PATH.format(lvl))
        quotas = conf.get_list(Templates.WORKER_TIERED_STORE_LEVEL_DIRS_QUOTA.format(lvl))
        for i, p in enumerate(paths):
            if p.startswith("hbm"):
                want += parse_space_size(quotas[min(i, len(quotas) - 1)])
    if want > 0.95 * total:
        return FAILED, f"HBM quota {want} exceeds 95% of device memory {total}"
    return OK, f"HBM quota {want} of {total} bytes"


@task("worker.pinned.memory", ("worker",), "validate pinned host memory can be allocated")
def _pinned(conf):
    try:
        import torch
        if torch.cuda.device_count() == 0:
            return SKIPPED, "no HIP device"
        torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
        return OK, "pinned 64MB"
    except Exception as e:  # noqa: BLE001
        return FAILED, f"cannot pin host memory: {e}"


@task("cluster.rccl.library", ("cluster",), "validate RCCL is available for the xGMI data plane")
def _rccl(conf):
    try:
        import torch.distributed as dist
        if not dist.is_nccl_available():
            return WARNING, "torch.distributed has no RCCL backend; peer transfers use gRPC"
        return OK, "RCCL backend available"
    except Exception as e:  # noqa: BLE001
        return WARNING, str(e)


@task("cluster.xgmi.topology", ("cluster",), "report xGMI links between visible GPUs")
def _xgmi(conf):
    smi = shutil.which("rocm-smi")
    if smi is None:
        return SKIPPED, "rocm-smi not on PATH"
    import subprocess
    try:
        r = subprocess.run([smi, "--showtopotype"], capture_output=True, text=True, timeout=30)
    except Exception as e:  # noqa: BLE001
        return SKIPPED, str(e)
    return (OK if "XGMI" in r.stdout else WARNING), ("xGMI links present" if "XGMI" in r.stdout
                                                     else "no xGMI links reported")


@task("ufs.root.accessible", ("master",), "validate the root UFS is accessible")
def _ufs(conf):
    root = conf.get("alluxio.master.mount.table.root.ufs")
    try:
        from ..underfs import registry
        ufs = registry.create(root, conf)
        if not ufs.exists(root):
            return WARNING, f"root UFS {root} does not exist yet"
        ufs.list_status(root)
        return OK, f"root UFS {root} is listable"
    except Exception as e:  # noqa: BLE001
        return FAILED, f"root UFS {root}: {e}"


def _hadoop_xml(path: str) -> dict[str, str]:
    """``<configuration><property><name/><value/></property>...`` (HadoopConfigurationFileParser)."""
    import xml.etree.ElementTree as ET
    out = {}
    for prop in ET.parse(path).getroot().iter("property"):
        name, value = prop.findtext("name"), prop.findtext("value")
        if name:
            out[name.strip()] = (value or "").strip()
    return out


def _hdfs_root(conf):
    root = conf.get("alluxio.master.mount.table.root.ufs")
    return root if root.startswith("hdfs://") else None


@task("ufs.hdfs.config.parity", ("master", "worker"),
      "validate the HDFS core-site/hdfs-site files parse and agree with HADOOP_CONF_DIR")
def _hdfs_conf(conf):
    """HdfsConfValidationTask + HdfsConfParityValidationTask: the files named by
    ``alluxio.underfs.hdfs.configuration`` (``:``-separated) must be valid Hadoop XML, and keys set
    in both them and ``$HADOOP_CONF_DIR`` must not disagree."""
    if _hdfs_root(conf) is None:
        return SKIPPED, "root UFS is not HDFS"
    files = [f for f in (conf.get("alluxio.underfs.hdfs.configuration") or "").split(":") if f and os.path.exists(f)]
    if not files:
        return WARNING, "no file of alluxio.underfs.hdfs.configuration exists (client defaults are used)"
    merged: dict[str, str] = {}
    for f in files:
        try:
            merged.update(_hadoop_xml(f))
        except Exception as e:  # noqa: BLE001
            return FAILED, f"cannot parse {f}: {e}"
    hd = os.environ.get("HADOOP_CONF_DIR")
    if hd:
        diffs = []
        for name in ("core-site.xml", "hdfs-site.xml"):
            fp = os.path.join(hd, name)
            if os.path.exists(fp):
                for k, v in _hadoop_xml(fp).items():
                    if k in merged and merged[k] != v:
                        diffs.append(f"{k}: {merged[k]!r} vs {v!r} in {fp}")
        if diffs:
            return WARNING, "HDFS configuration differs from HADOOP_CONF_DIR: " + "; ".join(diffs[:5])
    return OK, f"{len(merged)} HDFS properties from {len(files)} file(s)"


@task("ufs.hdfs.reachable", ("master", "worker"),
      "validate the HDFS NameNode answers ClientProtocol calls (HdfsVersionValidationTask)")
def _hdfs_reachable(conf):
    root = _hdfs_root(conf)
    if root is None:
        return SKIPPED, "root UFS is not HDFS"
    try:
        from ..underfs import registry
        ufs = registry.create(root, conf)
        d = ufs.nn.get_server_defaults()
        st = ufs.nn.get_fs_stats()
        ufs.close()
    except Exception as e:  # noqa: BLE001
        return FAILED, f"NameNode of {root}: {e}"
    return OK, (f"NameNode of {root} reachable over Hadoop IPC v9: block size {d.blockSize}, "
                f"checksum type {d.checksumType}, {st.remaining} of {st.capacity} bytes free")


@task("ufs.superuser", ("master",), "validate the Alluxio user owns (or may administer) the root UFS")
def _ufs_superuser(conf):
    """UfsSuperUserValidationTask: without owning the UFS root, setOwner/chmod of persisted files
    (and permission sync) fails."""
    import getpass
    root = conf.get("alluxio.master.mount.table.root.ufs")
    try:
        from ..underfs import registry
        ufs = registry.create(root, conf)
        st = ufs.get_status(root)
    except Exception as e:  # noqa: BLE001
        return SKIPPED, f"cannot stat root UFS {root}: {e}"
    if st is None:
        return SKIPPED, f"root UFS {root} does not exist"
    me = getpass.getuser()
    if not st.owner or st.owner == me or me == "root":
        return OK, f"{me} owns or administers {root}"
    return WARNING, f"{root} is owned by {st.owner}, not {me}: UFS owner/mode updates may be refused"


@task("worker.storage.space", ("worker",), "validate each disk tier directory has room for its quota")
def _storage_space(conf):
    """StorageSpaceValidationTask: the sum of a tier's quotas on one filesystem must fit its free space
    (device tiers are checked by worker.hbm.quota, DRAM tiers by the memory of the host)."""
    from ..utils.format import parse_space_size
    problems, checked = [], 0
    for lvl in range(conf.get_int("alluxio.worker.tieredstore.levels")):
        paths = (conf.get_raw(f"alluxio.worker.tieredstore.level{lvl}.dirs.path") or "").split(",")
        quotas = (conf.get_raw(f"alluxio.worker.tieredstore.level{lvl}.dirs.quota") or "").split(",")
        for i, path in enumerate(p.strip() for p in paths):
            if not path or path.startswith(("hbm", "dram")) or path == "mem":
                continue
            q = parse_space_size(quotas[min(i, len(quotas) - 1)].strip()) if quotas[0].strip() else 0
            probe = path
            while probe and not os.path.exists(probe):
                probe = os.path.dirname(probe.rstrip("/"))
            if not probe:
                continue
            free = shutil.disk_usage(probe).free
            checked += 1
            if q > free:
                problems.append(f"{path}: quota {q} > free {free}")
    if problems:
        return WARNING, "; ".join(problems)
    return (OK, f"{checked} disk tier dir(s) fit their quotas") if checked else (SKIPPED, "no disk tier dirs")


@task("journal.folder.writable", ("master",), "validate the journal folder is writable")
def _journal(conf):
    folder = conf.get("alluxio.master.journal.folder")
    if folder.startswith("file://"):
        folder = folder[7:]
    probe = folder
    while probe and not os.path.exists(probe):  # nearest existing ancestor; never creates dirs
        probe = os.path.dirname(probe.rstrip("/"))
    if probe and os.access(probe, os.W_OK):
        return OK, f"{folder} is writable" + ("" if probe == folder else f" (creatable under {probe})")
    return FAILED, f"{folder} is not writable"


@task("ulimit.open.files", ("master", "worker"), "validate the open-file limit")
def _ulimit(conf):
    import resource
    soft, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
    return (OK if soft >= 4096 else WARNING), f"open files soft limit {soft}"


def validate_env(target="all", conf=None, out=None, only=None) -> dict:
    from ..conf import Configuration
    conf = conf or Configuration(load_site=True)
    out = out or sys.stdout
    results = {}
    for name, (fn, targets, desc) in TASKS.items():
        if only and name not in only:
            continue
        if target != "all" and target not in targets:
            continue
        try:
            res, msg = fn(conf)
        except Exception as e:  # noqa: BLE001
            res, msg = FAILED, str(e)
        results[name] = res
        print(f"Validating {name}... {res}: {msg}", file=out)
    return results


def validate_conf(conf=None, out=None) -> list[str]:
    from ..conf import Configuration
    from ..conf.keys import is_valid
    conf = conf or Configuration(load_site=True)
    bad = [k for k in conf.to_map() if k.startswith("alluxio.") and not is_valid(k)]
    out = out or sys.stdout
    for k in bad:
        print(f"Unrecognized property key: {k}", file=out)
    print("All configuration properties are valid." if not bad else f"{len(bad)} invalid properties.", file=out)
    return bad


def main_env(argv=None, out=None) -> int:
    argv = list(argv or [])
    target = argv[0] if argv and not argv[0].startswith("-") else "all"
    if target == "list":
        for name, (_, targets, desc) in TASKS.items():
            print(f"{name}: {desc} ({', '.join(targets)})", file=out or sys.stdout)
        return 0
    res = validate_env(target, out=out)
    return 1 if FAILED in res.values() else 0


def main_conf(argv=None, out=None) -> int:
    return 1 if validate_conf(out=out) else 0
