"""Job plans: configs + PlanDefinition SPI (selectExecutors / runTask / join).

Parity: job/server/src/main/java/alluxio/job/plan/PlanDefinition.java and the plans under
job/server/src/main/java/alluxio/job/plan/: load/LoadDefinition.java (:60-150 — distribute the
non-cached blocks of a path over workers, each task reads its blocks through the local worker
with CACHE), persist/PersistDefinition.java, replicate/{Replicate,Evict,Move}Definition.java,
migrate/MigrateDefinition.java (distributed cp/mv), stress/StressBenchDefinition.java (:60-130 —
run a stress bench on N job workers, merge results).  Job configs travel as JSON in the
``jobConfig`` bytes of RunPRequest / RunTaskCommand.
"""
from __future__ import annotations

import dataclasses
import json
import logging
import random

from ..proto import pb
from ..utils import exceptions as ex

LOG = logging.getLogger(__name__)

_REGISTRY: dict[str, type] = {}


def plan(name):
    def deco(cls):
        cls.type_name = name
        _REGISTRY[name] = cls
        return cls
    return deco


@dataclasses.dataclass
class JobConfig:
    type_name = "base"

    def to_bytes(self) -> bytes:
        d = dataclasses.asdict(self)
        d["@type"] = self.type_name
        return json.dumps(d).encode()

    @staticmethod
    def from_bytes(b: bytes) -> "JobConfig":
        d = json.loads(b.decode())
        t = d.pop("@type")
        cls = CONFIGS[t]
        if cls is CompositeConfig:
            d["jobs"] = [JobConfig.from_bytes(json.dumps(j).encode()) if isinstance(j, dict) else j
                         for j in d["jobs"]]
        return cls(**d)

    def definition(self) -> "PlanDefinition":
        return _REGISTRY[self.type_name]()


CONFIGS: dict[str, type] = {}


def config(name):
    def deco(cls):
        cls.type_name = name
        CONFIGS[name] = cls
        return cls
    return deco


@config("load")
@dataclasses.dataclass
class LoadConfig(JobConfig):
    path: str = "/"
    replication: int = 1
    worker_set: list = dataclasses.field(default_factory=list)
    excluded_worker_set: list = dataclasses.field(default_factory=list)
    local_only: bool = False


@config("persist")
@dataclasses.dataclass
class PersistConfig(JobConfig):
    path: str = "/"
    mount_id: int = 0
    overwrite: bool = True
    ufs_path: str = ""


@config("replicate")
@dataclasses.dataclass
class ReplicateConfig(JobConfig):
    block_id: int = 0
    replicas: int = 1
    path: str = ""
    medium: str = ""


@config("evict")
@dataclasses.dataclass
class EvictConfig(JobConfig):
    block_id: int = 0
    replicas: int = 1


@config("move")
@dataclasses.dataclass
class MoveConfig(JobConfig):
    block_id: int = 0
    worker_host: str = ""
    medium: str = ""


@config("migrate")
@dataclasses.dataclass
class MigrateConfig(JobConfig):
    source: str = "/"
    destination: str = "/"
    write_type: str = "ASYNC_THROUGH"
    overwrite: bool = False
    delete_source: bool = False


@config("transform")
@dataclasses.dataclass
class TransformConfig(JobConfig):
    db: str = ""
    table: str = ""
    transform: str = ""      # the transformation definition, e.g. "file.count.max=100"
    partitions: list = dataclasses.field(default_factory=list)   # [{spec, files, format, dst}]


@config("stress")
@dataclasses.dataclass
class StressBenchConfig(JobConfig):
    bench: str = "worker"          # worker | client-io | master | ufs-io
    args: list = dataclasses.field(default_factory=list)
    cluster_limit: int = 0


@config("composite")
@dataclasses.dataclass
class CompositeConfig(JobConfig):
    jobs: list = dataclasses.field(default_factory=list)
    sequential: bool = True

    def to_bytes(self) -> bytes:
        return json.dumps({"@type": "composite", "sequential": self.sequential,
                           "jobs": [json.loads(j.to_bytes()) for j in self.jobs]}).encode()


class RunTaskContext:
    """What a task sees on the job worker: a client FileSystem and the co-located block worker."""

    def __init__(self, fs, worker=None, worker_address=None, job_id=0, task_id=0):
        self.fs = fs
        self.worker = worker
        self.worker_address = worker_address
        self.job_id = job_id
        self.task_id = task_id


class PlanDefinition:
    def select_executors(self, cfg, job_workers: list, fs) -> list[tuple[object, object]]:
        """[(job worker info, task args)] — one task per entry."""
        raise NotImplementedError

    def run_task(self, cfg, args, ctx: RunTaskContext):
        raise NotImplementedError

    def join(self, cfg, task_results: dict):
        return {"tasks": len(task_results)}


def _worker_key(addr) -> str:
    return f"{addr.host}:{addr.rpcPort}"


def _find_job_worker(job_workers, block_worker_addr):
    for jw in job_workers:
        if jw.address.host == block_worker_addr.host and jw.block_worker_port == block_worker_addr.rpcPort:
            return jw
    return None


# ----------------------------------------------------------------------------------------------
@plan("load")
class LoadDefinition(PlanDefinition):
    def select_executors(self, cfg, job_workers, fs):
        statuses = [s for s in fs.list_status(cfg.path, recursive=True) if not s.info.folder] \
            if fs.get_status(cfg.path).info.folder else [fs.get_status(cfg.path)]
        usable = [jw for jw in job_workers
                  if (not cfg.worker_set or jw.address.host in cfg.worker_set)
                  and jw.address.host not in cfg.excluded_worker_set]
        if not usable:
            raise ex.FailedPreconditionException("no job worker available for load")
        if len(usable) > 1 and (cfg.replication < 0 or cfg.replication >= len(usable)):
            return self._collective_plan(statuses, usable)
        if len(usable) > 2 and cfg.replication > 1:
            return self._collective_plan(statuses, usable, copies=cfg.replication)
        assign: dict[int, list] = {}
        for st in statuses:
            for fbi in st.info.fileBlockInfos:
                have = {(l.workerAddress.host, l.workerAddress.rpcPort) for l in fbi.blockInfo.locations}
                need = cfg.replication - len(have)
                if need <= 0:
                    continue
                cands = [jw for jw in usable if (jw.address.host, jw.block_worker_port) not in have]
                random.shuffle(cands)
                for jw in cands[:need]:
                    assign.setdefault(jw.id, []).append((st.info.path, fbi.blockInfo.blockId))
        by_id = {jw.id: jw for jw in usable}
        return [(by_id[w], blocks) for w, blocks in assign.items()]

    @staticmethod
    def _collective_plan(statuses, usable, copies: int | None = None):
        """``distributedLoad --replication`` >= the worker count (every worker gets every block):
        each block gets one owner -- a worker already caching it, else a worker that loads it from
        the UFS (round-robin) -- and then all workers exchange the blocks with RCCL all-gathers
        over the node's transfer plane (TransferPlane.replicate_all: every xGMI link busy at
        once) instead of N-1 point-to-point copies per block.  Every worker receives the same
        block list, in the same order: the collective's call sequence is identical on all ranks.

        With ``copies`` < the worker count, blocks already on ``copies`` workers are left out and
        the rest go around the ring of participants with RCCL send/recv
        (TransferPlane.replicate_ring): the owner and its ``copies - 1`` successors hold each block."""
        keys = {jw.id: f"{jw.address.host}:{jw.block_worker_port}" for jw in usable}
        usable_keys = set(keys.values())
        blocks, loads, rr, complete = [], {jw.id: [] for jw in usable}, 0, True
        for st in statuses:
            for fbi in st.info.fileBlockInfos:
                bi = fbi.blockInfo
                holders = [f"{l.workerAddress.host}:{l.workerAddress.rpcPort}" for l in bi.locations]
                held = [h for h in holders if h in usable_keys]
                if copies is not None and len(held) >= copies:
                    continue
                complete &= copies is None and set(held) >= usable_keys
                if held:
                    owner = held[0]
                else:
                    jw = usable[rr % len(usable)]
                    rr += 1
                    owner = keys[jw.id]
                    loads[jw.id].append((st.info.path, bi.blockId))
                blocks.append((st.info.path, bi.blockId, bi.length, owner, bool(held)))
        if complete:
            return []
        participants = sorted(usable_keys)
        if not blocks:
            return []
        return [(jw, {"collective": True, "participants": participants, "blocks": blocks, "load": loads[jw.id],
                      "copies": copies}) for jw in usable]

    def _run_collective(self, args, ctx) -> int:
        w = ctx.worker
        if w is None:
            return 0
        loaded = self._load_blocks([tuple(x) for x in args["load"]], ctx) if args["load"] else 0
        plane = getattr(w, "transfer_plane", None)
        if plane is not None and sorted(plane.addr_to_rank) == list(args["participants"]):
            # the decision depends only on the plane membership every participant shares, so
            # either all participants enter the collective or none does
            todo = [(bid, n, plane.addr_to_rank[owner]) for _, bid, n, owner, _ in args["blocks"]]
            if args.get("copies"):
                return loaded + plane.replicate_ring(todo, args["copies"])
            return loaded + plane.replicate_all(todo)
        # no common transfer plane: pull what was cached somewhere, load the rest from the UFS
        from ..worker.remote import remote_block_fetcher
        rest = []
        parts, copies = list(args["participants"]), args.get("copies")
        from ..parallel.transfer import _addr_key
        me = parts.index(_addr_key(w.address)) if _addr_key(w.address) in parts else None
        for path, bid, n, owner, held in args["blocks"]:
            if w.has_block(bid):
                continue
            if copies and me is not None and (me - parts.index(owner)) % len(parts) >= copies:
                continue                      # not one of this block's ring positions
            if held:
                host, port = owner.rsplit(":", 1)
                remote_block_fetcher(w, host, int(port), n)(bid)
                loaded += n
            else:
                rest.append((path, bid))
        return loaded + (self._load_blocks(rest, ctx) if rest else 0)

    def run_task(self, cfg, args, ctx):
        if isinstance(args, dict) and args.get("collective"):
            return self._run_collective(args, ctx)
        return self._load_blocks(args, ctx)

    def _load_blocks(self, args, ctx):
        loaded = 0
        from_ufs = []       # UFS blocks go to the worker in one bulk ingest call
        statuses = {}
        for path, block_id in args:
            st = statuses.get(path)
            if st is None:
                st = statuses[path] = ctx.fs.get_status(path)
            idx = list(st.info.blockIds).index(block_id)
            opts = pb.dataserver.OpenUfsBlockOptions(
                ufs_path=st.info.ufsPath, offset_in_file=idx * st.info.blockSizeBytes,
                block_size=st.info.fileBlockInfos[idx].blockInfo.length, mountId=st.info.mountId)
            if ctx.worker is not None and ctx.worker.has_block(block_id):
                continue
            locs = st.info.fileBlockInfos[idx].blockInfo.locations
            if ctx.worker is not None and locs:
                src = locs[0].workerAddress
                plane = getattr(ctx.worker, "transfer_plane", None)
                reach = [l.workerAddress for l in locs if plane is not None and plane.can_reach(l.workerAddress)]
                if reach:               # a peer on this node: pull over xGMI (gRPC fallback inside)
                    plane.pull_block(block_id, reach[0], opts.block_size)
                else:
                    from ..worker.remote import remote_block_fetcher
                    remote_block_fetcher(ctx.worker, src.host, src.rpcPort, opts.block_size)(block_id)
                loaded += opts.block_size
            elif ctx.worker is not None:
                from_ufs.append((block_id, opts))
        if from_ufs:
            ctx.worker.cache_blocks_from_ufs(from_ufs)
            loaded += sum(o.block_size for b, o in from_ufs if ctx.worker.has_block(b))
        return loaded

    def join(self, cfg, task_results):
        return {"bytes_loaded": sum(v or 0 for v in task_results.values())}


@plan("persist")
class PersistDefinition(PlanDefinition):
    def select_executors(self, cfg, job_workers, fs):
        if not job_workers:
            raise ex.FailedPreconditionException("no job worker available for persist")
        st = fs.get_status(cfg.path)
        # prefer the worker holding the most bytes of the file
        score = {}
        for fbi in st.info.fileBlockInfos:
            for l in fbi.blockInfo.locations:
                jw = _find_job_worker(job_workers, l.workerAddress)
                if jw is not None:
                    score[jw.id] = score.get(jw.id, 0) + fbi.blockInfo.length
        best = max(job_workers, key=lambda jw: score.get(jw.id, 0))
        return [(best, cfg.path)]

    def run_task(self, cfg, args, ctx):
        from .persist import persist_file
        return persist_file(ctx.fs, args)


@plan("replicate")
class ReplicateDefinition(PlanDefinition):
    def select_executors(self, cfg, job_workers, fs):
        bi = fs.ctx.block_master().GetBlockInfo(pb.block.GetBlockInfoPRequest(blockId=cfg.block_id)).blockInfo
        have = {(l.workerAddress.host, l.workerAddress.rpcPort) for l in bi.locations}
        cands = [jw for jw in job_workers if (jw.address.host, jw.block_worker_port) not in have]
        random.shuffle(cands)
        src = (bi.locations[0].workerAddress.host, bi.locations[0].workerAddress.rpcPort) if bi.locations else None
        return [(jw, {"src": src, "length": bi.length, "path": cfg.path}) for jw in cands[:cfg.replicas]]

    def run_task(self, cfg, args, ctx):
        if ctx.worker is None or ctx.worker.has_block(cfg.block_id):
            return 0
        plane = getattr(ctx.worker, "transfer_plane", None)
        if plane is not None and args["src"] is not None and plane.can_reach(args["src"]):
            plane.pull_block(cfg.block_id, args["src"], args["length"])
        elif args["src"] is not None:
            from ..worker.remote import remote_block_fetcher
            remote_block_fetcher(ctx.worker, args["src"][0], args["src"][1], args["length"])(cfg.block_id)
        elif args["path"]:
            st = ctx.fs.get_status(args["path"])
            idx = list(st.info.blockIds).index(cfg.block_id)
            ctx.worker.cache_block_from_ufs(cfg.block_id, pb.dataserver.OpenUfsBlockOptions(
                ufs_path=st.info.ufsPath, offset_in_file=idx * st.info.blockSizeBytes, block_size=args["length"],
                mountId=st.info.mountId))
        return args["length"]


@plan("evict")
class EvictDefinition(PlanDefinition):
    def select_executors(self, cfg, job_workers, fs):
        bi = fs.ctx.block_master().GetBlockInfo(pb.block.GetBlockInfoPRequest(blockId=cfg.block_id)).blockInfo
        holders = [jw for l in bi.locations for jw in [_find_job_worker(job_workers, l.workerAddress)] if jw]
        random.shuffle(holders)
        return [(jw, None) for jw in holders[:cfg.replicas]]

    def run_task(self, cfg, args, ctx):
        from ..utils import ids
        if ctx.worker is not None and ctx.worker.has_block(cfg.block_id):
            ctx.worker.remove_block(ids.MIGRATE_DATA_SESSION_ID, cfg.block_id)
            return 1
        return 0


@plan("move")
class MoveDefinition(PlanDefinition):
    def select_executors(self, cfg, job_workers, fs):
        return [(jw, None) for jw in job_workers if not cfg.worker_host or jw.address.host == cfg.worker_host][:1]

    def run_task(self, cfg, args, ctx):
        from ..utils import ids
        if ctx.worker is not None and ctx.worker.has_block(cfg.block_id):
            ctx.worker.move_block(ids.MIGRATE_DATA_SESSION_ID, cfg.block_id, medium=cfg.medium)
            return 1
        return 0


@plan("migrate")
class MigrateDefinition(PlanDefinition):
    def select_executors(self, cfg, job_workers, fs):
        if not job_workers:
            raise ex.FailedPreconditionException("no job worker available for migrate")
        src = fs.get_status(cfg.source)
        if src.info.folder:
            pairs = []
            base = cfg.source.rstrip("/")
            for s in fs.list_status(cfg.source, recursive=True):
                if not s.info.folder:
                    pairs.append((s.info.path, cfg.destination.rstrip("/") + s.info.path[len(base):]))
        else:
            dst = cfg.destination
            try:
                if fs.get_status(dst).info.folder:
                    dst = dst.rstrip("/") + "/" + src.info.name
            except ex.NotFoundException:
                pass
            pairs = [(src.info.path, dst)]
        out = []
        for i, pair in enumerate(pairs):
            out.append((job_workers[i % len(job_workers)], pair))
        return out

    def run_task(self, cfg, args, ctx):
        src, dst = args
        if ctx.fs.exists(dst, load_metadata="NEVER"):
            if not cfg.overwrite:
                raise ex.FileAlreadyExistsException(f"{dst} already exists")
            ctx.fs.delete(dst)
        n = 0
        with ctx.fs.open_file(src) as fin, ctx.fs.create_file(dst, write_type=cfg.write_type) as fout:
            while True:
                data = fin.read(8 << 20)
                if not data:
                    break
                fout.write(data)
                n += len(data)
        if cfg.delete_source:
            ctx.fs.delete(src)
        return n

    def join(self, cfg, task_results):
        return {"files": len(task_results), "bytes": sum(v or 0 for v in task_results.values())}


@plan("transform")
class TransformDefinition(PlanDefinition):
    """Table transformation (reference job/server/.../plan/transform/CompactDefinition.java +
    format/{csv,orc,parquet}: rewrite each partition's files as at most ``file.count.max``
    Parquet files under the transformation's location)."""

    @staticmethod
    def _max_files(defn: str) -> int:
        for kv in defn.replace(";", " ").split():
            k, _, v = kv.partition("=")
            if k.strip() == "file.count.max":
                return max(1, int(v))
        return 100

    def select_executors(self, cfg, job_workers, fs):
        if not job_workers:
            raise ex.FailedPreconditionException("no job worker available for transform")
        return [(job_workers[i % len(job_workers)], p) for i, p in enumerate(cfg.partitions)]

    def run_task(self, cfg, args, ctx):
        import io
        import posixpath

        import pyarrow as pa
        import pyarrow.parquet as pq

        from ..table.udb import format_of, read_table_bytes
        tables = [read_table_bytes(ctx.fs.read_file(f), format_of(f)) for f in args["files"]]
        tbl = pa.concat_tables(tables, promote_options="default") if len(tables) > 1 else tables[0]
        n = min(self._max_files(cfg.transform), max(1, tbl.num_rows))
        ctx.fs.create_directory(args["dst"], recursive=True, allow_exists=True)
        per = -(-tbl.num_rows // n)
        out = []
        for i in range(n):
            part = tbl.slice(i * per, per)
            if part.num_rows == 0 and i > 0:
                break
            buf = io.BytesIO()
            pq.write_table(part, buf)
            path = posixpath.join(args["dst"], f"part-{i:05d}.parquet")
            if ctx.fs.exists(path):
                ctx.fs.delete(path)
            ctx.fs.write_file(path, buf.getvalue())
            out.append(path)
        return {"spec": args["spec"] or "_", "files": out}

    def join(self, cfg, task_results):
        return {r["spec"]: r["files"] for r in task_results.values() if r}


@plan("stress")
class StressBenchDefinition(PlanDefinition):
    def select_executors(self, cfg, job_workers, fs):
        ws = list(job_workers)
        if cfg.cluster_limit > 0:
            ws = ws[:cfg.cluster_limit]
        out = []
        for i, jw in enumerate(ws):
            args = list(cfg.args)
            # each task gets its own base directory (reference BaseParameters --id / task id)
            if "--base" in args:
                j = args.index("--base") + 1
                args[j] = f"{args[j].rstrip('/')}/task{i}"
            elif cfg.bench != "ufs-io":
                args += ["--base", f"/stress-{cfg.bench}-base/task{i}"]
            out.append((jw, args))
        return out

    def run_task(self, cfg, args, ctx):
        from ..stress import run_local
        return run_local(cfg.bench, args, ctx.fs)

    def join(self, cfg, task_results):
        from ..stress import merge_results
        return merge_results(cfg.bench, list(task_results.values()))
