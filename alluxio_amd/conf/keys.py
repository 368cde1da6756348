"""Typed property-key registry.

Parity: core/common/src/main/java/alluxio/conf/PropertyKey.java (504 named keys + templates),
core/common/src/main/java/alluxio/conf/Source.java:30-80 (source priority).  Every reference key
name and default is registered from :mod:`keys_table`; this module adds the per-tier templates
(``alluxio.worker.tieredstore.level{N}.*``, PropertyKey.java:2933-2985) and the MI355X-specific
keys (HBM arena sizing, page size, GPU device selection, RCCL data plane).
"""
from __future__ import annotations

import enum
import re
import threading

from .keys_table import KEYS as _REFERENCE_KEYS


class Scope(enum.Flag):
    MASTER = 1
    WORKER = 2
    CLIENT = 4
    SERVER = MASTER | WORKER
    ALL = MASTER | WORKER | CLIENT
    NONE = 0


class PropertyKey:
    __slots__ = ("name", "default", "scope", "aliases", "description", "template")

    def __init__(self, name, default=None, scope=Scope.ALL, aliases=(), description="",
                 template=None):
        self.name = name
        self.default = None if default is None else str(default)
        self.scope = scope
        self.aliases = tuple(aliases)
        self.description = description
        self.template = template

    def __str__(self) -> str:
        return self.name

    def __repr__(self) -> str:
        return f"PropertyKey({self.name!r})"

    def __hash__(self) -> int:
        return hash(self.name)

    def __eq__(self, other) -> bool:
        if isinstance(other, str):
            return self.name == other
        return isinstance(other, PropertyKey) and other.name == self.name


_REGISTRY: dict[str, PropertyKey] = {}
_ALIASES: dict[str, str] = {}
_LOCK = threading.Lock()


def register(key: PropertyKey) -> PropertyKey:
    with _LOCK:
        _REGISTRY[key.name] = key
        for a in key.aliases:
            _ALIASES[a] = key.name
    return key


for _name, _default, _scope, _aliases in _REFERENCE_KEYS:
    register(PropertyKey(_name, _default, Scope[_scope], _aliases))


class Template:
    """Parametrised key families (reference ``PropertyKey.Template``)."""

    def __init__(self, fmt: str, regex: str, default_fn=None, scope=Scope.ALL):
        self.fmt = fmt
        self.regex = re.compile(regex)
        self.default_fn = default_fn
        self.scope = scope

    def format(self, *args) -> PropertyKey:
        name = self.fmt % args
        with _LOCK:
            k = _REGISTRY.get(name)
        if k is not None:
            return k
        default = self.default_fn(*args) if self.default_fn else None
        return register(PropertyKey(name, default, self.scope, template=self))

    def match(self, name: str):
        return self.regex.fullmatch(name)


_TIER_ALIAS_DEFAULTS = {0: "MEM", 1: "SSD", 2: "HDD"}
_TIER_MEDIUM_DEFAULTS = {0: "HBM", 1: "DRAM", 2: "SSD"}


class Templates:
    WORKER_TIERED_STORE_LEVEL_ALIAS = Template(
        "alluxio.worker.tieredstore.level%d.alias", r"alluxio\.worker\.tieredstore\.level(\d+)\.alias",
        lambda i: _TIER_ALIAS_DEFAULTS.get(i), Scope.WORKER)
    WORKER_TIERED_STORE_LEVEL_DIRS_PATH = Template(
        "alluxio.worker.tieredstore.level%d.dirs.path",
        r"alluxio\.worker\.tieredstore\.level(\d+)\.dirs\.path",
        lambda i: {0: "hbm:0"}.get(i, "/tmp/alluxio_amd/tier%d" % i), Scope.WORKER)
    WORKER_TIERED_STORE_LEVEL_DIRS_QUOTA = Template(
        "alluxio.worker.tieredstore.level%d.dirs.quota",
        r"alluxio\.worker\.tieredstore\.level(\d+)\.dirs\.quota",
        lambda i: {0: "4GB", 1: "8GB"}.get(i, "16GB"), Scope.WORKER)
    WORKER_TIERED_STORE_LEVEL_DIRS_MEDIUMTYPE = Template(
        "alluxio.worker.tieredstore.level%d.dirs.mediumtype",
        r"alluxio\.worker\.tieredstore\.level(\d+)\.dirs\.mediumtype",
        lambda i: _TIER_MEDIUM_DEFAULTS.get(i, "SSD"), Scope.WORKER)
    WORKER_TIERED_STORE_LEVEL_HIGH_WATERMARK_RATIO = Template(
        "alluxio.worker.tieredstore.level%d.watermark.high.ratio",
        r"alluxio\.worker\.tieredstore\.level(\d+)\.watermark\.high\.ratio",
        lambda i: "0.95", Scope.WORKER)
    WORKER_TIERED_STORE_LEVEL_LOW_WATERMARK_RATIO = Template(
        "alluxio.worker.tieredstore.level%d.watermark.low.ratio",
        r"alluxio\.worker\.tieredstore\.level(\d+)\.watermark\.low\.ratio",
        lambda i: "0.7", Scope.WORKER)
    WORKER_TIERED_STORE_LEVEL_RESERVED_RATIO = Template(
        "alluxio.worker.tieredstore.level%d.reserved.ratio",
        r"alluxio\.worker\.tieredstore\.level(\d+)\.reserved\.ratio",
        lambda i: None, Scope.WORKER)
    MASTER_TIERED_STORE_GLOBAL_LEVEL_ALIAS = Template(
        "alluxio.master.tieredstore.global.level%d.alias",
        r"alluxio\.master\.tieredstore\.global\.level(\d+)\.alias",
        lambda i: _TIER_ALIAS_DEFAULTS.get(i), Scope.MASTER)
    LOCALITY_TIER = Template("alluxio.locality.%s", r"alluxio\.locality\.(\w+)")
    MASTER_MOUNT_TABLE_OPTION = Template(
        "alluxio.master.mount.table.%s.option", r"alluxio\.master\.mount\.table\.(\w+)\.option")
    USER_NETWORK_KEEPALIVE_TIME = Template(
        "alluxio.user.network.%s.keepalive.time", r"alluxio\.user\.network\.(\w+)\.keepalive\.time")


# --- MI355X-specific keys --------------------------------------------------------------------
K = {}


def _k(attr: str, name: str, default, scope=Scope.ALL, description=""):
    key = register(PropertyKey(name, default, scope, description=description))
    K[attr] = key
    return key


_k("PROXY_HDFS_RPC_PORT", "alluxio.proxy.hdfs.rpc.port", "-1", Scope.NONE,
   "NameNode (Hadoop IPC ClientProtocol) port of the proxy's HDFS-protocol gateway; -1 disables it, "
   "0 picks a free port.  Hadoop clients then use hdfs://<proxy>:<port>/.")
_k("PROXY_HDFS_DATA_PORT", "alluxio.proxy.hdfs.data.port", "0", Scope.NONE,
   "DataNode (DataTransferProtocol) port of the HDFS-protocol gateway (0: a free port).")
_k("PROXY_HDFS_HOSTNAME", "alluxio.proxy.hdfs.hostname", "", Scope.NONE,
   "Host the gateway advertises as its DataNode address (default: the bind host).")
_k("WORKER_GPU_DEVICE", "alluxio.worker.gpu.device", "-1", Scope.WORKER,
   "HIP device index this worker owns (-1: LOCAL_RANK or 0).")
_k("WORKER_HBM_PAGE_SIZE", "alluxio.worker.hbm.page.size", "2MB", Scope.WORKER,
   "Fixed page size of the HBM arena; blocks are ceil(len/page) pages.")
_k("WORKER_HBM_ARENA_FRACTION", "alluxio.worker.hbm.arena.fraction", "0.0", Scope.WORKER,
   "If >0, size the HBM tier as this fraction of free device memory (overrides the quota).")
_k("WORKER_DATA_CRC_ENABLED", "alluxio.worker.data.crc.enabled", "false", Scope.WORKER,
   "Compute a CRC32C per page when a block is committed (HIP kernel).")
_k("WORKER_DATA_CRC_DEVICE_ENABLED", "alluxio.worker.data.crc.device.enabled", "true", Scope.WORKER,
   "Compute the per-page CRC32C of every block committed to the HBM tier (device kernel); peers "
   "verify pulled blocks against it (alluxio.worker.peer.verify.crc).")
_k("WORKER_PEER_VERIFY_CRC", "alluxio.worker.peer.verify.crc", "true", Scope.WORKER,
   "Verify a block pulled from a peer worker against the source's CRC32Cs before committing it.")
_k("USER_SHORT_CIRCUIT_VERIFY_CRC", "alluxio.user.short.circuit.verify.crc", "false", Scope.CLIENT,
   "Verify a short-circuit (HIP IPC / shared DRAM) block against its worker's CRC32Cs at open.")
_k("WORKER_DATA_COMPRESSION", "alluxio.worker.data.compression", "NONE", Scope.WORKER,
   "Block codec for the host tiers: NONE | LZ4.")
_k("WORKER_RCCL_ENABLED", "alluxio.worker.rccl.enabled", "true", Scope.WORKER,
   "Use RCCL over xGMI for worker<->worker block transfer when ranks share a node.")
_k("WORKER_DATA_SERVER_DOMAIN_SOCKET_DEFAULT", "alluxio.worker.data.server.domain.socket.default.enabled", "true",
   Scope.WORKER, "With no alluxio.worker.data.server.domain.socket.address set, listen on a per-worker Unix "
   "domain socket under /tmp/alluxio-uds-<uid> as well, so same-node clients skip loopback TCP "
   "(profiles/r6_remote_read_uds.md: one stream 15.4 vs 8.7 GB/s).")
_k("WORKER_DATA_SERVER_NATIVE_COMMIT_ENABLED", "alluxio.worker.data.server.native.commit.enabled", "true",
   Scope.WORKER, "Commit natively written blocks in C++ (streamed per-page CRC32C, store commit, one master "
   "CommitBlocks report per group of blocks) instead of one Python NativeWriteCommit per block.")
_k("WORKER_HBM_EVICT_BATCH_BYTES", "alluxio.worker.hbm.evict.batch.bytes", "1GB", Scope.WORKER,
   "With an HBM tier, the least one eviction round frees (at most 1/32 of the smallest HBM dir): "
   "the device victim selection runs once per batch of evicting creates, not once per create. "
   "alluxio.worker.tieredstore.free.ahead.bytes, when larger, wins.")
_k("USER_NATIVE_READER_NEXT_BLOCK_START", "alluxio.user.native.reader.next.block.start.enabled", "false",
   Scope.CLIENT, "A large sequential read that runs into the next remote block starts that block's ReadBlock "
   "stream while it still reads the current one. Off by default: one stream cached +2.5%, cold -15% on "
   "the same box (the next block's read-through competes with the current one; "
   "profiles/r6_next_block_start_ab.jsonl).")
_k("WORKER_DATA_SERVER_NATIVE_WRITE_WINDOW", "alluxio.worker.data.server.native.write.window", "4MB",
   Scope.WORKER, "HTTP/2 stream window of request streams on the native data server (WriteBlock uploads): "
   "how many bytes a writer may have in flight before the worker has taken them.")
_k("WORKER_IPC_ENABLED", "alluxio.worker.ipc.enabled", "true", Scope.WORKER,
   "Hand out HIP IPC handles for short-circuit reads of HBM pages.")
_k("WORKER_STAGING_BUFFER_SIZE", "alluxio.worker.staging.buffer.size", "64MB", Scope.WORKER,
   "Pinned host staging ring used for UFS->HBM and HBM->host copies.")
_k("WORKER_EVICTION_DEVICE_ENABLED", "alluxio.worker.eviction.device.enabled", "true", Scope.WORKER,
   "Keep the LRU/LRFU annotations in HBM and select eviction victims with the grid-wide device "
   "select (K4-K6) when the store has an HBM tier; false = host sort.")
_k("WORKER_UFS_INGEST_CHUNK_SIZE", "alluxio.worker.ufs.ingest.chunk.size", "8MB", Scope.WORKER,
   "UFS read size of the UFS->HBM ingest pipeline (one pinned staging buffer each).")
_k("WORKER_UFS_INGEST_DEPTH", "alluxio.worker.ufs.ingest.depth", "3", Scope.WORKER,
   "Staging buffers per ingest pipeline: UFS reads run this many chunks ahead of the H2D DMA.")
_k("UNDERFS_LZ4_FRAME_DECODE", "alluxio.underfs.lz4.frame.decode", "false", Scope.SERVER,
   "Present *.lz4 files of a mount that are LZ4 frames (independent blocks, content size) as their "
   "decompressed bytes; HBM workers decode them on the GPU when caching (mount option or site key).")
_k("WORKER_UFS_INGEST_BULK_STAGING_SIZE", "alluxio.worker.ufs.ingest.bulk.staging.size", "64MB", Scope.WORKER,
   "Pinned staging of the bulk small-file ingest (two halves: preads fill one while the other is "
   "copied into HBM).")
_k("WORKER_UFS_INGEST_BULK_THREADS", "alluxio.worker.ufs.ingest.bulk.threads", "16", Scope.WORKER,
   "Native reader threads of the bulk small-file ingest.")
_k("WORKER_TIEREDSTORE_EVICTION_DEMOTE", "alluxio.worker.tieredstore.eviction.demote", "true", Scope.WORKER,
   "Eviction from a tier with a lower tier demotes the victims into it (one batched HBM->DRAM / "
   "DRAM->SSD move, making room there recursively) instead of dropping them.")
_k("WORKER_HBM_DEVICE_ALLOC_ENABLED", "alluxio.worker.hbm.device.alloc.enabled", "true", Scope.WORKER,
   "Claim the pages of bulk block creates and of the bulk UFS ingest with the device page magazine "
   "(K7: resident free-page bitmap in HBM, claim kernel + fused scatter).  Bulk creates of 150k pages "
   "run 3x faster than the host bitmap scan, ingest at parity (profiles/r3_evict_bench_arc.jsonl); "
   "single small creates stay on the host scan (below alloc.min.pages).")
_k("WORKER_PAGE_ACCOUNTING_CHECK", "alluxio.worker.debug.page.accounting.check", "false", Scope.WORKER,
   "Debug: after every bulk create / bulk UFS ingest, verify that the host page pool, the K7 device "
   "magazine (its HBM bitmap against mag_pages) and the block page lists partition each arena "
   "(BlockStore::check_pages); violations are logged and counted in PageAccountingErrors.")
_k("WORKER_HBM_DEVICE_ALLOC_MIN_PAGES", "alluxio.worker.hbm.device.alloc.min.pages", "1024", Scope.WORKER,
   "Smallest bulk create (in pages) that uses the device allocator when it is enabled.")
_k("WORKER_DATA_SERVER_NATIVE_ENABLED", "alluxio.worker.data.server.native.enabled", "true", Scope.WORKER,
   "Serve the BlockWorker service on a native HTTP/2 gRPC data port (csrc/data_server.cpp): ReadBlock "
   "of a block in the store is streamed from C++ I/O threads (HBM chunks DMA'd into pinned staging), "
   "other calls are bridged to the Python servicer.  Advertised as WorkerNetAddress.dataPort.")
_k("WORKER_DATA_SERVER_NATIVE_PORT", "alluxio.worker.data.server.native.port", "0", Scope.WORKER,
   "Port of the native data server (0: any free port; the worker advertises it when registering).")
_k("WORKER_DATA_SERVER_NATIVE_IO_THREADS", "alluxio.worker.data.server.native.io.threads", "8", Scope.WORKER,
   "epoll I/O threads of the native data server (each stages and sends the chunks of its connections).")
_k("WORKER_DATA_SERVER_NATIVE_STREAM_THREADS", "alluxio.worker.data.server.native.stream.threads", "128",
   Scope.WORKER, "Threads running streaming calls the native data server bridges to Python (writes, UFS "
   "read-through).")
_k("USER_NATIVE_READER_ENABLED", "alluxio.user.native.reader.enabled", "true", Scope.CLIENT,
   "Host reads of FileInStream go through the native chunk-buffered reader (csrc/block_source.cpp): a "
   "read(buf) inside the buffered chunk is a memcpy; refills come from HIP-IPC HBM (D2H DMA), shared "
   "DRAM, the in-process store or a native gRPC ReadBlock stream.")
_k("USER_SHORT_CIRCUIT_WRITE_ENABLED", "alluxio.user.short.circuit.write.enabled", "true", Scope.CLIENT,
   "Blocks written to a same-node worker in another process go into its shared arena directly "
   "(OpenDeviceWrite: HBM pages mapped through HIP IPC, DRAM through its memfd) instead of over "
   "WriteBlock; needs alluxio.user.short.circuit.enabled.")
_k("USER_NATIVE_WRITER_ENABLED", "alluxio.user.native.writer.enabled", "true", Scope.CLIENT,
   "Block writes to a remote (other-process) worker use the native gRPC client (csrc/block_source.cpp "
   "GrpcBlockSink: WriteBlock over HTTP/2 with the chunks framed around the caller's bytes, GIL "
   "released) instead of grpcio.  UFS-fallback writes keep grpcio.")
_k("WORKER_DATA_SERVER_NATIVE_UFS_WRITE_ENABLED", "alluxio.worker.data.server.native.ufs.write.enabled", "true",
   Scope.WORKER,
   "UFS_FILE WriteBlock streams (THROUGH / CACHE_THROUGH writes of remote clients) into a mount the "
   "worker has found to be a local directory are written by the native data server's I/O threads "
   "(temp file renamed over the target at the end) instead of the Python servicer.")
_k("WORKER_DATA_SERVER_NATIVE_UFS_READ_ENABLED", "alluxio.worker.data.server.native.ufs.read.enabled", "true",
   Scope.WORKER,
   "ReadBlock of a block the worker does not hold, with open_ufs_block_options of a mount the worker has "
   "found to be a local directory or a plain-HTTP S3 endpoint, is read through natively: a background "
   "thread reads the UFS into pinned slots (alluxio.worker.ufs.ingest.chunk.size x .depth), copies each "
   "into a temp block and the I/O thread streams it as it lands; the block is committed at the end.")
_k("WORKER_DATA_SERVER_NATIVE_UFS_READ_MAX_ACTIVE", "alluxio.worker.data.server.native.ufs.read.max.active",
   "256", Scope.WORKER, "Concurrent native cold reads (one UFS reader thread each); more go to Python.")
_k("WORKER_DATA_SERVER_NATIVE_UFS_READAHEAD_ENABLED", "alluxio.worker.data.server.native.ufs.readahead.enabled",
   "true", Scope.WORKER, "A native whole-block read-through reads the first two UFS reads of the file's next "
   "block (one chunk, then one alluxio.worker.ufs.ingest.chunk.size slot) into pinned buffers once its own "
   "reads are done; the next block's cold stream sends them without waiting on the UFS. Pieces expire "
   "after 5 s.")
_k("WORKER_DATA_SERVER_NATIVE_UFS_CREATE_AFTER_READS", "alluxio.worker.data.server.native.ufs.create.after.reads",
   "2", Scope.WORKER, "UFS reads a native read-through sends before it creates its temp block in the store (the "
   "create allocates pages and may evict). 0: one per slot (alluxio.worker.ufs.ingest.depth). A/B on one box: "
   "2 reads 9.2-9.7 GB/s for one cold stream, one per slot 8.0-8.8 (profiles/r6_cold_create_ab.jsonl).")
_k("USER_FILE_CACHE_THROUGH_TEE_ENABLED", "alluxio.user.file.cache.through.tee.enabled", "true", Scope.CLIENT,
   "CACHE_THROUGH writes whose cache block and UFS file stream go to the same worker send each byte "
   "once (to the block stream); after the block commits, the UFS stream is told to append it and the "
   "worker copies it from its store (AppendBlock).  false = every byte is sent to both streams.")
_k("USER_FILE_CACHE_THROUGH_TEE_OBJECT_STORE_ENABLED", "alluxio.user.file.cache.through.tee.object.store.enabled",
   "auto", Scope.CLIENT,
   "The CACHE_THROUGH tee for files in object-store mounts (s3://...): true, false, or auto = tee a "
   "block when at least ...tee.object.store.min.streams CACHE_THROUGH streams are open in this client "
   "process.  Measured into S3 (profiles/r5_persist.md): 16 writers 10.3 GB/s teed vs 6.4 with two "
   "streams; 4 writers 4.1 vs 4.6; one 4 GiB writer 3.3 vs 4.8 (two streams upload parts as the bytes "
   "arrive).")
_k("USER_FILE_CACHE_THROUGH_TEE_OBJECT_STORE_MIN_STREAMS", "alluxio.user.file.cache.through.tee.object.store.min.streams",
   "8", Scope.CLIENT, "Open CACHE_THROUGH streams from which object-store blocks are teed in auto mode.")
_k("JOB_PERSIST_WORKER_APPEND_ENABLED", "alluxio.job.persist.worker.append.enabled", "true", Scope.ALL,
   "Persist jobs of files cached on one worker open the file's UFS stream on that worker and append "
   "its blocks from the store (AppendBlock, no bytes through the job process); false = read the file "
   "through the client and write it to the UFS.")
_k("MASTER_JOURNAL_NATIVE_WRITER_ENABLED", "alluxio.master.journal.native.writer.enabled", "true",
   Scope.MASTER,
   "UFS journal logs are written by the native group-commit writer (csrc/journal_log.cpp): a C++ "
   "thread frames, writes and fsyncs the queued entries and sends the replies of the RPCs each commit "
   "releases without taking the GIL.  false = the Python AsyncJournalWriter.")
_k("UNDERFS_OBJECT_STORE_UPLOAD_BUFFER_SIZE", "alluxio.underfs.object.store.upload.buffer.size", "256MB",
   Scope.SERVER,
   "Memory one object-store write may hold in multipart part buffers (parts of "
   "alluxio.underfs.s3.streaming.upload.partition.size): parts in flight = this / the part size, so an "
   "object of any size is written with bounded memory.")
_k("USER_SHORT_CIRCUIT_OPEN_TIMEOUT", "alluxio.user.short.circuit.open.timeout", "30s", Scope.CLIENT,
   "Deadline of importing a worker's HBM arena through HIP IPC; an import that has not returned by "
   "then makes short-circuit unavailable for that arena and the client reads over the data port.")
_k("USER_FILE_CACHE_THROUGH_OVERLAP_MIN", "alluxio.user.file.cache.through.overlap.min", "256KB", Scope.CLIENT,
   "CACHE_THROUGH write() calls of at least this many bytes send the UFS copy on the stream's helper "
   "thread while the cache copy runs; smaller ones write the two one after the other.")
_k("USER_DEVICE_READ_PARALLELISM", "alluxio.user.device.read.parallelism", "4", Scope.CLIENT,
   "A read into device or host memory that spans several blocks held by remote workers reads up to "
   "this many blocks at once, each over its own native ReadBlock stream (1: one block after another).")
_k("WORKER_NETWORK_WRITER_STAGING_SIZE", "alluxio.worker.network.writer.staging.size", "4MB", Scope.WORKER,
   "Pinned staging buffer per native WriteBlock stream of an HBM worker (H2D DMA of received chunks).")
_k("WORKER_TIEREDSTORE_DRAM_PREFAULT", "alluxio.worker.tieredstore.dram.prefault", "false", Scope.WORKER,
   "Populate the pages of DRAM-tier arenas in the background at startup (GPU hosts pin, and so "
   "populate, them anyway): first writes into a shared-memory page otherwise pay a fault that "
   "allocates and zeroes it.")
_k("USER_NATIVE_READER_BUFFER_SIZE", "alluxio.user.native.reader.buffer.size", "4MB", Scope.CLIENT,
   "Chunk buffer (pinned when a GPU is present) of the native host reader: bytes fetched per refill. "
   "4 MiB: short-circuit readers in 4 processes x 64 threads reach 81-84% of the same-run D2H copy roof "
   "(1 MiB: 21-33% when the processes share the GPU's NUMA node -- 4x the refill syncs; "
   "profiles/r5_host_read_numa.md).")
_k("USER_NATIVE_READER_PREFETCH_ENABLED", "alluxio.user.native.reader.prefetch.enabled", "true", Scope.CLIENT,
   "The native host reader fetches the next chunk of the block into its second buffer on a native "
   "thread pool while read(buf) calls drain the current one.")
_k("USER_READ_BATCH_SIZE", "alluxio.user.read.batch.size", "256", Scope.CLIENT,
   "Max read requests coalesced into one page-gather launch.")
_k("USER_FILE_READ_DEVICE", "alluxio.user.file.read.device", "cuda", Scope.CLIENT,
   "Preferred destination of client reads: cuda (HBM) or cpu (pinned host).")

_k("MASTER_HA_PRIMARY_SELECTOR", "alluxio.master.ha.primary.selector", "NONE", Scope.MASTER,
   "NONE (single master) or FILE_LOCK (HA: masters sharing the journal folder elect a primary "
   "with an exclusive lock on alluxio.master.ha.lock.file).")
_k("MASTER_HA_LOCK_FILE", "alluxio.master.ha.lock.file", "${alluxio.master.journal.folder}/.primary.lock",
   Scope.MASTER, "Election lock file for FILE_LOCK primary selection.")
_k("WEB_SERVER_ENABLED", "alluxio.web.server.enabled", "true", Scope.SERVER,
   "Serve the HTTP endpoints (/metrics/json, /metrics/prometheus, /api/v1/...) from master and "
   "worker processes.")
_k("JOB_MASTER_EMBEDDED_ENABLED", "alluxio.job.master.embedded.enabled", "true", Scope.MASTER,
   "Serve the job master from the file-system master process (same RPC port) instead of a "
   "separate job-master process.")
_k("JOB_WORKER_ENABLED", "alluxio.job.worker.enabled", "true", Scope.WORKER,
   "Run a job worker inside each block-worker process (tasks share the worker's HBM store).")
_k("USER_INPROCESS_TRANSPORT_ENABLED", "alluxio.user.network.inprocess.transport.enabled", "true", Scope.CLIENT,
   "Call servers that live in the same process directly instead of through gRPC (false forces "
   "every RPC over the network stack, as a client in another process would).")
_k("UNDERFS_OZONE_S3G_ENDPOINT", "alluxio.underfs.ozone.s3g.endpoint", None, Scope.SERVER,
   "Ozone S3 gateway endpoint used by the o3fs:// and ofs:// connectors (default "
   "http://<om-host>:9878).")


def get(name: str) -> PropertyKey:
    """Resolve a key by name, alias or template match."""
    with _LOCK:
        k = _REGISTRY.get(name)
        if k is None and name in _ALIASES:
            k = _REGISTRY[_ALIASES[name]]
    if k is not None:
        return k
    for t in vars(Templates).values():
        if isinstance(t, Template):
            m = t.match(name)
            if m:
                arg = m.group(1)
                return t.format(int(arg) if arg.isdigit() else arg)
    return register(PropertyKey(name, None, Scope.ALL))


def is_valid(name: str) -> bool:
    with _LOCK:
        if name in _REGISTRY or name in _ALIASES:
            return True
    return any(isinstance(t, Template) and t.match(name) for t in vars(Templates).values())


def all_keys() -> list[PropertyKey]:
    with _LOCK:
        return list(_REGISTRY.values())
