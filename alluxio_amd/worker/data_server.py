"""Native data port of a worker: the BlockWorker gRPC service on the C++ HTTP/2 front end.

Parity: core/server/worker/src/main/java/alluxio/worker/grpc/GrpcDataServer.java:50-198 (the
worker's data server, a Netty gRPC server of BlockWorkerImpl), BlockReadHandler.java:111-152 and
core/common/src/main/java/alluxio/grpc/ReadResponseMarshaller.java:38-80.

``ReadBlock`` of a block the store holds is answered on the C++ I/O threads (csrc/data_server.cpp:
read lock for the call, HBM chunks DMA'd into pinned staging, ``offset_received`` window), and so
are the chunks of an ALLUXIO_BLOCK ``WriteBlock`` (written into the temp block as they arrive; the
commit -- CRC32C, the master's CommitBlock -- runs in Python as the internal ``NativeWriteCommit``
call posted at the client's half-close, whose reply ends the stream; reference
BlockWriteHandler.java), and so are UFS_FILE writes into a mount the worker has found to be a
local directory (temp file renamed over the target at the half-close; reference
UfsFileWriteHandler.java).  Every other BlockWorker call -- UFS writes and read-through,
OpenLocalBlock, AsyncCache, ... -- runs the same Python servicer as the grpcio port, through the
front end's streaming bridge.  The port is
advertised as ``WorkerNetAddress.dataPort``; clients stream block bytes from it
(client/streams.py ``GrpcBlockReader.native_source``).
"""
from __future__ import annotations

import logging

from .services import SVC_BLOCK_WORKER

LOG = logging.getLogger(__name__)

READ_BLOCK_PATH = f"/{SVC_BLOCK_WORKER}/ReadBlock"
WRITE_BLOCK_PATH = f"/{SVC_BLOCK_WORKER}/WriteBlock"
COMMIT_PATH = f"/{SVC_BLOCK_WORKER}/NativeWriteCommit"
COMMIT_BATCH_PATH = f"/{SVC_BLOCK_WORKER}/NativeCommitBatch"
RESOLVE_MOUNT_PATH = f"/{SVC_BLOCK_WORKER}/ResolveUfsMount"
READ_RANGE_PATH = f"/{SVC_BLOCK_WORKER}/ReadUfsRange"


def available() -> bool:
    from ..ops.native import lib
    return bool(lib().FrameRpcServer.grpc_available())


class WorkerDataServer:
    def __init__(self, rpc_server, worker, conf, host: str, domain_socket: str | None = None):
        from ..ops.native import lib
        from ..rpc.native import NativeRpcFrontend
        self.worker = worker
        self.frontend = NativeRpcFrontend(
            rpc_server, host, conf.get_int("alluxio.worker.data.server.native.port", "0"),
            fast_threads=2, blocking_threads=conf.get_int("alluxio.worker.data.server.native.blocking.threads", "8"),
            io_threads=conf.get_int("alluxio.worker.data.server.native.io.threads", "8"),
            services={SVC_BLOCK_WORKER}, bridge_services={SVC_BLOCK_WORKER},
            stream_threads=conf.get_int("alluxio.worker.data.server.native.stream.threads", "128"))
        # request streams (WriteBlock uploads) get a window of a few chunks
        lib().set_stream_window(self.frontend.server,
                                conf.get_bytes("alluxio.worker.data.server.native.write.window", "4MB"))
        if domain_socket:
            # the domain-socket data server (same-node clients skip TCP): same service, same port
            import os
            os.makedirs(os.path.dirname(domain_socket) or ".", exist_ok=True)
            lib().listen_unix(self.frontend.server, domain_socket)
        # mounts the I/O threads reach by themselves (local directories, plain-HTTP S3), registered
        # by the worker after it served a first call of the mount in Python (note_ufs_mount)
        self.ufs_roots = lib().UfsMounts()
        worker.native_ufs_roots = self.ufs_roots
        native_cold = conf.get_bool("alluxio.worker.data.server.native.ufs.read.enabled", "true")
        # the native block commit (csrc/data_server.cpp BlockCommitter): WriteBlock streams and cold
        # read-throughs hand their blocks to a committer thread -- streamed per-page CRC32C of HBM
        # blocks, store commit, one NativeCommitBatch (master CommitBlocks) per group of blocks
        self.stats = lib().DataServerStats()
        self.committer = None
        if conf.get_bool("alluxio.worker.data.server.native.commit.enabled", "true"):
            self.committer = lib().BlockCommitter(
                worker.native, self.frontend.method_index(COMMIT_BATCH_PATH),
                conf.get_bool("alluxio.worker.data.crc.device.enabled", "true"),
                conf.get_bool("alluxio.worker.data.crc.enabled"), self.stats)
        # ReadBlock: cached blocks from the store; cold blocks of registered mounts read through
        # from the UFS on a background thread per call and committed via NativeWriteCommit
        self.stats = lib().serve_block_reads(
            self.frontend.server, self.frontend.method_index(READ_BLOCK_PATH), worker.native,
            conf.get_bytes("alluxio.worker.network.reader.max.chunk.size.bytes", "2MB"),
            conf.get_bytes("alluxio.worker.network.reader.buffer.size", "4MB"),
            mounts=self.ufs_roots if native_cold else None,
            commit_method=self.frontend.method_index(COMMIT_PATH),
            ufs_slot_bytes=conf.get_bytes("alluxio.worker.ufs.ingest.chunk.size", "8MB"),
            ufs_depth=conf.get_int("alluxio.worker.ufs.ingest.depth", "3"),
            ufs_max_active=conf.get_int("alluxio.worker.data.server.native.ufs.read.max.active", "256"),
            stats=self.stats, committer=self.committer,
            resolve_method=self.frontend.method_index(RESOLVE_MOUNT_PATH),
            read_range_method=self.frontend.method_index(READ_RANGE_PATH),
            ufs_readahead=conf.get_bool("alluxio.worker.data.server.native.ufs.readahead.enabled"),
            ufs_create_after_reads=conf.get_int("alluxio.worker.data.server.native.ufs.create.after.reads"))
        # WriteBlock of ALLUXIO_BLOCK writes: chunks into the store on the I/O threads, the commit
        # (CRC, master report) as the internal NativeWriteCommit call (BlockWorkerService).
        # UFS_FILE writes of mounts the worker found to be local directories: into the file.
        native_ufs_write = conf.get_bool("alluxio.worker.data.server.native.ufs.write.enabled", "true")
        lib().serve_block_writes(
            self.frontend.server, self.frontend.method_index(WRITE_BLOCK_PATH),
            self.frontend.method_index(COMMIT_PATH), worker.native,
            conf.get_bytes("alluxio.worker.network.writer.staging.size", "4MB"), self.stats,
            self.ufs_roots if native_ufs_write else None, committer=self.committer)
        self.port = None

    def start(self) -> int:
        self.port = self.frontend.start()
        m = self.worker.metrics
        st = self.stats
        m.gauge("DataServerNativeStreams", lambda: st.streams)
        m.gauge("DataServerBridgedStreams", lambda: st.declined)
        # bytes the C++ server sent count in the worker's read metrics (BytesReadDomain for
        # same-node domain-socket clients, BytesReadRemote otherwise)
        m.counter("BytesReadAlluxio").add_source(lambda: st.bytes)
        m.counter("BytesReadDomain").add_source(lambda: st.domain_bytes)
        m.counter("BytesReadRemote").add_source(lambda: st.bytes - st.domain_bytes)
        m.counter("BytesWrittenAlluxio").add_source(lambda: st.write_bytes)
        m.gauge("DataServerNativeWriteStreams", lambda: st.write_streams)
        m.gauge("DataServerNativeUfsWriteStreams", lambda: st.ufs_write_streams)
        m.counter("BytesWrittenUfsAll").add_source(lambda: st.ufs_write_bytes)
        m.gauge("DataServerNativeColdStreams", lambda: st.cold_streams)
        m.gauge("DataServerNativeColdActive", lambda: st.cold_active)
        m.gauge("DataServerNativeCommits", lambda: st.commits)
        m.gauge("DataServerNativeCommitBatches", lambda: st.commit_batches)
        m.gauge("DataServerNativeCommitFailures", lambda: st.commit_failures)
        return self.port

    def stop(self) -> None:
        import time
        self.frontend.stop()
        self.committer = None      # its thread drains what it holds, then exits (it owns a store ref)
        # background UFS readers of cancelled cold reads finish their current read, wait for their
        # H2D copies and drop their temp blocks: the store must outlive them
        self.stats.stop_background_reads()   # next-block read-aheads outlive their streams
        deadline = time.time() + 30
        while (self.stats.cold_active > 0 or self.stats.store_tasks > 0) and time.time() < deadline:
            time.sleep(0.01)                # (and AppendBlock copies out of the store on the file pool)
