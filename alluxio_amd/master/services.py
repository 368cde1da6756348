"""gRPC service handlers of the master (proto <-> master method adapters).

Parity: core/server/master/src/main/java/alluxio/master/file/FileSystemMasterClientServiceHandler.java
(:122-408), FileSystemMasterWorkerServiceHandler, block/BlockMasterClientServiceHandler,
block/BlockMasterWorkerServiceHandler, meta/MetaMaster*ServiceHandler, metrics/
MetricsMasterClientServiceHandler, ServiceVersionClientServiceHandler.
"""
from __future__ import annotations

from ..rpc.marshal import RawReply, length_delimited
from ..proto import enum_name, pb
from ..security.acl import bits_from_proto, mode_from_pmode

SVC_FS_CLIENT = "alluxio.grpc.file.FileSystemMasterClientService"
SVC_FS_WORKER = "alluxio.grpc.file.FileSystemMasterWorkerService"
SVC_FS_JOB = "alluxio.grpc.file.FileSystemMasterJobService"
SVC_BLOCK_CLIENT = "alluxio.grpc.block.BlockMasterClientService"
SVC_BLOCK_WORKER = "alluxio.grpc.block.BlockMasterWorkerService"
SVC_META_CLIENT = "alluxio.grpc.meta.MetaMasterClientService"
SVC_META_CONFIG = "alluxio.grpc.meta.MetaMasterConfigurationService"
SVC_META_MASTER = "alluxio.grpc.meta.MetaMasterMasterService"
SVC_METRICS = "alluxio.grpc.metric.MetricsMasterClientService"
SVC_VERSION = "alluxio.grpc.version.ServiceVersionClientService"
SVC_JOURNAL = "alluxio.grpc.journal.JournalMasterClientService"
SVC_SASL = "alluxio.grpc.sasl.SaslAuthenticationService"

LOAD_TYPES = {0: "NEVER", 1: "ONCE", 2: "ALWAYS"}


def _common(opts):
    c = opts.commonOptions if opts is not None and opts.HasField("commonOptions") else None
    return c


def _sync_interval(opts) -> int:
    c = _common(opts)
    return c.syncIntervalMs if c is not None and c.HasField("syncIntervalMs") else -1


def _ttl(opts):
    c = _common(opts)
    if c is not None and c.HasField("ttl"):
        return c.ttl, enum_name(pb.grpc.TtlAction, c.ttlAction) if c.HasField("ttlAction") else "DELETE"
    return None, None


class FileSystemMasterClientServiceHandler:
    def __init__(self, fsm):
        self.m = fsm

    def CheckConsistency(self, req, ctx):
        return pb.file.CheckConsistencyPResponse(inconsistentPaths=self.m.check_consistency(req.path))

    def CompleteFile(self, req, ctx):
        o = req.options
        self.m.complete_file(req.path, ufs_length=o.ufsLength, async_persist=o.HasField("asyncPersistOptions"),
                             persistence_wait_ms=o.asyncPersistOptions.persistenceWaitTime
                             if o.HasField("asyncPersistOptions") else 0)
        return pb.file.CompleteFilePResponse()

    def CreateDirectory(self, req, ctx):
        o = req.options
        ttl, action = _ttl(o)
        self.m.create_directory(req.path, recursive=o.recursive, allow_exists=o.allowExists,
                                mode=mode_from_pmode(o.mode) if o.HasField("mode") else None,
                                write_type=enum_name(pb.file.WritePType, o.writeType) if o.HasField("writeType")
                                else "MUST_CACHE", ttl=ttl if ttl is not None else -1, ttl_action=action or "DELETE")
        return pb.file.CreateDirectoryPResponse()

    def CreateFile(self, req, ctx):
        o = req.options
        ttl, action = _ttl(o)
        fi = self.m.create_file(
            req.path, block_size=o.blockSizeBytes or None, recursive=o.recursive,
            mode=mode_from_pmode(o.mode) if o.HasField("mode") else None,
            replication_min=o.replicationMin, replication_max=o.replicationMax if o.HasField("replicationMax") else -1,
            replication_durable=o.replicationDurable if o.HasField("replicationDurable") else 1,
            write_type=enum_name(pb.file.WritePType, o.writeType) if o.HasField("writeType") else "CACHE_THROUGH",
            ttl=ttl if ttl is not None else -1, ttl_action=action or "DELETE",
            persistence_wait_ms=o.persistenceWaitTime)
        return pb.file.CreateFilePResponse(fileInfo=fi)

    def Free(self, req, ctx):
        self.m.free(req.path, recursive=req.options.recursive, forced=req.options.forced)
        return pb.file.FreePResponse()

    def GetFilePath(self, req, ctx):
        return pb.file.GetFilePathPResponse(path=self.m.get_file_path(req.fileId))

    def GetMountTable(self, req, ctx):
        r = pb.file.GetMountTablePResponse()
        for k, v in self.m.get_mount_table().items():
            r.mountPoints[k].CopyFrom(v)
        return r

    def GetSyncPathList(self, req, ctx):
        return pb.file.GetSyncPathListPResponse(syncPaths=[
            pb.file.SyncPointInfo(syncPointUri=p, syncStatus=2) for p in sorted(self.m.sync_points)])

    def GetNewBlockIdForFile(self, req, ctx):
        return pb.file.GetNewBlockIdForFilePResponse(id=self.m.get_new_block_id_for_file(req.path))

    def GetStatus(self, req, ctx):
        o = req.options
        lt = LOAD_TYPES.get(o.loadMetadataType, "ONCE") if o.HasField("loadMetadataType") else "ONCE"
        fi = self.m.get_status(req.path, load_metadata=lt, sync_interval_ms=_sync_interval(o),
                               access_mode=bits_from_proto(o.accessMode) if o.HasField("accessMode") else 4,
                               raw=True)
        # cached serialized FileInfo -> GetStatusPResponse{fileInfo=1} without a protobuf round trip
        return RawReply(length_delimited(0x0A, fi), pb.file.GetStatusPResponse)

    def ListStatus(self, req, ctx):
        o = req.options
        lt = LOAD_TYPES.get(o.loadMetadataType, "ONCE") if o.HasField("loadMetadataType") else "ONCE"
        bodies = self.m.list_status(req.path, recursive=o.recursive, load_metadata=lt,
                                    sync_interval_ms=_sync_interval(o), raw=True)
        for b in bodies:       # ListStatusPResponse{fileInfos=1*}, <= 10000 entries each
            yield RawReply(b, pb.file.ListStatusPResponse)

    def Mount(self, req, ctx):
        o = req.options
        self.m.mount(req.alluxioPath, req.ufsPath, read_only=o.readOnly, shared=o.shared,
                     properties=dict(o.properties))
        return pb.file.MountPResponse()

    def Remove(self, req, ctx):
        o = req.options
        self.m.delete(req.path, recursive=o.recursive, alluxio_only=o.alluxioOnly, unchecked=o.unchecked)
        return pb.file.DeletePResponse()

    def Rename(self, req, ctx):
        self.m.rename(req.path, req.dstPath, persist=req.options.persist)
        return pb.file.RenamePResponse()

    def ReverseResolve(self, req, ctx):
        return pb.file.ReverseResolvePResponse(alluxioPath=self.m.reverse_resolve(req.ufsUri))

    def ScheduleAsyncPersistence(self, req, ctx):
        self.m.schedule_async_persistence(req.path, req.options.persistenceWaitTime)
        return pb.file.ScheduleAsyncPersistencePResponse()

    def SetAcl(self, req, ctx):
        from ..security.acl import AclEntry
        entries = [AclEntry.from_pacl_entry(e) for e in req.entries]
        self.m.set_acl(req.path, enum_name(pb.file.SetAclAction, req.action), entries,
                       recursive=req.options.recursive)
        return pb.file.SetAclPResponse()

    def SetAttribute(self, req, ctx):
        o = req.options
        ttl, action = _ttl(o)
        self.m.set_attribute(
            req.path, pinned=o.pinned if o.HasField("pinned") else None, ttl=ttl, ttl_action=action,
            persisted=o.persisted if o.HasField("persisted") else None,
            owner=o.owner if o.HasField("owner") else None, group=o.group if o.HasField("group") else None,
            mode=mode_from_pmode(o.mode) if o.HasField("mode") else None, recursive=o.recursive,
            replication_min=o.replicationMin if o.HasField("replicationMin") else None,
            replication_max=o.replicationMax if o.HasField("replicationMax") else None,
            pinned_media=list(o.pinnedMedia) or None)
        return pb.file.SetAttributePResponse()

    def StartSync(self, req, ctx):
        self.m.start_sync(req.path)
        return pb.file.StartSyncPResponse()

    def StopSync(self, req, ctx):
        self.m.stop_sync(req.path)
        return pb.file.StopSyncPResponse()

    def Unmount(self, req, ctx):
        self.m.unmount(req.alluxioPath)
        return pb.file.UnmountPResponse()

    def UpdateMount(self, req, ctx):
        o = req.options
        self.m.update_mount(req.alluxioPath, read_only=o.readOnly if o.HasField("readOnly") else None,
                            shared=o.shared if o.HasField("shared") else None,
                            properties=dict(o.properties) if o.properties else None)
        return pb.file.UpdateMountPResponse()

    def UpdateUfsMode(self, req, ctx):
        self.m.update_ufs_mode(req.ufsPath, enum_name(pb.file.UfsPMode, req.options.ufsMode))
        return pb.file.UpdateUfsModePResponse()


class FileSystemMasterWorkerServiceHandler:
    def __init__(self, fsm):
        self.m = fsm

    def FileSystemHeartbeat(self, req, ctx):
        return pb.file.FileSystemHeartbeatPResponse(command=self.m.worker_heartbeat(req.workerId,
                                                                                  list(req.persistedFiles)))

    def GetFileInfo(self, req, ctx):
        return pb.file.GetFileInfoPResponse(fileInfo=self.m.get_file_info_by_id(req.fileId))

    def GetPinnedFileIds(self, req, ctx):
        return pb.file.GetPinnedFileIdsPResponse(pinnedFileIds=self.m.pinned_file_ids())

    def GetUfsInfo(self, req, ctx):
        return pb.file.GetUfsInfoPResponse(ufsInfo=self.m.get_ufs_info(req.mountId))


class BlockMasterClientServiceHandler:
    def __init__(self, bm):
        self.m = bm

    def GetBlockInfo(self, req, ctx):
        return pb.block.GetBlockInfoPResponse(blockInfo=self.m.block_info(req.blockId))

    def GetBlockMasterInfo(self, req, ctx):
        info = pb.block.BlockMasterInfo(capacityBytes=self.m.capacity_bytes(), usedBytes=self.m.used_bytes(),
                                        freeBytes=self.m.capacity_bytes() - self.m.used_bytes(),
                                        liveWorkerNum=self.m.worker_count(), lostWorkerNum=self.m.lost_worker_count())
        for k, v in self.m.capacity_on_tiers().items():
            info.capacityBytesOnTiers[k] = v
        for k, v in self.m.used_on_tiers().items():
            info.usedBytesOnTiers[k] = v
        return pb.block.GetBlockMasterInfoPResponse(blockMasterInfo=info)

    def GetCapacityBytes(self, req, ctx):
        return pb.block.GetCapacityBytesPResponse(bytes=self.m.capacity_bytes())

    def GetUsedBytes(self, req, ctx):
        return pb.block.GetUsedBytesPResponse(bytes=self.m.used_bytes())

    def GetWorkerInfoList(self, req, ctx):
        return pb.block.GetWorkerInfoListPResponse(workerInfos=self.m.worker_info_list())

    def GetWorkerReport(self, req, ctx):
        rng = enum_name(pb.block.WorkerRange, req.workerRange) if req.HasField("workerRange") else "ALL"
        infos = []
        if rng in ("ALL", "LIVE", "SPECIFIED"):
            infos += self.m.worker_info_list()
        if rng in ("ALL", "LOST", "SPECIFIED"):
            infos += self.m.lost_workers_info_list()
        if rng == "SPECIFIED" and req.addresses:
            want = set(req.addresses)
            infos = [w for w in infos if w.address.host in want]
        return pb.block.GetWorkerInfoListPResponse(workerInfos=infos)

    def GetWorkerLostStorage(self, req, ctx):
        return pb.block.GetWorkerLostStoragePResponse(workerLostStorageInfo=self.m.worker_lost_storage())


def _loc_blocks(entries) -> dict:
    out = {}
    for e in entries:
        out.setdefault((e.key.tierAlias, e.key.mediumType), []).extend(e.value.blockId)
    return out


class BlockMasterWorkerServiceHandler:
    def __init__(self, bm, metrics_master=None):
        self.m = bm
        self.metrics_master = metrics_master

    def BlockHeartbeat(self, req, ctx):
        added = _loc_blocks(req.addedBlocks)
        for tier, tl in req.addedBlocksOnTiers.items():
            added.setdefault((tier, ""), []).extend(tl.tiers)
        lost = {k: list(v.storage) for k, v in req.lostStorage.items()}
        if self.metrics_master is not None and req.options.metrics:
            self.metrics_master.worker_heartbeat(req.workerId, list(req.options.metrics))
        cmd, data = self.m.worker_heartbeat(req.workerId, dict(req.usedBytesOnTiers), list(req.removedBlockIds),
                                            added, lost_storage=lost)
        return pb.block.BlockHeartbeatPResponse(command=pb.grpc.Command(
            commandType=pb.grpc.CommandType.values_by_name[cmd].number, data=data))

    def CommitBlock(self, req, ctx):
        self.m.commit_block(req.workerId, req.usedBytesOnTier, req.tierAlias, req.mediumType, req.blockId, req.length)
        return pb.block.CommitBlockPResponse()

    def CommitBlocks(self, req, ctx):
        """Extension: a batch of CommitBlock reports in one call (bulk UFS ingest)."""
        self.m.commit_blocks(req.workerId, list(req.blockIds), list(req.lengths), list(req.tierIndex),
                             list(req.tiers), list(req.mediums), dict(req.usedBytesOnTiers))
        return pb.block.CommitBlocksPResponse()

    def CommitBlockInUfs(self, req, ctx):
        self.m.commit_block_in_ufs(req.blockId, req.length)
        return pb.block.CommitBlockInUfsPResponse()

    def GetWorkerId(self, req, ctx):
        return pb.block.GetWorkerIdPResponse(workerId=self.m.get_worker_id(req.workerNetAddress))

    def RegisterWorker(self, req, ctx):
        blocks = _loc_blocks(req.currentBlocks)
        for tier, tl in req.currentBlocksOnTiers.items():
            blocks.setdefault((tier, ""), []).extend(tl.tiers)
        self.m.worker_register(req.workerId, list(req.storageTiers), dict(req.totalBytesOnTiers),
                               dict(req.usedBytesOnTiers), blocks,
                               {k: list(v.storage) for k, v in req.lostStorage.items()})
        return pb.block.RegisterWorkerPResponse()


class ServiceVersionHandler:
    """Service versions; also advertises the native framed-RPC port (``nativeRpcPort``, an
    extension field Java clients ignore) through which our clients reach the same services."""
    VERSIONS = {i: 1 for i in range(17)}

    def __init__(self):
        self.native_port = 0

    def getServiceVersion(self, req, ctx):
        return pb.version.GetServiceVersionPResponse(version=self.VERSIONS.get(req.serviceType, 1),
                                                     nativeRpcPort=self.native_port)


class SaslHandler:
    """SIMPLE/NOSASL handshake: acknowledge the client's identity (reference
    SaslAuthenticationServiceHandler + PlainSaslServer for SIMPLE)."""

    def authenticate(self, request_iter, ctx):
        for msg in request_iter:
            yield pb.sasl.SaslMessage(messageType=1, clientId=msg.clientId, channelRef=msg.channelRef,
                                      authenticationScheme=msg.authenticationScheme)
            return
