"""Block worker data-plane service and block master services (package alluxio.grpc.block).

Contract source: core/transport/src/main/proto/grpc/block_worker.proto:13-170 and
grpc/block_master.proto:1-287.  The MI355X build adds *extension* messages (field numbers in
the 1000+ range on new messages only, never on existing ones) for the HIP-IPC short-circuit
handle and the RCCL transfer descriptors; reference clients never see them.
"""

SCHEMA = r"""
package alluxio.grpc.block
msg CheckRequest
msg CheckResponse
msg Chunk data=1:bytes
enum RequestType ALLUXIO_BLOCK=0 UFS_FILE=1 UFS_FALLBACK_BLOCK=2
msg ReadRequest block_id=1:i64 offset=2:i64 length=3:i64 promote=4:bool chunk_size=5:i64
    open_ufs_block_options=6:alluxio.proto.dataserver.OpenUfsBlockOptions offset_received=7:i64
    position_short=8:bool
msg ReadResponse chunk=1:Chunk
msg WriteRequestCommand type=1:RequestType id=2:i64 offset=3:i64 tier=4:i32 flush=5:bool
    create_ufs_file_options=6:alluxio.proto.dataserver.CreateUfsFileOptions
    create_ufs_block_options=7:alluxio.proto.dataserver.CreateUfsBlockOptions
    medium_type=8:str pin_on_create=9:bool space_to_reserve=10:i64 hold_for_append=20:bool
msg AppendBlock block_id=1:i64 length=2:i64
msg WriteRequest command=1:WriteRequestCommand|value chunk=2:Chunk|value append_block=20:AppendBlock|value
msg WriteResponse offset=1:i64
msg NativeWriteCommitRequest session_id=1:i64 block_id=2:i64 length=3:i64 pin=4:bool ufs_read=5:bool
    hold_for_append=6:bool
msg NativeCommitBatchRequest block_id=1:i64* length=2:i64* crc_piece=3:i64* crc=4:bytes* ufs_read=5:bool*
msg NativeCommitBatchResponse failed=1:i64* message=2:str
msg ResolveUfsMountRequest mount_id=1:i64 ufs_path=2:str
msg ResolveUfsMountResponse native=1:bool
msg ReadUfsRangeRequest mount_id=1:i64 ufs_path=2:str offset=3:i64 length=4:i64
msg ReadUfsRangeResponse data=1:bytes
msg AsyncCacheRequest block_id=1:i64 source_host=2:str source_port=3:i32
    open_ufs_block_options=4:alluxio.proto.dataserver.OpenUfsBlockOptions length=5:i64
msg AsyncCacheResponse
msg OpenLocalBlockRequest block_id=1:i64 promote=2:bool
msg OpenLocalBlockResponse path=1:str
msg CreateLocalBlockRequest block_id=1:i64 tier=3:i32 space_to_reserve=4:i64
    only_reserve_space=5:bool cleanup_on_failure=6:bool medium_type=7:str pin_on_create=8:bool
msg CreateLocalBlockResponse path=1:str
msg RemoveBlockRequest block_id=1:i64
msg RemoveBlockResponse
msg MoveBlockRequest block_id=1:i64 medium_type=2:str
msg MoveBlockResponse
msg ClearMetricsRequest
msg ClearMetricsResponse

# --- MI355X extensions: device short-circuit + RCCL transfer plane --------------------------
msg PageRun first_page=1:i64 num_pages=2:i64
msg DeviceBlockHandle block_id=1:i64 length=2:i64 page_size=3:i64 pages=4:i64*
    arena_ipc_handle=5:bytes arena_bytes=6:i64 device=7:i32 lock_id=8:i64 crc32c=9:u32*
    node_id=10:str pid=11:i32 arena_offset=12:i64 host_fd=13:i32 arena_kind=14:str
msg OpenDeviceBlockRequest block_id=1:i64 promote=2:bool session_id=3:i64 reader_gpu=4:i32
msg UnlockDeviceBlockRequest block_id=1:i64 lock_id=2:i64 session_id=3:i64
msg UnlockDeviceBlockResponse
msg OpenDeviceWriteRequest block_id=1:i64 length=2:i64 tier=3:i32 medium_type=4:str pin_on_create=5:bool
    session_id=6:i64
msg CommitDeviceWriteRequest block_id=1:i64 session_id=2:i64 length=3:i64 pin_on_create=4:bool abort=5:bool
    hold_for_append=6:bool
msg CommitDeviceWriteResponse
msg PeerTransferRequest block_id=1:i64 src_rank=2:i32 dst_rank=3:i32 offset=4:i64 length=5:i64
    tag=6:i64 src_address=7:str handle=8:DeviceBlockHandle
msg PeerTransferResponse ok=1:bool message=2:str
msg SessionHeartbeatRequest session_ids=1:i64*
msg SessionHeartbeatResponse unknown_session_ids=1:i64*

rpc BlockWorker ReadBlock *ReadRequest *ReadResponse
rpc BlockWorker WriteBlock *WriteRequest *WriteResponse
rpc BlockWorker OpenLocalBlock *OpenLocalBlockRequest *OpenLocalBlockResponse
rpc BlockWorker CreateLocalBlock *CreateLocalBlockRequest *CreateLocalBlockResponse
rpc BlockWorker AsyncCache AsyncCacheRequest AsyncCacheResponse
rpc BlockWorker RemoveBlock RemoveBlockRequest RemoveBlockResponse
rpc BlockWorker MoveBlock MoveBlockRequest MoveBlockResponse
rpc BlockWorker ClearMetrics ClearMetricsRequest ClearMetricsResponse
rpc BlockWorker OpenDeviceBlock OpenDeviceBlockRequest DeviceBlockHandle
rpc BlockWorker UnlockDeviceBlock UnlockDeviceBlockRequest UnlockDeviceBlockResponse
rpc BlockWorker PeerTransfer PeerTransferRequest PeerTransferResponse
rpc BlockWorker NativeWriteCommit NativeWriteCommitRequest WriteResponse
rpc BlockWorker NativeCommitBatch NativeCommitBatchRequest NativeCommitBatchResponse
rpc BlockWorker ResolveUfsMount ResolveUfsMountRequest ResolveUfsMountResponse
rpc BlockWorker ReadUfsRange ReadUfsRangeRequest ReadUfsRangeResponse
rpc BlockWorker OpenDeviceWrite OpenDeviceWriteRequest DeviceBlockHandle
rpc BlockWorker CommitDeviceWrite CommitDeviceWriteRequest CommitDeviceWriteResponse
rpc BlockWorker SessionHeartbeat SessionHeartbeatRequest SessionHeartbeatResponse

# --- block master ----------------------------------------------------------------------------
enum BlockMasterInfoField CAPACITY_BYTES=1 CAPACITY_BYTES_ON_TIERS=2 FREE_BYTES=3
    LIVE_WORKER_NUM=4 LOST_WORKER_NUM=5 USED_BYTES=6 USED_BYTES_ON_TIERS=7
msg BlockMasterInfo capacityBytes=1:i64 capacityBytesOnTiers=2:{str,i64} freeBytes=3:i64
    liveWorkerNum=4:i32 lostWorkerNum=5:i32 usedBytes=6:i64 usedBytesOnTiers=7:{str,i64}
msg GetBlockInfoPOptions
msg GetBlockInfoPRequest blockId=1:i64 options=2:GetBlockInfoPOptions
msg GetBlockInfoPResponse blockInfo=1:alluxio.grpc.BlockInfo
msg GetCapacityBytesPOptions
msg GetCapacityBytesPResponse bytes=1:i64
msg GetBlockMasterInfoPOptions filters=1:BlockMasterInfoField*
msg GetBlockMasterInfoPResponse blockMasterInfo=1:BlockMasterInfo
msg GetUsedBytesPOptions
msg GetUsedBytesPResponse bytes=1:i64
msg WorkerInfo id=1:i64 address=2:alluxio.grpc.WorkerNetAddress lastContactSec=3:i32 state=4:str
    capacityBytes=5:i64 usedBytes=6:i64 startTimeMs=7:i64 capacityBytesOnTiers=8:{str,i64}
    usedBytesOnTiers=9:{str,i64}
enum WorkerRange ALL=1 LIVE=2 LOST=3 SPECIFIED=4
enum WorkerInfoField ADDRESS=1 WORKER_CAPACITY_BYTES=2 WORKER_CAPACITY_BYTES_ON_TIERS=3 ID=4
    LAST_CONTACT_SEC=5 START_TIME_MS=6 STATE=7 WORKER_USED_BYTES=8 WORKER_USED_BYTES_ON_TIERS=9
msg GetWorkerReportPOptions addresses=1:str* fieldRanges=2:WorkerInfoField* workerRange=3:WorkerRange
msg GetWorkerInfoListPOptions
msg GetWorkerInfoListPResponse workerInfos=1:WorkerInfo*
msg StorageList storage=1:str*
msg WorkerLostStorageInfo address=1:alluxio.grpc.WorkerNetAddress lostStorage=2:{str,StorageList}
msg GetWorkerLostStoragePOptions
msg GetWorkerLostStoragePResponse workerLostStorageInfo=1:WorkerLostStorageInfo*
msg TierList tiers=1:i64*
msg BlockIdList blockId=1:i64*
msg BlockHeartbeatPOptions metrics=1:alluxio.grpc.Metric* capacityBytesOnTiers=2:{str,i64}
msg LocationBlockIdListEntry key=1:alluxio.grpc.BlockStoreLocationProto value=2:BlockIdList
msg BlockHeartbeatPRequest workerId=1:i64 usedBytesOnTiers=2:{str,i64} removedBlockIds=3:i64*
    addedBlocksOnTiers=4:{str,TierList} options=5:BlockHeartbeatPOptions
    lostStorage=6:{str,StorageList} addedBlocks=7:LocationBlockIdListEntry*
msg BlockHeartbeatPResponse command=1:alluxio.grpc.Command
msg CommitBlockPOptions
msg CommitBlockPRequest workerId=1:i64 usedBytesOnTier=2:i64 tierAlias=3:str blockId=4:i64
    length=5:i64 options=6:CommitBlockPOptions mediumType=7:str
msg CommitBlockPResponse
msg CommitBlocksPRequest workerId=1001:i64 blockIds=1002:i64* lengths=1003:i64* tierIndex=1004:i32*
    tiers=1005:str* mediums=1006:str* usedBytesOnTiers=1007:{str,i64}
msg CommitBlocksPResponse
msg CommitBlockInUfsPOptions
msg CommitBlockInUfsPRequest blockId=1:i64 length=2:i64 options=3:CommitBlockInUfsPOptions
msg CommitBlockInUfsPResponse
msg GetWorkerIdPOptions
msg GetWorkerIdPRequest workerNetAddress=1:alluxio.grpc.WorkerNetAddress options=2:GetWorkerIdPOptions
msg GetWorkerIdPResponse workerId=1:i64
msg RegisterWorkerPOptions configs=1:alluxio.grpc.ConfigProperty*
msg RegisterWorkerPRequest workerId=1:i64 storageTiers=2:str* totalBytesOnTiers=3:{str,i64}
    usedBytesOnTiers=4:{str,i64} currentBlocksOnTiers=5:{str,TierList}
    options=6:RegisterWorkerPOptions lostStorage=7:{str,StorageList}
    currentBlocks=8:LocationBlockIdListEntry*
msg RegisterWorkerPResponse

rpc BlockMasterClientService GetBlockInfo GetBlockInfoPRequest GetBlockInfoPResponse
rpc BlockMasterClientService GetBlockMasterInfo GetBlockMasterInfoPOptions GetBlockMasterInfoPResponse
rpc BlockMasterClientService GetCapacityBytes GetCapacityBytesPOptions GetCapacityBytesPResponse
rpc BlockMasterClientService GetUsedBytes GetUsedBytesPOptions GetUsedBytesPResponse
rpc BlockMasterClientService GetWorkerInfoList GetWorkerInfoListPOptions GetWorkerInfoListPResponse
rpc BlockMasterClientService GetWorkerReport GetWorkerReportPOptions GetWorkerInfoListPResponse
rpc BlockMasterClientService GetWorkerLostStorage GetWorkerLostStoragePOptions GetWorkerLostStoragePResponse
rpc BlockMasterWorkerService BlockHeartbeat BlockHeartbeatPRequest BlockHeartbeatPResponse
rpc BlockMasterWorkerService CommitBlock CommitBlockPRequest CommitBlockPResponse
rpc BlockMasterWorkerService CommitBlockInUfs CommitBlockInUfsPRequest CommitBlockInUfsPResponse
rpc BlockMasterWorkerService CommitBlocks CommitBlocksPRequest CommitBlocksPResponse
rpc BlockMasterWorkerService GetWorkerId GetWorkerIdPRequest GetWorkerIdPResponse
rpc BlockMasterWorkerService RegisterWorker RegisterWorkerPRequest RegisterWorkerPResponse
"""
