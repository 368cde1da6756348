"""File-system master services (package alluxio.grpc.file).

Contract source: core/transport/src/main/proto/grpc/file_system_master.proto:1-676 (23 client
RPCs at :470-590, worker/job services at :639-675).
"""

SCHEMA = r"""
package alluxio.grpc.file
enum WritePType MUST_CACHE=1 TRY_CACHE=2 CACHE_THROUGH=3 THROUGH=4 ASYNC_THROUGH=5 NONE=6
enum ReadPType NO_CACHE=1 CACHE=2 CACHE_PROMOTE=3
enum LoadMetadataPType NEVER=0 ONCE=1 ALWAYS=2
msg FileSystemMasterCommonPOptions syncIntervalMs=1:i64 ttl=2:i64 ttlAction=3:alluxio.grpc.TtlAction
msg CheckConsistencyPOptions commonOptions=1:FileSystemMasterCommonPOptions
msg CheckConsistencyPRequest path=1:str options=2:CheckConsistencyPOptions
msg CheckConsistencyPResponse inconsistentPaths=1:str*
msg ScheduleAsyncPersistencePOptions commonOptions=1:FileSystemMasterCommonPOptions
    persistenceWaitTime=2:i64
msg CompleteFilePOptions ufsLength=1:i64 asyncPersistOptions=2:ScheduleAsyncPersistencePOptions
    commonOptions=3:FileSystemMasterCommonPOptions
msg CompleteFilePRequest path=1:str options=2:CompleteFilePOptions
msg CompleteFilePResponse
msg OpenFilePOptions readType=1:ReadPType maxUfsReadConcurrency=2:i32
    commonOptions=3:FileSystemMasterCommonPOptions updateLastAccessTime=4:bool@true
msg CreateDirectoryPOptions recursive=1:bool allowExists=2:bool mode=3:alluxio.grpc.PMode
    writeType=4:WritePType commonOptions=5:FileSystemMasterCommonPOptions
msg CreateDirectoryPRequest path=1:str options=2:CreateDirectoryPOptions
msg CreateDirectoryPResponse
msg CreateFilePOptions blockSizeBytes=1:i64 recursive=2:bool mode=3:alluxio.grpc.PMode
    replicationMax=4:i32 replicationMin=5:i32 replicationDurable=6:i32 writeTier=7:i32
    writeType=8:WritePType commonOptions=9:FileSystemMasterCommonPOptions persistenceWaitTime=10:i64
msg CreateFilePRequest path=1:str options=2:CreateFilePOptions
msg CreateFilePResponse fileInfo=1:FileInfo
msg DeletePOptions recursive=1:bool alluxioOnly=2:bool unchecked=3:bool
    commonOptions=4:FileSystemMasterCommonPOptions
msg DeletePRequest path=1:str options=2:DeletePOptions
msg DeletePResponse
msg FreePOptions recursive=1:bool forced=2:bool commonOptions=3:FileSystemMasterCommonPOptions
msg FreePRequest path=1:str options=2:FreePOptions
msg FreePResponse
msg GetNewBlockIdForFilePOptions commonOptions=1:FileSystemMasterCommonPOptions
msg GetNewBlockIdForFilePRequest path=1:str options=2:GetNewBlockIdForFilePOptions
msg GetNewBlockIdForFilePResponse id=1:i64
msg GetStatusPOptions loadMetadataType=1:LoadMetadataPType commonOptions=2:FileSystemMasterCommonPOptions
    accessMode=3:alluxio.grpc.Bits updateTimestamps=4:bool@true
msg GetStatusPRequest path=1:str options=2:GetStatusPOptions
msg GetStatusPResponse fileInfo=1:FileInfo
msg ExistsPOptions loadMetadataType=1:LoadMetadataPType commonOptions=2:FileSystemMasterCommonPOptions
enum SyncPointStatus Not_Initially_Synced=0 Syncing=1 Initially_Synced=2
msg SyncPointInfo syncPointUri=1:str syncStatus=2:SyncPointStatus
msg GetSyncPathListPRequest
msg GetSyncPathListPResponse syncPaths=1:SyncPointInfo*
msg ListStatusPOptions loadDirectChildren=1:bool loadMetadataType=2:LoadMetadataPType
    commonOptions=3:FileSystemMasterCommonPOptions recursive=4:bool resultsRequired=5:bool
msg ListStatusPRequest path=1:str options=2:ListStatusPOptions
msg ListStatusPResponse fileInfos=1:FileInfo*
msg LoadMetadataPOptions recursive=1:bool createAncestors=2:bool
    loadDescendantType=3:alluxio.grpc.fscommon.LoadDescendantPType
    commonOptions=4:FileSystemMasterCommonPOptions
enum PAclEntryType Owner=0 NamedUser=1 OwningGroup=2 NamedGroup=3 Mask=4 Other=5
enum PAclAction Read=0 Write=1 Execute=2
msg PAclEntry type=1:PAclEntryType subject=2:str actions=3:PAclAction* isDefault=4:bool
msg PAcl owner=1:str owningGroup=2:str entries=3:PAclEntry* mode=4:i32 isDefault=5:bool
    isDefaultEmpty=6:bool
msg FileBlockInfo blockInfo=1:alluxio.grpc.BlockInfo offset=2:i64
    ufsLocations=3:alluxio.grpc.WorkerNetAddress* ufsStringLocations=4:str*
msg FileInfo fileId=1:i64 name=2:str path=3:str ufsPath=4:str length=5:i64 blockSizeBytes=6:i64
    creationTimeMs=7:i64 completed=8:bool folder=9:bool pinned=10:bool cacheable=11:bool
    persisted=12:bool blockIds=13:i64* lastModificationTimeMs=14:i64 ttl=15:i64 owner=16:str
    group=17:str mode=18:i32 persistenceState=19:str mountPoint=20:bool
    fileBlockInfos=21:FileBlockInfo* ttlAction=22:alluxio.grpc.TtlAction mountId=23:i64
    inAlluxioPercentage=24:i32 inMemoryPercentage=25:i32 ufsFingerprint=26:str acl=27:PAcl
    defaultAcl=28:PAcl replicationMax=29:i32 replicationMin=30:i32 lastAccessTimeMs=31:i64
    xattr=32:{str,bytes}
msg GetFilePathPRequest fileId=1:i64
msg GetFilePathPResponse path=1:str
msg MountPOptions readOnly=1:bool properties=2:{str,str} shared=3:bool
    commonOptions=4:FileSystemMasterCommonPOptions
msg MountPRequest alluxioPath=1:str ufsPath=2:str options=3:MountPOptions
msg MountPResponse
msg MountPointInfo ufsUri=1:str ufsType=2:str ufsCapacityBytes=3:i64@-1 ufsUsedBytes=4:i64@-1
    readOnly=5:bool properties=6:{str,str} shared=7:bool
msg GetMountTablePRequest
msg GetMountTablePResponse mountPoints=1:{str,MountPointInfo}
msg PersistFile fileId=1:i64 blockIds=2:i64*
msg PersistCommandOptions persistFiles=1:PersistFile*
msg FileSystemCommandOptions persistOptions=1:PersistCommandOptions
msg FileSystemCommand commandType=1:alluxio.grpc.CommandType commandOptions=2:FileSystemCommandOptions
msg RenamePOptions commonOptions=1:FileSystemMasterCommonPOptions persist=2:bool
msg RenamePRequest path=1:str dstPath=2:str options=3:RenamePOptions
msg RenamePResponse
msg ReverseResolvePRequest ufsUri=1:str
msg ReverseResolvePResponse alluxioPath=1:str
msg SetAttributePOptions pinned=1:bool persisted=2:bool owner=3:str group=4:str
    mode=5:alluxio.grpc.PMode recursive=6:bool replicationMax=7:i32 replicationMin=8:i32
    commonOptions=9:FileSystemMasterCommonPOptions pinnedMedia=10:str*
msg SetAttributePRequest path=1:str options=2:SetAttributePOptions
msg SetAttributePResponse
enum SetAclAction REPLACE=0 MODIFY=1 REMOVE=2 REMOVE_ALL=3 REMOVE_DEFAULT=4
msg SetAclPOptions commonOptions=1:FileSystemMasterCommonPOptions recursive=2:bool
msg SetAclPRequest path=1:str action=2:SetAclAction entries=3:PAclEntry* options=4:SetAclPOptions
msg SetAclPResponse
msg ScheduleAsyncPersistencePRequest path=1:str options=2:ScheduleAsyncPersistencePOptions
msg ScheduleAsyncPersistencePResponse
msg StartSyncPOptions commonOptions=1:FileSystemMasterCommonPOptions
msg StartSyncPRequest path=1:str options=2:StartSyncPOptions
msg StartSyncPResponse
msg StopSyncPOptions commonOptions=1:FileSystemMasterCommonPOptions
msg StopSyncPRequest path=1:str options=2:StopSyncPOptions
msg StopSyncPResponse
msg UnmountPOptions commonOptions=1:FileSystemMasterCommonPOptions
msg UnmountPRequest alluxioPath=1:str options=2:UnmountPOptions
msg UnmountPResponse
msg UfsInfo uri=1:str properties=2:MountPOptions
enum UfsPMode NO_ACCESS=1 READ_ONLY=2 READ_WRITE=3
msg UpdateMountPRequest alluxioPath=1:str options=3:MountPOptions
msg UpdateMountPResponse
msg UpdateUfsModePOptions ufsMode=1:UfsPMode
msg UpdateUfsModePRequest ufsPath=1:str options=2:UpdateUfsModePOptions
msg UpdateUfsModePResponse
msg FileSystemHeartbeatPOptions persistedFileFingerprints=1:str*
msg FileSystemHeartbeatPRequest workerId=1:i64 persistedFiles=2:i64* options=3:FileSystemHeartbeatPOptions
msg FileSystemHeartbeatPResponse command=1:FileSystemCommand
msg GetFileInfoPOptions
msg GetFileInfoPRequest fileId=1:i64 options=2:GetFileInfoPOptions
msg GetFileInfoPResponse fileInfo=1:FileInfo
msg GetPinnedFileIdsPOptions
msg GetPinnedFileIdsPRequest options=1:GetPinnedFileIdsPOptions
msg GetPinnedFileIdsPResponse pinnedFileIds=1:i64*
msg GetUfsInfoPOptions
msg GetUfsInfoPRequest mountId=1:i64 options=2:GetUfsInfoPOptions
msg GetUfsInfoPResponse ufsInfo=1:UfsInfo

rpc FileSystemMasterClientService CheckConsistency CheckConsistencyPRequest CheckConsistencyPResponse
rpc FileSystemMasterClientService CompleteFile CompleteFilePRequest CompleteFilePResponse
rpc FileSystemMasterClientService CreateDirectory CreateDirectoryPRequest CreateDirectoryPResponse
rpc FileSystemMasterClientService CreateFile CreateFilePRequest CreateFilePResponse
rpc FileSystemMasterClientService Free FreePRequest FreePResponse
rpc FileSystemMasterClientService GetFilePath GetFilePathPRequest GetFilePathPResponse
rpc FileSystemMasterClientService GetMountTable GetMountTablePRequest GetMountTablePResponse
rpc FileSystemMasterClientService GetSyncPathList GetSyncPathListPRequest GetSyncPathListPResponse
rpc FileSystemMasterClientService GetNewBlockIdForFile GetNewBlockIdForFilePRequest GetNewBlockIdForFilePResponse
rpc FileSystemMasterClientService GetStatus GetStatusPRequest GetStatusPResponse
rpc FileSystemMasterClientService ListStatus ListStatusPRequest *ListStatusPResponse
rpc FileSystemMasterClientService Mount MountPRequest MountPResponse
rpc FileSystemMasterClientService Remove DeletePRequest DeletePResponse
rpc FileSystemMasterClientService Rename RenamePRequest RenamePResponse
rpc FileSystemMasterClientService ReverseResolve ReverseResolvePRequest ReverseResolvePResponse
rpc FileSystemMasterClientService ScheduleAsyncPersistence ScheduleAsyncPersistencePRequest ScheduleAsyncPersistencePResponse
rpc FileSystemMasterClientService SetAcl SetAclPRequest SetAclPResponse
rpc FileSystemMasterClientService SetAttribute SetAttributePRequest SetAttributePResponse
rpc FileSystemMasterClientService StartSync StartSyncPRequest StartSyncPResponse
rpc FileSystemMasterClientService StopSync StopSyncPRequest StopSyncPResponse
rpc FileSystemMasterClientService Unmount UnmountPRequest UnmountPResponse
rpc FileSystemMasterClientService UpdateMount UpdateMountPRequest UpdateMountPResponse
rpc FileSystemMasterClientService UpdateUfsMode UpdateUfsModePRequest UpdateUfsModePResponse
rpc FileSystemMasterWorkerService FileSystemHeartbeat FileSystemHeartbeatPRequest FileSystemHeartbeatPResponse
rpc FileSystemMasterWorkerService GetFileInfo GetFileInfoPRequest GetFileInfoPResponse
rpc FileSystemMasterWorkerService GetPinnedFileIds GetPinnedFileIdsPRequest GetPinnedFileIdsPResponse
rpc FileSystemMasterWorkerService GetUfsInfo GetUfsInfoPRequest GetUfsInfoPResponse
rpc FileSystemMasterJobService GetFileInfo GetFileInfoPRequest GetFileInfoPResponse
rpc FileSystemMasterJobService GetUfsInfo GetUfsInfoPRequest GetUfsInfoPResponse
"""
