"""Meta master, job master and journal master services.

Contract source: core/transport/src/main/proto/grpc/meta_master.proto:1-266,
grpc/job_master.proto:1-231, grpc/journal_master.proto:1-58, grpc/raft_journal.proto:67-77.
"""

SCHEMA = r"""
package alluxio.grpc.meta
msg ConfigProperties properties=1:alluxio.grpc.ConfigProperty*
msg GetConfigurationPOptions rawValue=1:bool ignoreClusterConf=2:bool ignorePathConf=3:bool
msg GetConfigurationPResponse clusterConfigs=1:alluxio.grpc.ConfigProperty*
    pathConfigs=2:{str,ConfigProperties} clusterConfigHash=3:str pathConfigHash=4:str
enum ConfigStatus PASSED=1 WARN=2 FAILED=3
enum Scope MASTER=1 WORKER=2 CLIENT=4 SERVER=3 ALL=7 NONE=0
msg InconsistentPropertyValues values=1:str*
msg InconsistentProperty name=1:str values=2:{str,InconsistentPropertyValues}
msg InconsistentProperties properties=1:InconsistentProperty*
msg ConfigCheckReport errors=1:{str,InconsistentProperties} warns=2:{str,InconsistentProperties}
    status=3:ConfigStatus
msg GetConfigReportPOptions
msg GetConfigReportPResponse report=1:ConfigCheckReport
msg MasterInfo leaderMasterAddress=1:str masterAddresses=2:alluxio.grpc.NetAddress* rpcPort=3:i32
    safeMode=4:bool startTimeMs=5:i64 upTimeMs=6:i64 version=7:str webPort=8:i32
    workerAddresses=9:alluxio.grpc.NetAddress* zookeeperAddresses=10:str*
enum MasterInfoField LEADER_MASTER_ADDRESS=0 MASTER_ADDRESSES=1 RPC_PORT=2 SAFE_MODE=3
    START_TIME_MS=4 UP_TIME_MS=5 VERSION=6 WEB_PORT=7 WORKER_ADDRESSES=8 ZOOKEEPER_ADDRESSES=9
msg GetMasterInfoPOptions filter=1:MasterInfoField*
msg GetMasterInfoPResponse masterInfo=1:MasterInfo
msg CheckpointPOptions
msg CheckpointPResponse masterHostname=1:str
enum BackupState None=1 Initiating=2 Transitioning=3 Running=4 Completed=5 Failed=6
msg BackupPOptions localFileSystem=1:bool runAsync=2:bool allowLeader=3:bool
msg BackupPRequest options=1:BackupPOptions targetDirectory=2:str
msg BackupPStatus backupId=1:str backupState=2:BackupState backupHost=3:str backupUri=4:str
    entryCount=5:i64 backupError=6:bytes
msg BackupStatusPRequest backupId=1:str
msg SetPathConfigurationPOptions
msg SetPathConfigurationPRequest path=1:str properties=2:{str,str} options=3:SetPathConfigurationPOptions
msg SetPathConfigurationPResponse
msg RemovePathConfigurationPOptions
msg RemovePathConfigurationPRequest path=1:str keys=2:str* options=3:RemovePathConfigurationPOptions
msg RemovePathConfigurationPResponse
msg GetConfigHashPOptions
msg GetConfigHashPResponse clusterConfigHash=1:str pathConfigHash=2:str
msg GetMasterIdPOptions
msg GetMasterIdPRequest masterAddress=1:alluxio.grpc.NetAddress options=2:GetMasterIdPOptions
msg GetMasterIdPResponse masterId=1:i64
enum MetaCommand MetaCommand_Unknown=0 MetaCommand_Nothing=1 MetaCommand_Register=2
msg RegisterMasterPOptions configs=1:alluxio.grpc.ConfigProperty*
msg RegisterMasterPRequest masterId=1:i64 options=2:RegisterMasterPOptions
msg RegisterMasterPResponse
msg MasterHeartbeatPOptions
msg MasterHeartbeatPRequest masterId=1:i64 options=2:MasterHeartbeatPOptions
msg MasterHeartbeatPResponse command=1:MetaCommand
msg JournalSequence master=1:str sequence=2:i64
msg BackupSuspendPRequest
msg BackupSuspendPResponse
msg BackupDelegatePRequest backupId=1:str request=2:BackupPRequest sequences=3:JournalSequence*
msg BackupDelegatePResponse
rpc BackupWorkerService SuspendJournals BackupSuspendPRequest BackupSuspendPResponse
rpc BackupWorkerService DelegateBackup BackupDelegatePRequest BackupDelegatePResponse
rpc BackupWorkerService GetBackupStatus BackupStatusPRequest BackupPStatus
rpc MetaMasterClientService Backup BackupPRequest BackupPStatus
rpc MetaMasterClientService GetBackupStatus BackupStatusPRequest BackupPStatus
rpc MetaMasterClientService GetConfigReport GetConfigReportPOptions GetConfigReportPResponse
rpc MetaMasterClientService GetMasterInfo GetMasterInfoPOptions GetMasterInfoPResponse
rpc MetaMasterClientService Checkpoint CheckpointPOptions CheckpointPResponse
rpc MetaMasterConfigurationService GetConfiguration GetConfigurationPOptions GetConfigurationPResponse
rpc MetaMasterConfigurationService SetPathConfiguration SetPathConfigurationPRequest SetPathConfigurationPResponse
rpc MetaMasterConfigurationService RemovePathConfiguration RemovePathConfigurationPRequest RemovePathConfigurationPResponse
rpc MetaMasterConfigurationService GetConfigHash GetConfigHashPOptions GetConfigHashPResponse
rpc MetaMasterMasterService GetMasterId GetMasterIdPRequest GetMasterIdPResponse
rpc MetaMasterMasterService RegisterMaster RegisterMasterPRequest RegisterMasterPResponse
rpc MetaMasterMasterService MasterHeartbeat MasterHeartbeatPRequest MasterHeartbeatPResponse

package alluxio.grpc.job
enum Status UNKNOWN=0 CREATED=1 CANCELED=2 FAILED=3 RUNNING=4 COMPLETED=5
enum JobType PLAN=1 TASK=2 WORKFLOW=3
msg JobUnused
msg JobInfo id=1:i64 errorMessage=2:str unused0=3:JobUnused* status=4:Status unused1=5:str
    lastUpdated=6:i64 name=7:str type=8:JobType result=9:bytes parentId=10:i64 children=11:JobInfo*
    workerHost=12:str description=13:str affectedPaths=14:str* errorType=15:str
msg StatusSummary status=1:Status count=2:i64
msg JobServiceSummary summaryPerStatus=1:StatusSummary* recentActivities=2:JobInfo*
    recentFailures=3:JobInfo* longestRunning=4:JobInfo*
msg JobWorkerHealth workerId=1:i64 loadAverage=2:f64* lastUpdated=3:i64 hostname=4:str
    taskPoolSize=5:i32 numActiveTasks=6:i32 unfinishedTasks=7:i32
msg RunTaskCommand jobId=1:i64 taskId=2:i64 jobConfig=3:bytes taskArgs=4:bytes
msg RegisterCommand
msg SetTaskPoolSizeCommand taskPoolSize=1:i32
msg CancelTaskCommand jobId=1:i64 taskId=2:i64
msg JobCommand runTaskCommand=1:RunTaskCommand cancelTaskCommand=2:CancelTaskCommand
    registerCommand=3:RegisterCommand setTaskPoolSizeCommand=4:SetTaskPoolSizeCommand
msg CancelPOptions
msg CancelPRequest jobId=1:i64 options=2:CancelPOptions
msg CancelPResponse
msg GetJobStatusPOptions
msg GetJobStatusPRequest jobId=1:i64 options=2:GetJobStatusPOptions
msg GetJobStatusPResponse jobInfo=1:JobInfo
msg GetJobStatusDetailedPOptions
msg GetJobStatusDetailedPRequest jobId=1:i64 options=2:GetJobStatusDetailedPOptions
msg GetJobStatusDetailedPResponse jobInfo=1:JobInfo
msg ListAllPOptions
msg ListAllPRequest options=1:ListAllPOptions
msg ListAllPResponse jobIds=1:i64* jobInfos=2:JobInfo*
msg RunPOptions
msg RunPRequest jobConfig=1:bytes options=2:RunPOptions
msg RunPResponse jobId=1:i64
msg GetJobServiceSummaryPOptions
msg GetJobServiceSummaryPRequest options=1:GetJobServiceSummaryPOptions
msg GetJobServiceSummaryPResponse summary=1:JobServiceSummary
msg GetAllWorkerHealthPOptions
msg GetAllWorkerHealthPRequest options=1:GetAllWorkerHealthPOptions
msg GetAllWorkerHealthPResponse workerHealths=1:JobWorkerHealth*
msg JobHeartbeatPOptions
msg JobHeartbeatPRequest jobWorkerHealth=1:JobWorkerHealth taskInfos=2:JobInfo*
    options=3:JobHeartbeatPOptions
msg JobHeartbeatPResponse commands=1:JobCommand*
msg RegisterJobWorkerPOptions
msg RegisterJobWorkerPRequest workerNetAddress=1:alluxio.grpc.WorkerNetAddress
    options=2:RegisterJobWorkerPOptions
msg RegisterJobWorkerPResponse id=1:i64
rpc JobMasterClientService Cancel CancelPRequest CancelPResponse
rpc JobMasterClientService GetJobStatus GetJobStatusPRequest GetJobStatusPResponse
rpc JobMasterClientService GetJobStatusDetailed GetJobStatusDetailedPRequest GetJobStatusDetailedPResponse
rpc JobMasterClientService GetJobServiceSummary GetJobServiceSummaryPRequest GetJobServiceSummaryPResponse
rpc JobMasterClientService ListAll ListAllPRequest ListAllPResponse
rpc JobMasterClientService Run RunPRequest RunPResponse
rpc JobMasterClientService GetAllWorkerHealth GetAllWorkerHealthPRequest GetAllWorkerHealthPResponse
rpc JobMasterWorkerService Heartbeat JobHeartbeatPRequest JobHeartbeatPResponse
rpc JobMasterWorkerService RegisterJobWorker RegisterJobWorkerPRequest RegisterJobWorkerPResponse

package alluxio.grpc.journal
enum QuorumServerState AVAILABLE=1 UNAVAILABLE=2
enum JournalDomain MASTER=1 JOB_MASTER=2
msg QuorumServerInfo serverAddress=1:alluxio.grpc.NetAddress serverState=2:QuorumServerState
msg GetQuorumInfoPOptions
msg GetQuorumInfoPRequest options=1:GetQuorumInfoPOptions
msg GetQuorumInfoPResponse domain=1:JournalDomain serverInfo=2:QuorumServerInfo*
msg RemoveQuorumServerPOptions
msg RemoveQuorumServerPRequest options=1:RemoveQuorumServerPOptions
    serverAddress=2:alluxio.grpc.NetAddress
msg RemoveQuorumServerPResponse
rpc JournalMasterClientService GetQuorumInfo GetQuorumInfoPRequest GetQuorumInfoPResponse
rpc JournalMasterClientService RemoveQuorumServer RemoveQuorumServerPRequest RemoveQuorumServerPResponse
"""
