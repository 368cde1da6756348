"""Shared wire types: alluxio.grpc (common), shared ACLs, dataserver options, version, SASL.

Field numbers/labels follow the reference contract in core/transport/src/main/proto/
(grpc/common.proto, proto/shared/acl.proto, proto/dataserver/protocol.proto,
proto/dataserver/status.proto, grpc/version.proto, grpc/sasl_server.proto, grpc/fscommon.proto).
"""

SCHEMA = r"""
package alluxio.grpc
enum Bits NONE=1 EXECUTE=2 WRITE=3 WRITE_EXECUTE=4 READ=5 READ_EXECUTE=6 READ_WRITE=7 ALL=8
enum MetricType GAUGE=0 COUNTER=1 METER=2 TIMER=3
enum CommandType Unknown=0 Nothing=1 Register=2 Free=3 Delete=4 Persist=5
enum TtlAction DELETE=0 FREE=1
msg PMode ownerBits=1:Bits! groupBits=2:Bits! otherBits=3:Bits!
msg LocalityTier tierName=1:str value=2:str
msg TieredIdentity tiers=1:LocalityTier*
msg NetAddress host=1:str rpcPort=2:i32
msg WorkerNetAddress host=1:str rpcPort=2:i32 dataPort=3:i32 webPort=4:i32 domainSocketPath=5:str
    tieredIdentity=6:TieredIdentity containerHost=7:str
msg BlockLocation workerId=1:i64 workerAddress=2:WorkerNetAddress tierAlias=3:str mediumType=4:str
msg BlockInfo blockId=1:i64 length=2:i64 locations=3:BlockLocation*
msg Metric instance=1:str source=2:str name=3:str value=4:f64 metricType=5:MetricType!
    tags=6:{str,str}
msg ConfigProperty name=1:str source=2:str value=3:str
msg Command commandType=1:CommandType data=2:i64*
msg BlockStoreLocationProto tierAlias=1:str mediumType=2:str

package alluxio.grpc.fscommon
enum LoadDescendantPType NONE=0 ONE=1 ALL=2

package alluxio.proto.shared
enum AclAction READ=0 WRITE=1 EXECUTE=2
enum AclEntryType OWNER=0 NAMED_USER=1 OWNING_GROUP=2 NAMED_GROUP=3 MASK=4 OTHER=5
msg AclActions actions=1:AclAction*
msg AclEntry type=1:AclEntryType subject=2:str actions=3:AclAction* isDefault=4:bool
msg NamedAclActions name=1:str actions=2:AclActions
msg AccessControlList owningUser=1:str owningGroup=2:str userActions=3:NamedAclActions*
    groupActions=4:NamedAclActions* maskActions=5:AclActions otherActions=6:AclActions
    isDefault=7:bool isEmpty=8:bool

package alluxio.proto.status
enum PStatus OK=0 CANCELLED=1 UNKNOWN=2 INVALID_ARGUMENT=3 DEADLINE_EXCEEDED=4 NOT_FOUND=5
    ALREADY_EXISTS=6 PERMISSION_DENIED=7 UNAUTHENTICATED=16 RESOURCE_EXHAUSTED=8
    FAILED_PRECONDITION=9 ABORTED=10 OUT_OF_RANGE=11 UNIMPLEMENTED=12 INTERNAL=13
    UNAVAILABLE=14 DATA_LOSS=15

package alluxio.proto.dataserver
msg OpenUfsBlockOptions ufs_path=1:str offset_in_file=2:i64 block_size=3:i64
    maxUfsReadConcurrency=4:i32 mountId=5:i64 no_cache=6:bool user=7:str block_in_ufs_tier=8:bool
msg CreateUfsFileOptions ufs_path=1:str owner=2:str group=3:str mode=4:i32 mount_id=5:i64
    acl=6:alluxio.proto.shared.AccessControlList
msg CreateUfsBlockOptions bytes_in_block_store=1:i64 mount_id=2:i64 fallback=3:bool
msg Response status=1:alluxio.proto.status.PStatus message=2:str

package alluxio.grpc.version
enum ServiceType UNKNOWN_SERVICE=0 FILE_SYSTEM_MASTER_CLIENT_SERVICE=1
    FILE_SYSTEM_MASTER_WORKER_SERVICE=2 FILE_SYSTEM_MASTER_JOB_SERVICE=3
    BLOCK_MASTER_CLIENT_SERVICE=4 BLOCK_MASTER_WORKER_SERVICE=5 META_MASTER_CONFIG_SERVICE=6
    META_MASTER_CLIENT_SERVICE=7 META_MASTER_MASTER_SERVICE=8 METRICS_MASTER_CLIENT_SERVICE=9
    JOB_MASTER_CLIENT_SERVICE=10 JOB_MASTER_WORKER_SERVICE=11 FILE_SYSTEM_WORKER_WORKER_SERVICE=12
    JOURNAL_MASTER_CLIENT_SERVICE=13 TABLE_MASTER_CLIENT_SERVICE=14
    META_MASTER_BACKUP_MESSAGING_SERVICE=15 RAFT_JOURNAL_SERVICE=16
msg GetServiceVersionPRequest serviceType=1:ServiceType
msg GetServiceVersionPResponse version=1:i64 nativeRpcPort=1000:i32
rpc ServiceVersionClientService getServiceVersion GetServiceVersionPRequest GetServiceVersionPResponse

package alluxio.grpc.sasl
enum SaslMessageType CHALLENGE=0 SUCCESS=1
enum ChannelAuthenticationScheme NOSASL=0 SIMPLE=1 CUSTOM=2
msg SaslMessage messageType=1:SaslMessageType message=2:bytes clientId=3:str
    authenticationScheme=4:ChannelAuthenticationScheme channelRef=5:str
rpc SaslAuthenticationService authenticate *SaslMessage *SaslMessage

package alluxio.proto.client
msg PPageStoreCommonOptions pageSize=1:i64 cacheSize=2:i64 alluxioVersion=3:str
msg PRocksPageStoreOptions commonOptions=1:PPageStoreCommonOptions
"""
