"""Journal entry schema (package alluxio.proto.journal) + metastore value encodings.

Contract source: core/transport/src/main/proto/proto/journal/{journal,file,block,meta,table}.proto
and proto/meta/{block,inode_meta}.proto.  ``JournalEntry`` is the one-of-many wrapper whose
length-delimited encoding is the UFS-journal log/checkpoint format (journal.proto:20-61).
"""

SCHEMA = r"""
package alluxio.proto.journal
msg StringPairEntry key=1:str value=2:str
msg ActiveSyncTxIdEntry mount_id=1:i64 tx_id=2:i64
msg AddSyncPointEntry syncpoint_path=1:str mount_id=2:i64
msg RemoveSyncPointEntry syncpoint_path=1:str mount_id=2:i64
msg AddMountPointEntry alluxio_path=1:str ufs_path=2:str readOnly=3:bool
    properties=4:StringPairEntry* shared=5:bool mount_id=6:i64
msg AsyncPersistRequestEntry file_id=1:i64
msg CompleteFileEntry block_ids=1:i64* id=2:i64 length=3:i64 op_time_ms=4:i64 ufs_fingerprint=5:str
msg DeleteFileEntry id=1:i64 recursive=2:bool op_time_ms=3:i64 alluxioOnly=4:bool path=5:str
msg DeleteMountPointEntry alluxio_path=1:str
msg NewBlockEntry id=1:i64
enum PTtlAction DELETE=0 FREE=1
msg UpdateInodeEntry id=1:i64 parent_id=2:i64 name=3:str persistence_state=4:str pinned=5:bool
    creation_time_ms=6:i64 last_modification_time_ms=7:i64 overwrite_modification_time=8:bool
    owner=9:str group=10:str mode=11:i32 ttl=12:i64 ttlAction=13:PTtlAction@DELETE
    acl=14:alluxio.proto.shared.AccessControlList ufs_fingerprint=15:str medium_type=16:str*
    xAttr=17:{str,bytes} last_access_time_ms=18:i64 overwrite_access_time=19:bool
msg UpdateInodeDirectoryEntry id=1:i64 mount_point=2:bool direct_children_loaded=3:bool
    defaultAcl=4:alluxio.proto.shared.AccessControlList
msg UpdateInodeFileEntry id=1:i64 block_size_bytes=2:i64 length=3:i64 completed=4:bool
    cacheable=5:bool set_blocks=7:i64* replication_max=8:i32 replication_min=9:i32
    persist_job_id=10:i64 temp_ufs_path=11:str path=12:str
msg InodeDirectoryEntry id=1:i64 parent_id=2:i64 name=3:str persistence_state=4:str pinned=5:bool
    creation_time_ms=6:i64 last_modification_time_ms=7:i64 owner=8:str group=9:str mode=10:i32
    mount_point=11:bool direct_children_loaded=12:bool ttl=13:i64 ttlAction=14:PTtlAction@DELETE
    acl=15:alluxio.proto.shared.AccessControlList defaultAcl=16:alluxio.proto.shared.AccessControlList
    path=17:str medium_type=18:str* xAttr=19:{str,bytes} last_access_time_ms=20:i64
msg InodeDirectoryIdGeneratorEntry container_id=1:i64 sequence_number=2:i64
msg InodeFileEntry id=1:i64 parent_id=2:i64 name=3:str persistence_state=4:str pinned=5:bool
    creation_time_ms=6:i64 last_modification_time_ms=7:i64 block_size_bytes=8:i64 length=9:i64
    completed=10:bool cacheable=11:bool blocks=12:i64* ttl=13:i64 owner=14:str group=15:str
    mode=16:i32 ttlAction=17:PTtlAction@DELETE ufs_fingerprint=18:str
    acl=19:alluxio.proto.shared.AccessControlList replication_max=20:i32 replication_min=21:i32
    persist_job_id=22:i64 temp_ufs_path=23:str replication_durable=24:i32 path=25:str
    medium_type=26:str* should_persist_time=27:i64 xAttr=28:{str,bytes} last_access_time_ms=29:i64
msg InodeLastModificationTimeEntry id=1:i64 last_modification_time_ms=2:i64
msg PersistDirectoryEntry id=1:i64
msg PersistFileEntry id=1:i64 length=2:i64 op_time_ms=3:i64
msg RenameEntry id=1:i64 dst_path=2:str op_time_ms=3:i64 new_parent_id=4:i64 new_name=5:str
    path=6:str new_path=7:str
enum PSetAclAction REPLACE=0 MODIFY=1 REMOVE=2 REMOVE_ALL=3 REMOVE_DEFAULT=4
msg SetAclEntry id=1:i64 op_time_ms=2:i64 action=3:PSetAclAction
    entries=4:alluxio.proto.shared.AclEntry* recursive=5:bool
msg SetAttributeEntry id=1:i64 op_time_ms=2:i64 pinned=3:bool ttl=4:i64 persisted=5:bool
    owner=6:str group=7:str permission=8:i32 ttlAction=9:PTtlAction@DELETE ufs_fingerprint=10:str
    persistJobId=11:i64 tempUfsPath=12:str replication_max=13:i32 replication_min=14:i32
enum UfsMode NO_ACCESS=0 READ_ONLY=1 READ_WRITE=2
msg UpdateUfsModeEntry ufsPath=1:str ufsMode=2:UfsMode@READ_WRITE
msg BlockContainerIdGeneratorEntry next_container_id=1:i64
msg BlockInfoEntry block_id=1:i64 length=2:i64
msg DeleteBlockEntry block_id=1:i64
msg PathPropertiesEntry path=1:str properties=2:{str,str}
msg RemovePathPropertiesEntry path=1:str
msg ClusterInfoEntry cluster_id=1:str
# table service entries (proto/journal/table.proto)
msg AttachDbEntry udb_type=1:str udb_connection_uri=2:str udb_db_name=3:str db_name=4:str
    config=5:{str,str}
msg DetachDbEntry db_name=1:str
msg UpdateDatabaseInfoEntry db_name=1:str location=2:str parameter=3:{str,str} owner_name=4:str
    comment=6:str
msg AddTableEntry db_name=1:str table_name=2:str owner=3:str schema_json=4:str
    layout_json=5:str parameters=6:{str,str} partitions_json=7:str*
msg RemoveTableEntry db_name=1:str table_name=2:str version=4:i64
msg AddTransformJobInfoEntry db_name=1:str table_name=2:str definition=3:str job_id=4:i64
    transformed_layouts=5:{str,str}
msg RemoveTransformJobInfoEntry db_name=1:str table_name=2:str
msg CompleteTransformTableEntry db_name=1:str table_name=2:str definition=3:str
    transformed_layouts=4:{str,str}

msg JournalEntry sequence_number=1:i64 active_sync_tx_id=34:ActiveSyncTxIdEntry
    add_table=43:AddTableEntry add_sync_point=32:AddSyncPointEntry
    add_mount_point=2:AddMountPointEntry async_persist_request=16:AsyncPersistRequestEntry
    attach_db=44:AttachDbEntry block_container_id_generator=3:BlockContainerIdGeneratorEntry
    block_info=4:BlockInfoEntry cluster_info=42:ClusterInfoEntry complete_file=5:CompleteFileEntry
    delete_block=29:DeleteBlockEntry delete_file=6:DeleteFileEntry
    delete_mount_point=8:DeleteMountPointEntry detach_db=45:DetachDbEntry
    inode_directory=9:InodeDirectoryEntry
    inode_directory_id_generator=10:InodeDirectoryIdGeneratorEntry inode_file=11:InodeFileEntry
    inode_last_modification_time=12:InodeLastModificationTimeEntry new_block=38:NewBlockEntry
    path_properties=40:PathPropertiesEntry persist_directory=15:PersistDirectoryEntry
    remove_path_properties=41:RemovePathPropertiesEntry remove_table=50:RemoveTableEntry
    remove_transform_job_info=47:RemoveTransformJobInfoEntry
    remove_sync_point=33:RemoveSyncPointEntry rename=19:RenameEntry set_acl=31:SetAclEntry
    set_attribute=27:SetAttributeEntry add_transform_job_info=46:AddTransformJobInfoEntry
    complete_transform_table=48:CompleteTransformTableEntry
    update_database_info=49:UpdateDatabaseInfoEntry update_ufs_mode=30:UpdateUfsModeEntry
    update_inode=35:UpdateInodeEntry update_inode_directory=36:UpdateInodeDirectoryEntry
    update_inode_file=37:UpdateInodeFileEntry journal_entries=39:JournalEntry*

package alluxio.proto.meta
msg BlockMeta length=1:i64
msg BlockLocation worker_id=1:i64 tier=2:str medium_type=3:str
msg Inode id=1:i64 creation_time_ms=2:i64 is_directory=3:bool ttl=4:i64 ttl_action=5:alluxio.grpc.TtlAction@DELETE
    last_modified_ms=25:i64 name=6:str parent_id=7:i64 persistence_state=8:str is_pinned=9:bool
    access_acl=10:alluxio.proto.shared.AccessControlList ufs_fingerprint=11:str medium_type=27:str*
    last_accessed_ms=30:i64 is_mount_point=12:bool has_direct_children_loaded=13:bool child_count=26:i64
    default_acl=14:alluxio.proto.shared.AccessControlList block_size_bytes=15:i64 blocks=16:i64*
    is_cacheable=17:bool is_completed=18:bool length=19:i64 replication_durable=20:i32 replication_max=21:i32
    replication_min=22:i32 should_persist_time=28:i64 persist_job_id=23:i64 persist_job_temp_ufs_path=24:str
    xAttr=29:{str,bytes}
"""
