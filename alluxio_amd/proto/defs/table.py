"""Catalog (table) service.

Contract source: core/transport/src/main/proto/grpc/table/table_master.proto:1-404 (TableInfo,
Schema, Layout, Partition, column statistics, SyncStatus, constraint domains and the 12
TableMasterClientService RPCs).  Nested enums are flattened to package level.
"""

SCHEMA = r"""
package alluxio.grpc.table
msg FieldSchema id=1:u32 name=2:str type=3:str comment=4:str
msg Schema cols=1:FieldSchema*
enum PrincipalType USER=0 ROLE=1
msg Database db_name=1:str description=2:str location=3:str parameter=4:{str,str} owner_name=5:str
    owner_type=6:PrincipalType comment=7:str
enum TableType NATIVE=0 IMPORTED=1
msg LayoutSpec spec=1:str
msg PartitionSpec spec=1:str
msg BooleanColumnStatsData num_trues=1:i64 num_falses=2:i64 num_nulls=3:i64 bit_vectors=4:str
msg LongColumnStatsData low_value=1:i64 high_value=2:i64 num_nulls=3:i64 num_distincts=4:i64 bit_vectors=5:str
msg DoubleColumnStatsData low_value=1:f64 high_value=2:f64 num_nulls=3:i64 num_distincts=4:i64
    bit_vectors=5:str
msg Decimal scale=1:i32! unscaled=2:bytes!
msg DecimalColumnStatsData low_value=1:Decimal high_value=2:Decimal num_nulls=3:i64 num_distincts=4:i64
    bit_vectors=5:str
msg StringColumnStatsData max_col_len=1:i64 avg_col_len=2:f64 num_nulls=3:i64 num_distincts=4:i64
    bit_vectors=5:str
msg BinaryColumnStatsData max_col_len=1:i64 avg_col_len=2:f64 num_nulls=3:i64 bit_vectors=4:str
msg Date days_since_epoch=1:i64!
msg DateColumnStatsData low_value=1:Date high_value=2:Date num_nulls=3:i64 num_distincts=4:i64
    bit_vectors=5:str
msg ColumnStatisticsData boolean_stats=1:BooleanColumnStatsData|data long_stats=2:LongColumnStatsData|data
    double_stats=3:DoubleColumnStatsData|data string_stats=4:StringColumnStatsData|data
    binary_stats=5:BinaryColumnStatsData|data decimal_stats=6:DecimalColumnStatsData|data
    date_stats=7:DateColumnStatsData|data
msg ColumnStatisticsInfo col_name=1:str col_type=2:str data=3:ColumnStatisticsData
msg Layout layout_type=1:str layout_spec=2:LayoutSpec layout_data=3:bytes stats=4:{str,ColumnStatisticsInfo}
msg TableInfo db_name=1:str table_name=2:str type=3:TableType owner=4:str schema=5:Schema layout=6:Layout
    parameters=7:{str,str} partition_cols=8:FieldSchema* previous_version=9:i64 version=10:i64
    version_creation_time=11:i64
msg Transformation layout=1:Layout definition=2:str
msg Partition partition_spec=1:PartitionSpec base_layout=2:Layout transformations=3:Transformation*
    version=4:i64 version_creation_time=5:i64
msg SyncStatus tables_errors=1:{str,str} tables_ignored=2:str* tables_unchanged=3:str* tables_updated=4:str*
    tables_removed=5:str*
msg GetAllDatabasesPRequest
msg GetAllDatabasesPResponse database=1:str*
msg GetAllTablesPRequest database=1:str
msg GetAllTablesPResponse table=1:str*
msg GetDatabasePRequest db_name=1:str
msg GetDatabasePResponse db=1:Database
msg GetTablePRequest db_name=1:str table_name=2:str
msg GetTablePResponse table_info=1:TableInfo
msg AttachDatabasePRequest udb_type=1:str udb_connection_uri=2:str udb_db_name=3:str db_name=4:str
    options=5:{str,str} ignore_sync_errors=6:bool
msg AttachDatabasePResponse success=1:bool sync_status=2:SyncStatus
msg DetachDatabasePRequest db_name=1:str
msg DetachDatabasePResponse success=1:bool
msg SyncDatabasePRequest db_name=1:str
msg SyncDatabasePResponse success=1:bool status=2:SyncStatus
msg FileStatistics column=1:{str,ColumnStatisticsInfo}
msg GetTableColumnStatisticsPRequest db_name=1:str table_name=2:str col_names=3:str*
msg GetPartitionColumnStatisticsPRequest db_name=1:str table_name=2:str col_names=3:str* part_names=4:str*
msg GetTableColumnStatisticsPResponse statistics=1:ColumnStatisticsInfo*
msg ColumnStatisticsList statistics=1:ColumnStatisticsInfo*
msg GetPartitionColumnStatisticsPResponse partition_statistics=1:{str,ColumnStatisticsList}
msg Value long_type=1:i64|value double_type=2:f64|value string_type=3:str|value boolean_type=4:bool|value
msg Range low=1:Value high=2:Value
msg RangeSet ranges=1:Range*
msg EquatableValueSet candidates=1:Value* white_list=2:bool
msg AllOrNoneSet all=1:bool
msg Domain range=1:RangeSet|value_set equatable=2:EquatableValueSet|value_set all_or_none=3:AllOrNoneSet|value_set
msg Constraint column_constraints=1:{str,Domain}
msg ReadTablePRequest db_name=1:str table_name=2:str constraint=3:Constraint
msg ReadTablePResponse partitions=1:Partition*
msg TransformTablePRequest db_name=1:str table_name=2:str definition=3:str
msg TransformTablePResponse job_id=1:i64
msg GetTransformJobInfoPRequest job_id=1:i64
msg TransformJobInfo db_name=1:str table_name=2:str definition=3:str job_id=4:i64 job_status=5:alluxio.grpc.job.Status
    job_error=6:str
msg GetTransformJobInfoPResponse info=1:TransformJobInfo*
rpc TableMasterClientService GetAllDatabases GetAllDatabasesPRequest GetAllDatabasesPResponse
rpc TableMasterClientService GetAllTables GetAllTablesPRequest GetAllTablesPResponse
rpc TableMasterClientService GetDatabase GetDatabasePRequest GetDatabasePResponse
rpc TableMasterClientService GetTable GetTablePRequest GetTablePResponse
rpc TableMasterClientService AttachDatabase AttachDatabasePRequest AttachDatabasePResponse
rpc TableMasterClientService DetachDatabase DetachDatabasePRequest DetachDatabasePResponse
rpc TableMasterClientService SyncDatabase SyncDatabasePRequest SyncDatabasePResponse
rpc TableMasterClientService GetTableColumnStatistics GetTableColumnStatisticsPRequest GetTableColumnStatisticsPResponse
rpc TableMasterClientService GetPartitionColumnStatistics GetPartitionColumnStatisticsPRequest GetPartitionColumnStatisticsPResponse
rpc TableMasterClientService ReadTable ReadTablePRequest ReadTablePResponse
rpc TableMasterClientService TransformTable TransformTablePRequest TransformTablePResponse
rpc TableMasterClientService GetTransformJobInfo GetTransformJobInfoPRequest GetTransformJobInfoPResponse
"""
