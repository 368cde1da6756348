"""Catalog (table) service: table master, under-database SPI, client and shell.

``TableClient`` mirrors table/client/src/main/java/alluxio/client/table/TableMasterClient.java;
``TableShell`` the ``alluxio table`` commands of table/shell/.../TableShell.java (attachdb,
detachdb, ls, sync, transform, transformStatus).
"""
from __future__ import annotations

import json
import sys

from ..proto import enum_name, pb

SVC_TABLE = "alluxio.grpc.table.TableMasterClientService"


class TableClient:
    def __init__(self, channel):
        self.stub = channel.stub(SVC_TABLE)

    def attach_database(self, udb_type, uri, udb_db, db_name, options=None, ignore_sync_errors=False):
        r = self.stub.AttachDatabase(pb.table.AttachDatabasePRequest(
            udb_type=udb_type, udb_connection_uri=uri, udb_db_name=udb_db, db_name=db_name,
            options=options or {}, ignore_sync_errors=ignore_sync_errors))
        return r.success, r.sync_status

    def detach_database(self, db):
        return self.stub.DetachDatabase(pb.table.DetachDatabasePRequest(db_name=db)).success

    def sync_database(self, db):
        return self.stub.SyncDatabase(pb.table.SyncDatabasePRequest(db_name=db)).status

    def databases(self):
        return list(self.stub.GetAllDatabases(pb.table.GetAllDatabasesPRequest()).database)

    def tables(self, db):
        return list(self.stub.GetAllTables(pb.table.GetAllTablesPRequest(database=db)).table)

    def database(self, db):
        return self.stub.GetDatabase(pb.table.GetDatabasePRequest(db_name=db)).db

    def table(self, db, t):
        return self.stub.GetTable(pb.table.GetTablePRequest(db_name=db, table_name=t)).table_info

    def column_statistics(self, db, t, cols):
        return list(self.stub.GetTableColumnStatistics(pb.table.GetTableColumnStatisticsPRequest(
            db_name=db, table_name=t, col_names=cols)).statistics)

    def partition_statistics(self, db, t, cols, parts):
        r = self.stub.GetPartitionColumnStatistics(pb.table.GetPartitionColumnStatisticsPRequest(
            db_name=db, table_name=t, col_names=cols, part_names=parts))
        return {k: list(v.statistics) for k, v in r.partition_statistics.items()}

    def read_table(self, db, t, constraint=None):
        req = pb.table.ReadTablePRequest(db_name=db, table_name=t)
        if constraint is not None:
            req.constraint.CopyFrom(constraint)
        return list(self.stub.ReadTable(req).partitions)

    def transform_table(self, db, t, definition=""):
        return self.stub.TransformTable(pb.table.TransformTablePRequest(db_name=db, table_name=t,
                                                                        definition=definition)).job_id

    def transform_job_info(self, job_id=0):
        return list(self.stub.GetTransformJobInfo(pb.table.GetTransformJobInfoPRequest(job_id=job_id)).info)


class TableShell:
    def __init__(self, channel=None, out=None):
        if channel is None:
            from ..client.context import FileSystemContext
            channel = FileSystemContext().master_channel()
        self.c = TableClient(channel)
        self.out = out or sys.stdout

    def p(self, *a):
        print(*a, file=self.out)

    def run(self, argv) -> int:
        if not argv:
            self.p("Usage: alluxio table [attachdb|detachdb|ls|sync|transform|transformStatus]")
            return 1
        cmd, a = argv[0], argv[1:]
        try:
            if cmd == "attachdb":
                opts, pos, udb_db = {}, [], ""
                i = 0
                while i < len(a):
                    if a[i] == "-o":
                        k, _, v = a[i + 1].partition("=")
                        opts[k] = v
                        i += 2
                    elif a[i] == "--db":
                        udb_db = a[i + 1]
                        i += 2
                    else:
                        pos.append(a[i])
                        i += 1
                udb_type, uri = pos[0], pos[1]
                db = pos[2] if len(pos) > 2 else (udb_db or uri.rstrip("/").rsplit("/", 1)[-1])
                ok, st = self.c.attach_database(udb_type, uri, udb_db, db, opts, "--ignore-sync-errors" in a)
                self.p(f"{'Attached' if ok else 'Failed to attach'} database {db}: updated={list(st.tables_updated)} "
                       f"errors={dict(st.tables_errors)}")
                return 0 if ok else -1
            if cmd == "detachdb":
                self.c.detach_database(a[0])
                return 0
            if cmd == "sync":
                st = self.c.sync_database(a[0])
                self.p(f"updated={list(st.tables_updated)} unchanged={list(st.tables_unchanged)} "
                       f"removed={list(st.tables_removed)}")
                return 0
            if cmd == "ls":
                if not a:
                    for d in self.c.databases():
                        self.p(d)
                elif len(a) == 1:
                    for t in self.c.tables(a[0]):
                        self.p(t)
                else:
                    ti = self.c.table(a[0], a[1])
                    self.p(f"TABLE {ti.db_name}.{ti.table_name} (version {ti.version})")
                    for col in ti.schema.cols:
                        self.p(f"  {col.name} {col.type}")
                    for pc in ti.partition_cols:
                        self.p(f"  PARTITIONED BY {pc.name} {pc.type}")
                    self.p(f"  LOCATION {ti.layout.layout_spec.spec}")
                return 0
            if cmd == "transform":
                jid = self.c.transform_table(a[0], a[1], a[2] if len(a) > 2 else "")
                self.p(f"Started transformation job with job ID {jid}, you can monitor the status of the job "
                       f"with './bin/alluxio table transformStatus {jid}'.")
                return 0
            if cmd == "transformStatus":
                for i in self.c.transform_job_info(int(a[0]) if a else 0):
                    self.p(json.dumps({"db": i.db_name, "table": i.table_name, "definition": i.definition,
                                       "job_id": i.job_id, "status": enum_name(pb.job.Status, i.job_status)
                                       if i.job_status else "", "error": i.job_error}))
                return 0
        except Exception as e:  # noqa: BLE001
            self.p(str(e))
            return -1
        self.p(f"{cmd} is an unknown command.")
        return 1
