"""Table (catalog) master.

Parity: table/server/master/src/main/java/alluxio/master/table/DefaultTableMaster.java:207,
AlluxioCatalog.java:472 (attach/detach/sync databases from an under-database, table/partition
metadata, column statistics, readTable with partition-column constraints), Database.java / Table.java
(versioned tables, sync diff into updated/unchanged/removed), transform/TransformManager.java:477
(transformTable submits a job-service job that rewrites each partition as Parquet with at most
``file.count.max`` files; on completion the partition gains a Transformation whose layout points at
the new files) and the journal entries of proto/journal/table.proto.
"""
from __future__ import annotations

import json
import logging
import posixpath
import threading
import time

from ..journal.system import Journaled, NoopJournalContext
from ..proto import enum_name, pb
from ..utils.exceptions import (AlreadyExistsException, InvalidArgumentException, NotFoundException)
from .udb import METASTORE_TYPES, UdbPartition, create_udb

LOG = logging.getLogger(__name__)
SVC_TABLE = "alluxio.grpc.table.TableMasterClientService"


class _Table:
    def __init__(self, db, name, owner, schema, layout, parameters, partitions, version=1):
        self.db, self.name, self.owner = db, name, owner
        self.schema = schema            # [[name, type], ...]
        self.layout = layout            # {"location", "format", "partition_cols", "stats", "part_stats"}
        self.parameters = dict(parameters)
        self.partitions = partitions    # [{"spec", "location", "files", "format", "transformations": []}]
        self.version = version
        self.created = int(time.time() * 1000)


class TableMaster(Journaled):
    journal_name = "TableMaster"

    def __init__(self, conf, journal_system=None, fs_factory=None, job_master=None):
        self.conf = conf
        self.journal = journal_system
        self.fs_factory = fs_factory
        self.job_master = job_master
        self.dbs: dict[str, dict] = {}
        self.tables: dict[tuple[str, str], _Table] = {}
        self.transforms: dict[int, dict] = {}
        self._lock = threading.RLock()
        self.catalog_path = conf.get("alluxio.table.catalog.path", "/catalog")

    # ---- journal ------------------------------------------------------------------------------
    def reset_state(self) -> None:
        self.dbs.clear()
        self.tables.clear()
        self.transforms.clear()

    def process_journal_entry(self, e) -> bool:
        if e.HasField("attach_db"):
            a = e.attach_db
            self.dbs[a.db_name] = {"udb_type": a.udb_type, "uri": a.udb_connection_uri, "udb_db": a.udb_db_name,
                                   "options": dict(a.config), "location": "", "parameter": {}, "owner": "",
                                   "comment": ""}
        elif e.HasField("update_database_info"):
            u = e.update_database_info
            d = self.dbs.get(u.db_name)
            if d is not None:
                d.update(location=u.location, parameter=dict(u.parameter), owner=u.owner_name, comment=u.comment)
        elif e.HasField("detach_db"):
            name = e.detach_db.db_name
            self.dbs.pop(name, None)
            for k in [k for k in self.tables if k[0] == name]:
                del self.tables[k]
        elif e.HasField("add_table"):
            a = e.add_table
            old = self.tables.get((a.db_name, a.table_name))
            parts = [json.loads(p) for p in a.partitions_json]
            self.tables[(a.db_name, a.table_name)] = _Table(
                a.db_name, a.table_name, a.owner, json.loads(a.schema_json or "[]"),
                json.loads(a.layout_json or "{}"), dict(a.parameters), parts, (old.version + 1) if old else 1)
        elif e.HasField("remove_table"):
            self.tables.pop((e.remove_table.db_name, e.remove_table.table_name), None)
        elif e.HasField("add_transform_job_info"):
            t = e.add_transform_job_info
            self.transforms[t.job_id] = {"db": t.db_name, "table": t.table_name, "definition": t.definition,
                                         "layouts": dict(t.transformed_layouts)}
        elif e.HasField("remove_transform_job_info"):
            r = e.remove_transform_job_info
            for jid in [j for j, v in self.transforms.items() if (v["db"], v["table"]) == (r.db_name, r.table_name)]:
                del self.transforms[jid]
        elif e.HasField("complete_transform_table"):
            c = e.complete_transform_table
            tbl = self.tables.get((c.db_name, c.table_name))
            if tbl is not None:
                for p in tbl.partitions:
                    lay = c.transformed_layouts.get(p["spec"] or "_")
                    if lay:
                        p.setdefault("transformations", []).append({"definition": c.definition,
                                                                    "layout": json.loads(lay)})
        else:
            return False
        return True

    def journal_entries(self):
        for name, d in self.dbs.items():
            a = pb.journal.AttachDbEntry(udb_type=d["udb_type"], udb_connection_uri=d["uri"], udb_db_name=d["udb_db"],
                                         db_name=name)
            for k, v in d["options"].items():
                a.config[k] = v
            yield pb.journal.JournalEntry(attach_db=a)
            u = pb.journal.UpdateDatabaseInfoEntry(db_name=name, location=d["location"], owner_name=d["owner"],
                                                   comment=d["comment"])
            for k, v in d["parameter"].items():
                u.parameter[k] = v
            yield pb.journal.JournalEntry(update_database_info=u)
        for t in self.tables.values():
            yield pb.journal.JournalEntry(add_table=self._table_entry(t.db, t.name, t.owner, t.schema, t.layout,
                                                                      t.parameters, t.partitions))
        for jid, v in self.transforms.items():
            e = pb.journal.AddTransformJobInfoEntry(db_name=v["db"], table_name=v["table"], definition=v["definition"],
                                                    job_id=jid)
            for k, l in v["layouts"].items():
                e.transformed_layouts[k] = l
            yield pb.journal.JournalEntry(add_transform_job_info=e)

    def _ctx(self):
        return NoopJournalContext() if self.journal is None else self.journal.create_context(self.journal_name)

    def _apply(self, ctx, e) -> None:
        self.apply_and_journal(ctx, e)

    @staticmethod
    def _table_entry(db, name, owner, schema, layout, params, parts):
        e = pb.journal.AddTableEntry(db_name=db, table_name=name, owner=owner, schema_json=json.dumps(schema),
                                     layout_json=json.dumps(layout, default=str),
                                     partitions_json=[json.dumps(p, default=str) for p in parts])
        for k, v in params.items():
            e.parameters[k] = v
        return e

    # ---- database ops -------------------------------------------------------------------------
    def _fs(self):
        return self.fs_factory()

    def _db_location(self, name, uri) -> str:
        if "://" in uri and not uri.startswith("alluxio://"):
            mp = posixpath.join(self.catalog_path, name, "ufs")
            fs = self._fs()
            if not fs.exists(mp):
                fs.create_directory(posixpath.dirname(mp), recursive=True, allow_exists=True)
                fs.mount(mp, uri, read_only=True)
            return mp
        if uri.startswith("alluxio://"):
            uri = "/" + uri[len("alluxio://"):].split("/", 1)[1]
        return uri

    def attach_database(self, udb_type, uri, udb_db, db_name, options=None, ignore_sync_errors=False):
        with self._lock:
            if db_name in self.dbs:
                raise AlreadyExistsException(f"database {db_name} already exists")
            metastore = (udb_type or "").lower() in METASTORE_TYPES
            location = uri if metastore else self._db_location(db_name, uri)
            udb = create_udb(udb_type, self._fs(), location, udb_db or db_name, options, catalog_db=db_name,
                             catalog_path=self.catalog_path)
            info = udb.get_database_info()
            if metastore:
                location = info.get("location") or uri
            with self._ctx() as ctx:
                a = pb.journal.AttachDbEntry(udb_type=udb_type, udb_connection_uri=uri, udb_db_name=udb_db,
                                             db_name=db_name)
                for k, v in (options or {}).items():
                    a.config[k] = v
                self._apply(ctx, pb.journal.JournalEntry(attach_db=a))
                u = pb.journal.UpdateDatabaseInfoEntry(db_name=db_name, location=location,
                                                       owner_name=info.get("owner_name", ""),
                                                       comment=info.get("comment", ""))
                for k, v in info.get("parameter", {}).items():
                    u.parameter[k] = v
                self._apply(ctx, pb.journal.JournalEntry(update_database_info=u))
            status = self._sync(db_name, udb, ignore_sync_errors)
            if status.tables_errors and not ignore_sync_errors:
                self.detach_database(db_name)
                return False, status
            return True, status

    def detach_database(self, db_name) -> bool:
        with self._lock:
            if db_name not in self.dbs:
                raise NotFoundException(f"database {db_name} does not exist")
            with self._ctx() as ctx:
                self._apply(ctx, pb.journal.JournalEntry(detach_db=pb.journal.DetachDbEntry(db_name=db_name)))
        return True

    def sync_database(self, db_name):
        with self._lock:
            d = self.dbs.get(db_name)
            if d is None:
                raise NotFoundException(f"database {db_name} does not exist")
            metastore = (d["udb_type"] or "").lower() in METASTORE_TYPES
            udb = create_udb(d["udb_type"], self._fs(), d["uri"] if metastore else d["location"],
                             d["udb_db"] or db_name, d["options"], catalog_db=db_name, catalog_path=self.catalog_path)
            return self._sync(db_name, udb, True)

    def _sync(self, db_name, udb, ignore_errors):
        st = pb.table.SyncStatus()
        names = udb.get_table_names()
        with self._ctx() as ctx:
            for name in names:
                try:
                    t = udb.get_table(name)
                except Exception as e:  # noqa: BLE001
                    st.tables_errors[name] = str(e)
                    continue
                layout = {"location": t.location, "format": t.format, "partition_cols": t.partition_cols,
                          "stats": t.stats, "part_stats": t.part_stats, "fingerprint": t.fingerprint()}
                parts = [{"spec": p.spec, "location": p.location, "files": p.files, "format": p.format,
                          "transformations": []} for p in t.partitions]
                old = self.tables.get((db_name, name))
                if old is not None and old.layout.get("fingerprint") == layout["fingerprint"]:
                    st.tables_unchanged.append(name)
                    continue
                self._apply(ctx, pb.journal.JournalEntry(add_table=self._table_entry(
                    db_name, name, "", [list(c) for c in t.schema], layout, {}, parts)))
                st.tables_updated.append(name)
            for (db, name) in [k for k in self.tables if k[0] == db_name and k[1] not in names]:
                self._apply(ctx, pb.journal.JournalEntry(remove_table=pb.journal.RemoveTableEntry(
                    db_name=db, table_name=name)))
                st.tables_removed.append(name)
        return st

    # ---- queries ------------------------------------------------------------------------------
    def get_database(self, name):
        d = self.dbs.get(name)
        if d is None:
            raise NotFoundException(f"database {name} does not exist")
        db = pb.table.Database(db_name=name, location=d["location"], owner_name=d["owner"], comment=d["comment"],
                               description=f"{d['udb_type']} database {d['udb_db'] or name}")
        for k, v in d["parameter"].items():
            db.parameter[k] = v
        return db

    def _table(self, db, name) -> _Table:
        if db not in self.dbs:
            raise NotFoundException(f"database {db} does not exist")
        t = self.tables.get((db, name))
        if t is None:
            raise NotFoundException(f"table {db}.{name} does not exist")
        return t

    @staticmethod
    def _stats_proto(col, s):
        ci = pb.table.ColumnStatisticsInfo(col_name=col, col_type=s["type"])
        t = s["type"]
        d = ci.data
        if t == "boolean":
            d.boolean_stats.CopyFrom(pb.table.BooleanColumnStatsData(num_trues=s.get("trues", 0),
                                                                     num_falses=s.get("falses", 0),
                                                                     num_nulls=s["nulls"]))
        elif t in ("int", "bigint", "timestamp"):
            d.long_stats.CopyFrom(pb.table.LongColumnStatsData(low_value=int(s.get("min", 0)), high_value=int(s.get("max", 0)),
                                                               num_nulls=s["nulls"], num_distincts=s.get("distinct", 0)))
        elif t == "double":
            d.double_stats.CopyFrom(pb.table.DoubleColumnStatsData(low_value=float(s.get("min", 0)),
                                                                   high_value=float(s.get("max", 0)),
                                                                   num_nulls=s["nulls"], num_distincts=s.get("distinct", 0)))
        elif t == "date":
            d.date_stats.CopyFrom(pb.table.DateColumnStatsData(
                low_value=pb.table.Date(days_since_epoch=int(s.get("min", 0))),
                high_value=pb.table.Date(days_since_epoch=int(s.get("max", 0))), num_nulls=s["nulls"],
                num_distincts=s.get("distinct", 0)))
        elif t == "binary":
            d.binary_stats.CopyFrom(pb.table.BinaryColumnStatsData(max_col_len=s.get("max_len", 0),
                                                                   avg_col_len=s.get("avg_len", 0.0), num_nulls=s["nulls"]))
        else:
            d.string_stats.CopyFrom(pb.table.StringColumnStatsData(max_col_len=s.get("max_len", 0),
                                                                   avg_col_len=s.get("avg_len", 0.0), num_nulls=s["nulls"],
                                                                   num_distincts=s.get("distinct", 0)))
        return ci

    def _layout_proto(self, loc, fmt, files, stats=None):
        lay = pb.table.Layout(layout_type="fs", layout_spec=pb.table.LayoutSpec(spec=loc),
                              layout_data=json.dumps({"location": loc, "format": fmt, "files": files}).encode())
        for c, s in (stats or {}).items():
            lay.stats[c].CopyFrom(self._stats_proto(c, s))
        return lay

    def get_table(self, db, name):
        t = self._table(db, name)
        ti = pb.table.TableInfo(db_name=db, table_name=name, type=pb.table.TableType.values_by_name["IMPORTED"].number,
                                owner=t.owner, version=t.version, version_creation_time=t.created,
                                previous_version=t.version - 1 if t.version > 1 else 0)
        ti.schema.cols.extend(pb.table.FieldSchema(id=i, name=c, type=ty) for i, (c, ty) in enumerate(t.schema))
        ti.partition_cols.extend(pb.table.FieldSchema(name=c, type=ty) for c, ty in t.layout.get("partition_cols", []))
        ti.layout.CopyFrom(self._layout_proto(t.layout.get("location", ""), t.layout.get("format", ""), [],
                                              t.layout.get("stats", {})))
        for k, v in t.parameters.items():
            ti.parameters[k] = v
        return ti

    def get_table_column_statistics(self, db, name, cols):
        t = self._table(db, name)
        stats = t.layout.get("stats", {})
        return [self._stats_proto(c, stats[c]) for c in cols if c in stats]

    def get_partition_column_statistics(self, db, name, cols, parts):
        t = self._table(db, name)
        ps = t.layout.get("part_stats", {})
        out = {}
        for p in parts:
            st = ps.get(p)
            if st is not None:
                out[p] = [self._stats_proto(c, st[c]) for c in cols if c in st]
        return out

    @staticmethod
    def _typed(v: str, domain_value):
        kind = domain_value.WhichOneof("value")
        try:
            if kind == "long_type":
                return int(v), domain_value.long_type
            if kind == "double_type":
                return float(v), domain_value.double_type
            if kind == "boolean_type":
                return v.lower() == "true", domain_value.boolean_type
        except ValueError:
            pass
        return v, getattr(domain_value, kind) if kind else ""

    def _matches(self, values: dict, constraint) -> bool:
        for col, dom in constraint.column_constraints.items():
            if col not in values:
                continue  # constraints on data columns do not prune partitions
            v = values[col]
            which = dom.WhichOneof("value_set")
            if which == "all_or_none":
                if not dom.all_or_none.all:
                    return False
            elif which == "equatable":
                hit = any(self._typed(v, c)[0] == self._typed(v, c)[1] for c in dom.equatable.candidates)
                if hit != dom.equatable.white_list:
                    return False
            elif which == "range":
                ok = False
                for r in dom.range.ranges:
                    lo_ok = not r.HasField("low") or self._typed(v, r.low)[0] >= self._typed(v, r.low)[1]
                    hi_ok = not r.HasField("high") or self._typed(v, r.high)[0] <= self._typed(v, r.high)[1]
                    ok = ok or (lo_ok and hi_ok)
                if not ok:
                    return False
        return True

    def read_table(self, db, name, constraint=None):
        t = self._table(db, name)
        out = []
        for p in t.partitions:
            up = UdbPartition(p["spec"], p["location"], p["files"], p["format"])
            if constraint is not None and not self._matches(up.values(), constraint):
                continue
            part = pb.table.Partition(partition_spec=pb.table.PartitionSpec(spec=p["spec"]), version=t.version,
                                      version_creation_time=t.created)
            part.base_layout.CopyFrom(self._layout_proto(p["location"], p["format"], p["files"],
                                                         t.layout.get("part_stats", {}).get(p["spec"], {})))
            for tr in p.get("transformations", []):
                lay = tr["layout"]
                part.transformations.add(definition=tr["definition"],
                                         layout=self._layout_proto(lay["location"], lay["format"], lay["files"]))
            out.append(part)
        return out

    # ---- transforms ---------------------------------------------------------------------------
    def transform_table(self, db, name, definition: str) -> int:
        from ..job import TransformConfig
        t = self._table(db, name)
        if self.job_master is None:
            raise InvalidArgumentException("transformTable needs the job service")
        dloc = self.dbs[db]["location"]
        base = posixpath.join(self.catalog_path, db, "tables", name, "_transformed", str(int(time.time() * 1000)))
        parts = [{"spec": p["spec"], "files": p["files"], "format": p["format"],
                  "dst": posixpath.join(base, p["spec"]) if p["spec"] else base} for p in t.partitions]
        jid = self.job_master.run(TransformConfig(db=db, table=name, transform=definition, partitions=parts))
        layouts = {p["spec"] or "_": json.dumps({"location": p["dst"], "format": "parquet", "files": []})
                   for p in parts}
        with self._ctx() as ctx:
            e = pb.journal.AddTransformJobInfoEntry(db_name=db, table_name=name, definition=definition, job_id=jid)
            for k, v in layouts.items():
                e.transformed_layouts[k] = v
            self._apply(ctx, pb.journal.JournalEntry(add_transform_job_info=e))
        del dloc
        return jid

    def transform_heartbeat(self) -> int:
        """TransformManager's job poller: finalise completed transformation jobs."""
        if self.job_master is None:
            return 0
        done = 0
        for jid, v in list(self.transforms.items()):
            if v.get("completed"):
                continue
            try:
                info = self.job_master.status(jid)
            except NotFoundException:
                continue
            if info.status != "COMPLETED":
                continue
            files = info.result or {}
            layouts = {}
            for spec, lay in v["layouts"].items():
                lj = json.loads(lay)
                lj["files"] = files.get(spec, [])
                layouts[spec] = json.dumps(lj)
            with self._ctx() as ctx:
                e = pb.journal.CompleteTransformTableEntry(db_name=v["db"], table_name=v["table"],
                                                           definition=v["definition"])
                for k, l in layouts.items():
                    e.transformed_layouts[k] = l
                self._apply(ctx, pb.journal.JournalEntry(complete_transform_table=e))
            v["completed"] = True
            done += 1
        return done

    def transform_job_infos(self, job_id: int = 0):
        out = []
        for jid, v in self.transforms.items():
            if job_id and jid != job_id:
                continue
            i = pb.table.TransformJobInfo(db_name=v["db"], table_name=v["table"], definition=v["definition"], job_id=jid)
            if self.job_master is not None:
                try:
                    st = self.job_master.status(jid)
                    i.job_status = pb.job.Status.values_by_name[st.status].number
                    i.job_error = st.error
                except NotFoundException:
                    pass
            out.append(i)
        return out


class TableMasterService:
    def __init__(self, tm: TableMaster):
        self.tm = tm

    def GetAllDatabases(self, req, ctx):
        return pb.table.GetAllDatabasesPResponse(database=sorted(self.tm.dbs))

    def GetAllTables(self, req, ctx):
        if req.database not in self.tm.dbs:
            raise NotFoundException(f"database {req.database} does not exist")
        return pb.table.GetAllTablesPResponse(table=sorted(n for d, n in self.tm.tables if d == req.database))

    def GetDatabase(self, req, ctx):
        return pb.table.GetDatabasePResponse(db=self.tm.get_database(req.db_name))

    def GetTable(self, req, ctx):
        return pb.table.GetTablePResponse(table_info=self.tm.get_table(req.db_name, req.table_name))

    def AttachDatabase(self, req, ctx):
        ok, st = self.tm.attach_database(req.udb_type, req.udb_connection_uri, req.udb_db_name, req.db_name,
                                         dict(req.options), req.ignore_sync_errors)
        return pb.table.AttachDatabasePResponse(success=ok, sync_status=st)

    def DetachDatabase(self, req, ctx):
        return pb.table.DetachDatabasePResponse(success=self.tm.detach_database(req.db_name))

    def SyncDatabase(self, req, ctx):
        return pb.table.SyncDatabasePResponse(success=True, status=self.tm.sync_database(req.db_name))

    def GetTableColumnStatistics(self, req, ctx):
        return pb.table.GetTableColumnStatisticsPResponse(
            statistics=self.tm.get_table_column_statistics(req.db_name, req.table_name, list(req.col_names)))

    def GetPartitionColumnStatistics(self, req, ctx):
        r = pb.table.GetPartitionColumnStatisticsPResponse()
        for p, st in self.tm.get_partition_column_statistics(req.db_name, req.table_name, list(req.col_names),
                                                             list(req.part_names)).items():
            r.partition_statistics[p].statistics.extend(st)
        return r

    def ReadTable(self, req, ctx):
        c = req.constraint if req.HasField("constraint") else None
        return pb.table.ReadTablePResponse(partitions=self.tm.read_table(req.db_name, req.table_name, c))

    def TransformTable(self, req, ctx):
        return pb.table.TransformTablePResponse(job_id=self.tm.transform_table(req.db_name, req.table_name,
                                                                               req.definition))

    def GetTransformJobInfo(self, req, ctx):
        return pb.table.GetTransformJobInfoPResponse(info=self.tm.transform_job_infos(req.job_id))


__all__ = ["TableMaster", "TableMasterService", "SVC_TABLE", "enum_name"]
