"""Under-database (UDB) SPI and the filesystem UDB.

Parity: table/server/common/src/main/java/alluxio/table/common/udb/UnderDatabase.java (getTableNames,
getTable, getDatabaseInfo), UdbTable.java (schema, partition columns, partitions, statistics),
UdbPartition / layout/HiveLayout.java, and table/server/underdb/hive (HiveDatabase: tables are
directories of data files, partitions are ``key=value`` sub-directories).

Metastore-backed UDBs (``hive`` over Thrift, ``glue`` over its JSON API) live in
:mod:`table.metastore`.  The ``fs`` type needs no metastore: a database is a directory (Alluxio path, or a UFS URI mounted under
``/catalog/<db>/ufs``); each sub-directory is a table of Parquet (schema + column statistics from
the footer) or CSV files (schema inferred, statistics computed); ``k=v`` sub-directories are
partitions.
"""
from __future__ import annotations

import io
import json
import posixpath

from ..utils.exceptions import NotFoundException, UnavailableException

DATA_EXT = (".parquet", ".parq", ".csv", ".orc")


class UdbPartition:
    def __init__(self, spec: str, location: str, files: list[str], fmt: str):
        self.spec, self.location, self.files, self.format = spec, location, files, fmt

    def values(self) -> dict[str, str]:
        out = {}
        for part in self.spec.split("/") if self.spec else []:
            k, _, v = part.partition("=")
            out[k] = v
        return out


class UdbTable:
    def __init__(self, name, location, schema: list[tuple[str, str]], partition_cols: list[tuple[str, str]],
                 partitions: list[UdbPartition], stats: dict, part_stats: dict, fmt: str):
        self.name, self.location, self.schema = name, location, schema
        self.partition_cols, self.partitions, self.stats = partition_cols, partitions, stats
        self.part_stats, self.format = part_stats, fmt

    def fingerprint(self) -> str:
        return json.dumps([self.schema, [(p.spec, p.files) for p in self.partitions]], sort_keys=True)


def _arrow_type_name(t) -> str:
    import pyarrow as pa
    if pa.types.is_boolean(t):
        return "boolean"
    if pa.types.is_integer(t):
        return "bigint" if t.bit_width > 32 else "int"
    if pa.types.is_floating(t):
        return "double"
    if pa.types.is_date(t):
        return "date"
    if pa.types.is_timestamp(t):
        return "timestamp"
    if pa.types.is_decimal(t):
        return f"decimal({t.precision},{t.scale})"
    if pa.types.is_binary(t) or pa.types.is_large_binary(t):
        return "binary"
    return "string"


def _stats_of_table(tbl) -> dict:
    """{column: {type, min, max, nulls, distinct, max_len, avg_len, trues, falses}} (exact)."""
    import pyarrow.compute as pc
    out = {}
    for name in tbl.column_names:
        col = tbl.column(name)
        t = _arrow_type_name(col.type)
        st = {"type": t, "nulls": int(col.null_count)}
        valid = pc.drop_null(col)
        if len(valid):
            if t == "boolean":
                st["trues"] = int(pc.sum(pc.cast(valid, "int64")).as_py() or 0)
                st["falses"] = len(valid) - st["trues"]
            elif t in ("string", "binary"):
                lens = pc.binary_length(valid) if t == "binary" else pc.utf8_length(valid)
                st["max_len"] = int(pc.max(lens).as_py())
                st["avg_len"] = float(pc.mean(lens).as_py())
                st["distinct"] = int(pc.count_distinct(valid).as_py())
            else:
                mm = pc.min_max(valid)
                lo, hi = mm["min"].as_py(), mm["max"].as_py()
                if t == "date":
                    import datetime
                    epoch = datetime.date(1970, 1, 1)
                    lo, hi = (lo - epoch).days, (hi - epoch).days
                elif t == "timestamp":
                    lo, hi = int(lo.timestamp()), int(hi.timestamp())
                elif t.startswith("decimal"):
                    lo, hi = str(lo), str(hi)
                st["min"], st["max"] = lo, hi
                st["distinct"] = int(pc.count_distinct(valid).as_py())
        out[name] = st
    return out


def merge_stats(parts: list[dict]) -> dict:
    out: dict = {}
    for p in parts:
        for c, s in p.items():
            m = out.setdefault(c, {"type": s["type"], "nulls": 0})
            m["nulls"] += s.get("nulls", 0)
            for k in ("trues", "falses"):
                if k in s:
                    m[k] = m.get(k, 0) + s[k]
            if "min" in s:
                m["min"] = s["min"] if "min" not in m else min(m["min"], s["min"])
                m["max"] = s["max"] if "max" not in m else max(m["max"], s["max"])
            if "max_len" in s:
                m["max_len"] = max(m.get("max_len", 0), s["max_len"])
                m["avg_len"] = s["avg_len"] if "avg_len" not in m else (m["avg_len"] + s["avg_len"]) / 2
            if "distinct" in s:
                m["distinct"] = max(m.get("distinct", 0), s["distinct"])
    return out


class UnderDatabase:
    def get_database_info(self) -> dict:  # pragma: no cover - interface
        raise NotImplementedError

    def get_table_names(self) -> list[str]:  # pragma: no cover - interface
        raise NotImplementedError

    def get_table(self, name: str) -> UdbTable:  # pragma: no cover - interface
        raise NotImplementedError


class FilesystemUnderDatabase(UnderDatabase):
    def __init__(self, fs, location: str, db_name: str, options: dict | None = None):
        self.fs = fs
        self.location = location.rstrip("/") or "/"
        self.db_name = db_name
        self.options = dict(options or {})

    def get_database_info(self) -> dict:
        return {"location": self.location, "parameter": dict(self.options), "owner_name": "",
                "comment": f"filesystem database at {self.location}"}

    def get_table_names(self) -> list[str]:
        try:
            kids = self.fs.list_status(self.location)
        except NotFoundException:
            raise UnavailableException(f"database location {self.location} does not exist") from None
        return sorted(k.name for k in kids if k.is_folder and not k.name.startswith(("_", ".")))

    def _read(self, path: str, fmt: str):
        return read_table_bytes(self.fs.read_file(path), fmt)

    def _scan(self, loc: str, depth: int = 0):
        """[(partition spec, location, [files])] below a table directory."""
        files, subs = [], []
        for s in self.fs.list_status(loc):
            if s.is_folder:
                if "=" in s.name and not s.name.startswith(("_", ".")):
                    subs.append(s)
            elif s.name.lower().endswith(DATA_EXT) and s.length > 0:
                files.append(s.path)
        out = []
        if files:
            out.append(("", loc, sorted(files)))
        for s in sorted(subs, key=lambda x: x.name):
            for spec, l2, f2 in self._scan(s.path, depth + 1):
                out.append((s.name + ("/" + spec if spec else ""), l2, f2))
        return out

    def get_table(self, name: str) -> UdbTable:
        loc = posixpath.join(self.location, name)
        parts = self._scan(loc)
        if not parts:
            raise NotFoundException(f"table {name} has no data files under {loc}")
        fmt = format_of(parts[0][2][0])
        schema: list[tuple[str, str]] = []
        pstats, partitions = {}, []
        for spec, ploc, files in parts:
            tables = [self._read(f, fmt) for f in files]
            if not schema:
                schema = [(f.name, _arrow_type_name(f.type)) for f in tables[0].schema]
            pstats[spec] = merge_stats([_stats_of_table(t) for t in tables])
            partitions.append(UdbPartition(spec, ploc, files, fmt))
        pcols = [(k, "string") for k in partitions[0].values()] if partitions and partitions[0].spec else []
        return UdbTable(name, loc, schema, pcols, partitions, merge_stats(list(pstats.values())), pstats, fmt)


def format_of(path: str) -> str:
    """Data format of a table file by extension: csv, orc or parquet (reference
    job/server/.../transform/format/{csv,orc,parquet})."""
    p = path.lower()
    if p.endswith(".csv"):
        return "csv"
    if p.endswith(".orc"):
        return "orc"
    return "parquet"


def read_table_bytes(data: bytes, fmt: str):
    """An Arrow table from one data file's bytes."""
    if fmt == "csv":
        import pyarrow.csv as pcsv
        return pcsv.read_csv(io.BytesIO(data))
    if fmt == "orc":
        import pyarrow.orc as porc
        return porc.ORCFile(io.BytesIO(data)).read()
    import pyarrow.parquet as pq
    return pq.read_table(io.BytesIO(data))


METASTORE_TYPES = ("hive", "glue")


def create_udb(udb_type: str, fs, location: str, db_name: str, options: dict | None = None,
               catalog_db: str | None = None, catalog_path: str = "/catalog") -> UnderDatabase:
    """``location`` is the database directory for ``fs`` UDBs and the metastore connection URI
    (``thrift://host:port`` / Glue region or endpoint) for ``hive`` / ``glue``; ``db_name`` is the
    under-database's name and ``catalog_db`` the Alluxio catalog's name for it."""
    t = (udb_type or "fs").lower()
    if t in ("fs", "filesystem", "file", "parquet"):
        return FilesystemUnderDatabase(fs, location, db_name, options)
    if t == "hive":
        from .metastore import HiveUnderDatabase
        return HiveUnderDatabase(fs, location, catalog_db or db_name, db_name, options, catalog_path)
    if t == "glue":
        from .metastore import GlueUnderDatabase
        return GlueUnderDatabase(fs, location, catalog_db or db_name, db_name, options, catalog_path)
    raise UnavailableException(f"unknown udb type {udb_type}")
