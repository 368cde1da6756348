"""Hive Metastore (Thrift binary) and AWS Glue (JSON 1.1, SigV4) under-databases
(reference table/server/underdb/{hive,glue}: HiveDatabaseTest, GlueDatabaseTest), against
in-process fakes speaking the same wire formats.  Table locations are UFS directories outside
Alluxio, which the UDB mounts under /catalog/<db>/tables/<table>."""
import io
import json
import os
import socket
import socketserver
import struct
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.rpc import Channel
from alluxio_amd.table import TableClient
from alluxio_amd.table import metastore as ms


def _parquet(path, tbl):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    pq.write_table(tbl, path)


@pytest.fixture
def warehouse(tmp_path):
    wh = tmp_path / "warehouse"
    for year in (2020, 2021):
        _parquet(str(wh / "sales" / f"year={year}" / "p0.parquet"),
                 pa.table({"id": list(range(year, year + 5)), "amt": [1.5 * i for i in range(5)]}))
    _parquet(str(wh / "users" / "u.parquet"), pa.table({"uid": [1, 2, 3], "name": ["a", "bb", "ccc"]}))
    return wh


# ---- fake Hive metastore -----------------------------------------------------------------------
def _hms_tables(wh):
    sd = lambda loc, cols: {"cols": [{"name": n, "type": t} for n, t in cols], "location": loc,  # noqa: E731
                            "inputFormat": "org.apache.hadoop.hive.ql.io.parquet.MapredParquetInputFormat",
                            "serdeInfo": {"name": "s", "serializationLib": "parquet"}, "parameters": {}}
    return {
        "sales": {"tableName": "sales", "dbName": "hdb", "owner": "hive",
                  "sd": sd(f"file://{wh}/sales", [("id", "bigint"), ("amt", "double")]),
                  "partitionKeys": [{"name": "year", "type": "int"}], "parameters": {"k": "v"},
                  "tableType": "EXTERNAL_TABLE"},
        "users": {"tableName": "users", "dbName": "hdb", "owner": "hive",
                  "sd": sd(f"file://{wh}/users", [("uid", "bigint"), ("name", "string")]),
                  "partitionKeys": [], "tableType": "EXTERNAL_TABLE"},
    }


class _HmsHandler(socketserver.BaseRequestHandler):
    def handle(self):
        buf = b""
        while True:
            chunk = self.request.recv(65536)
            if not chunk:
                return
            buf += chunk
            try:
                r = ms.ThriftReader(buf)
                name, _, seq = r.message()
                args = r.struct()
            except EOFError:
                continue
            buf = buf[r.p:]
            self.server.calls.append(name)
            tables, wh = self.server.tables, self.server.wh
            w = ms.ThriftWriter()
            w.message(name, ms.M_REPLY, seq)
            _, rtype, rspec = ms.HMS_METHODS[name]
            if name == "get_database":
                res = {"success": {"name": args[1], "description": "hive db", "locationUri": f"file://{wh}",
                                   "parameters": {"p": "1"}, "ownerName": "hive"}}
            elif name == "get_all_tables":
                res = {"success": sorted(tables)}
            elif name == "get_table":
                t = tables.get(args[2])
                res = {"success": t} if t else {"o1": {"message": f"NoSuchObjectException {args[2]}"}}
            else:
                res = {"success": [{"values": [str(y)], "dbName": "hdb", "tableName": "sales",
                                    "sd": dict(tables["sales"]["sd"], location=f"file://{wh}/sales/year={y}")}
                                   for y in (2020, 2021)]}
            w.struct(res, [(0, rtype, "success", rspec), (1, ms.T_STRUCT, "o1", ms.META_EXCEPTION)])
            self.request.sendall(w.getvalue())


@pytest.fixture
def hms(warehouse):
    srv = socketserver.ThreadingTCPServer(("127.0.0.1", 0), _HmsHandler)
    srv.daemon_threads = True
    srv.calls, srv.wh, srv.tables = [], warehouse, _hms_tables(warehouse)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    yield srv
    srv.shutdown()
    srv.server_close()


def test_thrift_codec_roundtrip():
    t = _hms_tables("/w")["sales"]
    w = ms.ThriftWriter()
    w.struct(t, ms.TABLE)
    back = ms.ThriftReader(w.getvalue()).struct(ms.TABLE)
    assert back["tableName"] == "sales" and back["sd"]["cols"][1] == {"name": "amt", "type": "double"}
    assert back["partitionKeys"] == [{"name": "year", "type": "int"}] and back["parameters"] == {"k": "v"}
    # unknown fields are skipped by a reader with a narrower table
    narrow = ms.ThriftReader(w.getvalue()).struct([(1, ms.T_STRING, "tableName", None)])
    assert narrow["tableName"] == "sales" and 8 in narrow


def test_hive_client_errors(hms):
    c = ms.HiveMetastoreClient(f"thrift://127.0.0.1:{hms.server_address[1]}")
    assert c.call("get_all_tables", db_name="hdb") == ["sales", "users"]
    from alluxio_amd.utils.exceptions import NotFoundException, UnavailableException
    with pytest.raises(NotFoundException):
        c.call("get_table", dbname="hdb", tbl_name="nope")
    c.close()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        dead = s.getsockname()[1]
    with pytest.raises(UnavailableException):
        ms.HiveMetastoreClient(f"thrift://127.0.0.1:{dead}").call("get_all_tables", db_name="x")


@pytest.fixture
def cluster(tmp_path):
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"},
                             work_dir=str(tmp_path / "c")) as c:
        yield c, TableClient(Channel(c.master.address))


def _check_sales(tc, db):
    assert tc.tables(db) == ["sales", "users"]
    ti = tc.table(db, "sales")
    assert [(f.name, f.type) for f in ti.schema.cols] == [("id", "bigint"), ("amt", "double")]
    assert [p.name for p in ti.partition_cols] == ["year"]
    parts = tc.read_table(db, "sales")
    assert [p.partition_spec.spec for p in parts] == ["year=2020", "year=2021"]
    ps = tc.partition_statistics(db, "sales", ["id"], ["year=2021"])
    assert ps["year=2021"][0].data.long_stats.low_value == 2021


def test_attach_hive_database(cluster, hms):
    c, tc = cluster
    ok, st = tc.attach_database("hive", f"thrift://127.0.0.1:{hms.server_address[1]}", "hdb", "hivedb")
    assert ok and sorted(st.tables_updated) == ["sales", "users"], st
    _check_sales(tc, "hivedb")
    fs = c.client()
    # the table locations were mounted into Alluxio: data files readable through the catalog path
    assert fs.exists("/catalog/hivedb/tables/users")
    assert any(s.name == "u.parquet" for s in fs.list_status("/catalog/hivedb/tables/users"))
    assert "get_partitions" in hms.calls
    st = tc.sync_database("hivedb")
    assert sorted(st.tables_unchanged) == ["sales", "users"]
    fs.close()


# ---- fake Glue -----------------------------------------------------------------------------
class _GlueHandler(BaseHTTPRequestHandler):
    def log_message(self, *a):
        pass

    def do_POST(self):
        n = int(self.headers.get("Content-Length", 0))
        body = json.loads(self.rfile.read(n) or b"{}")
        op = self.headers.get("X-Amz-Target", "").split(".")[-1]
        srv = self.server
        srv.calls.append(op)
        if srv.require_sig and not self.headers.get("Authorization", "").startswith("AWS4-HMAC-SHA256 Credential=AK/"):
            return self._send(400, {"__type": "UnrecognizedClientException", "message": "no signature"})
        wh = srv.wh
        cols = {"sales": [("id", "bigint"), ("amt", "double")], "users": [("uid", "bigint"), ("name", "string")]}
        if op == "GetDatabase":
            return self._send(200, {"Database": {"Name": body["Name"], "LocationUri": f"file://{wh}",
                                                 "Description": "glue db", "Parameters": {"g": "1"}}})
        if op == "GetTables":               # one table per page: exercises NextToken paging
            names = ["sales", "users"]
            i = int(body.get("NextToken", "0"))
            out = {"TableList": [{"Name": names[i]}]}
            if i + 1 < len(names):
                out["NextToken"] = str(i + 1)
            return self._send(200, out)
        if op == "GetTable":
            name = body["Name"]
            if name not in cols:
                return self._send(400, {"__type": "com.amazonaws#EntityNotFoundException", "message": name})
            t = {"Name": name, "StorageDescriptor": {
                "Columns": [{"Name": c, "Type": ty} for c, ty in cols[name]], "Location": f"file://{wh}/{name}",
                "InputFormat": "org.apache.hadoop.hive.ql.io.parquet.MapredParquetInputFormat"},
                "PartitionKeys": [{"Name": "year", "Type": "int"}] if name == "sales" else []}
            return self._send(200, {"Table": t})
        if op == "GetColumnStatisticsForTable":
            if body["TableName"] != "users":
                return self._send(200, {"ColumnStatisticsList": []})
            return self._send(200, {"ColumnStatisticsList": [
                {"ColumnName": "uid", "ColumnType": "bigint", "StatisticsData": {
                    "Type": "LONG", "LongColumnStatisticsData": {"MinimumValue": 1, "MaximumValue": 3,
                                                                 "NumberOfNulls": 0, "NumberOfDistinctValues": 3}}},
                {"ColumnName": "name", "ColumnType": "string", "StatisticsData": {
                    "Type": "STRING", "StringColumnStatisticsData": {"MaximumLength": 3, "AverageLength": 2.0,
                                                                     "NumberOfNulls": 0,
                                                                     "NumberOfDistinctValues": 3}}}]})
        if op == "GetPartitions":
            parts = [{"Values": [str(y)], "StorageDescriptor": {"Location": f"file://{wh}/sales/year={y}"}}
                     for y in (2020, 2021)]
            return self._send(200, {"Partitions": parts})
        return self._send(400, {"__type": "InvalidInputException", "message": op})

    def _send(self, code, obj):
        data = json.dumps(obj).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/x-amz-json-1.1")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)


@pytest.fixture
def glue(warehouse):
    srv = HTTPServer(("127.0.0.1", 0), _GlueHandler)
    srv.calls, srv.wh, srv.require_sig = [], warehouse, True
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    yield srv
    srv.shutdown()
    srv.server_close()


def test_attach_glue_database(cluster, glue):
    c, tc = cluster
    opts = {"aws.glue.endpoint": f"http://127.0.0.1:{glue.server_address[1]}", "aws.accesskey": "AK",
            "aws.secretkey": "SK", "aws.region": "us-west-2"}
    ok, st = tc.attach_database("glue", "us-west-2", "gdb", "gluedb", options=opts)
    assert ok and sorted(st.tables_updated) == ["sales", "users"], st
    _check_sales(tc, "gluedb")
    stats = {s.col_name: s for s in tc.column_statistics("gluedb", "users", ["uid", "name"])}
    assert stats["uid"].data.long_stats.high_value == 3 and stats["name"].data.string_stats.max_col_len == 3
    assert glue.calls.count("GetTables") == 2          # NextToken paging
    db = tc.database("gluedb") if hasattr(tc, "database") else None
    if db is not None:
        assert db.location == f"file://{glue.wh}"
    # unsigned requests are refused by the endpoint: the attach fails cleanly
    bad = dict(opts, **{"aws.accesskey": ""})
    with pytest.raises(Exception):
        tc.attach_database("glue", "us-west-2", "gdb", "gluedb2", options=bad)
