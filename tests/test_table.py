"""Catalog service (reference table/server/master/src/test: AlluxioCatalogTest, TableMasterTest,
transform integration): attach a filesystem UDB of Parquet/CSV tables, schema + statistics,
partition pruning through constraints, sync diffs, transform via the job service, journal replay."""
import io
import time

import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.proto import pb
from alluxio_amd.rpc import Channel
from alluxio_amd.table import TableClient, TableShell


def _parquet(tbl):
    b = io.BytesIO()
    pq.write_table(tbl, b)
    return b.getvalue()


@pytest.fixture
def env(tmp_path):
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"},
                             work_dir=str(tmp_path / "c")) as c:
        fs = c.client()
        for year in (2019, 2020, 2021):
            t = pa.table({"id": list(range(year, year + 10)), "price": [float(i) / 2 for i in range(10)],
                          "name": [f"item{i}" for i in range(10)], "ok": [i % 2 == 0 for i in range(10)]})
            fs.write_file(f"/wh/sales/year={year}/part-0.parquet", _parquet(t), write_type="MUST_CACHE")
        fs.write_file("/wh/users/u.csv", b"uid,city\n1,sf\n2,nyc\n3,sf\n", write_type="MUST_CACHE")
        import pyarrow.orc as porc
        b = io.BytesIO()
        porc.write_table(pa.table({"k": [3, 1, 2], "v": ["c", "a", "b"]}), b)
        fs.write_file("/wh/events/e.orc", b.getvalue(), write_type="MUST_CACHE")
        yield c, fs, TableClient(Channel(c.master.address))
        fs.close()


def test_attach_schema_stats_read(env):
    c, fs, tc = env
    ok, st = tc.attach_database("fs", "/wh", "", "wh")
    assert ok and sorted(st.tables_updated) == ["events", "sales", "users"]
    assert tc.databases() == ["wh"] and tc.tables("wh") == ["events", "sales", "users"]
    ti = tc.table("wh", "sales")
    assert [(f.name, f.type) for f in ti.schema.cols] == [("id", "bigint"), ("price", "double"),
                                                          ("name", "string"), ("ok", "boolean")]
    assert [p.name for p in ti.partition_cols] == ["year"]
    stats = {s.col_name: s for s in tc.column_statistics("wh", "sales", ["id", "price", "name", "ok"])}
    assert stats["id"].data.long_stats.low_value == 2019 and stats["id"].data.long_stats.high_value == 2030
    assert stats["price"].data.double_stats.high_value == 4.5
    assert stats["name"].data.string_stats.max_col_len == 5
    assert stats["ok"].data.boolean_stats.num_trues == 15
    ps = tc.partition_statistics("wh", "sales", ["id"], ["year=2020"])
    assert ps["year=2020"][0].data.long_stats.low_value == 2020
    parts = tc.read_table("wh", "sales")
    assert [p.partition_spec.spec for p in parts] == ["year=2019", "year=2020", "year=2021"]
    # constraint: year in {2020, 2021} (equatable white list) and year <= 2020 (range)
    con = pb.table.Constraint()
    con.column_constraints["year"].equatable.candidates.add(long_type=2020)
    con.column_constraints["year"].equatable.candidates.add(long_type=2021)
    con.column_constraints["year"].equatable.white_list = True
    assert [p.partition_spec.spec for p in tc.read_table("wh", "sales", con)] == ["year=2020", "year=2021"]
    con2 = pb.table.Constraint()
    con2.column_constraints["year"].range.ranges.add(high=pb.table.Value(long_type=2020))
    assert [p.partition_spec.spec for p in tc.read_table("wh", "sales", con2)] == ["year=2019", "year=2020"]
    u = tc.table("wh", "users")
    assert [f.name for f in u.schema.cols] == ["uid", "city"]
    # ORC table (reference transform/format/orc): schema and statistics from the ORC file
    ev = tc.table("wh", "events")
    assert [(f.name, f.type) for f in ev.schema.cols] == [("k", "bigint"), ("v", "string")]
    es = {s.col_name: s for s in tc.column_statistics("wh", "events", ["k"])}
    assert es["k"].data.long_stats.low_value == 1 and es["k"].data.long_stats.high_value == 3


def test_sync_detach_and_journal_replay(env):
    c, fs, tc = env
    tc.attach_database("fs", "/wh", "", "wh")
    st = tc.sync_database("wh")
    assert sorted(st.tables_unchanged) == ["events", "sales", "users"]
    fs.write_file("/wh/sales/year=2022/part-0.parquet",
                  _parquet(pa.table({"id": [1], "price": [1.0], "name": ["x"], "ok": [True]})), write_type="MUST_CACHE")
    fs.delete("/wh/users", recursive=True)
    st = tc.sync_database("wh")
    assert list(st.tables_updated) == ["sales"] and list(st.tables_removed) == ["users"]
    assert tc.table("wh", "sales").version == 2
    c.restart_master()
    tc2 = TableClient(Channel(c.master.address))
    assert tc2.tables("wh") == ["events", "sales"]
    assert len(tc2.read_table("wh", "sales")) == 4
    assert tc2.detach_database("wh") and tc2.databases() == []


def test_transform_via_job_service(env):
    c, fs, tc = env
    tc.attach_database("fs", "/wh", "", "wh")
    jid = tc.transform_table("wh", "sales", "file.count.max=2")
    tm = c.master.table_master
    for _ in range(500):
        c.drive_jobs()
        if tm.transform_heartbeat():
            break
        time.sleep(0.01)
    info = tc.transform_job_info(jid)[0]
    assert pb.job.Status.values_by_number[info.job_status].name == "COMPLETED", info
    parts = tc.read_table("wh", "sales")
    import json
    for p in parts:
        assert len(p.transformations) == 1
        lay = json.loads(p.transformations[0].layout.layout_data)
        assert 1 <= len(lay["files"]) <= 2
        back = pa.concat_tables([pq.read_table(io.BytesIO(fs.read_file(f))) for f in lay["files"]])
        assert back.num_rows == 10
    # an ORC table compacts to Parquet too
    jid2 = tc.transform_table("wh", "events", "file.count.max=1")
    for _ in range(500):
        c.drive_jobs()
        if tm.transform_heartbeat():
            break
        time.sleep(0.01)
    ev = tc.read_table("wh", "events")[0]
    lay = json.loads(ev.transformations[0].layout.layout_data)
    assert pq.read_table(io.BytesIO(fs.read_file(lay["files"][0]))).column("k").to_pylist() == [3, 1, 2]
    assert pb.job.Status.values_by_number[tc.transform_job_info(jid2)[0].job_status].name == "COMPLETED"
    out = io.StringIO()
    assert TableShell(Channel(c.master.address), out).run(["transformStatus", str(jid)]) == 0
    assert "COMPLETED" in out.getvalue()


def test_table_shell_and_errors(env):
    c, fs, tc = env
    out = io.StringIO()
    sh = TableShell(Channel(c.master.address), out)
    assert sh.run(["attachdb", "fs", "/wh", "wh"]) == 0
    assert sh.run(["ls"]) == 0 and "wh" in out.getvalue()
    assert sh.run(["ls", "wh", "sales"]) == 0 and "PARTITIONED BY year" in out.getvalue()
    assert sh.run(["attachdb", "hive", "thrift://x:9083", "h"]) == -1
    assert sh.run(["detachdb", "wh"]) == 0
