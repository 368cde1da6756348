"""``alluxio validateEnv`` tasks (integration/tools/validation/.../ValidateEnv.java), including the
HDFS ones (hdfs/HdfsConfValidationTask, HdfsConfParityValidationTask, HdfsVersionValidationTask,
UfsSuperUserValidationTask, StorageSpaceValidationTask) against the in-process mini HDFS."""
import io
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
from hdfs_fake import MiniDfs  # noqa: E402

from alluxio_amd.cli import validate  # noqa: E402
from alluxio_amd.conf import Configuration  # noqa: E402

XML = """<?xml version="1.0"?><configuration>
<property><name>dfs.replication</name><value>%s</value></property>
<property><name>fs.defaultFS</name><value>hdfs://nn:8020</value></property></configuration>"""


def test_hdfs_validation_tasks(tmp_path, monkeypatch):
    dfs = MiniDfs()
    try:
        (tmp_path / "hdfs-site.xml").write_text(XML % "3")
        hd = tmp_path / "hadoop"
        hd.mkdir()
        (hd / "hdfs-site.xml").write_text(XML % "2")
        conf = Configuration({"alluxio.master.mount.table.root.ufs": f"hdfs://127.0.0.1:{dfs.port}/",
                              "alluxio.underfs.hdfs.configuration": str(tmp_path / "hdfs-site.xml"),
                              "alluxio.worker.tieredstore.level0.dirs.path": str(tmp_path / "ssd"),
                              "alluxio.worker.tieredstore.level0.dirs.quota": "1PB"})
        only = ["ufs.hdfs.config.parity", "ufs.hdfs.reachable", "ufs.superuser", "worker.storage.space"]
        monkeypatch.delenv("HADOOP_CONF_DIR", raising=False)
        res = validate.validate_env(conf=conf, out=io.StringIO(), only=only)
        flat = res
        assert flat["ufs.hdfs.config.parity"] == "OK", res
        assert flat["ufs.hdfs.reachable"] == "OK", res
        assert flat["ufs.superuser"] in ("OK", "WARNING"), res
        assert flat["worker.storage.space"] == "WARNING", res            # 1 PB does not fit
        monkeypatch.setenv("HADOOP_CONF_DIR", str(hd))
        res = validate.validate_env(conf=conf, out=io.StringIO(), only=["ufs.hdfs.config.parity"])
        assert res["ufs.hdfs.config.parity"] == "WARNING"
    finally:
        dfs.stop()
    conf2 = Configuration({"alluxio.master.mount.table.root.ufs": str(tmp_path)})
    res = validate.validate_env(conf=conf2, out=io.StringIO(), only=["ufs.hdfs.reachable"])
    assert res["ufs.hdfs.reachable"] == "SKIPPED"
