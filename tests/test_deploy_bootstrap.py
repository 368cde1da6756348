"""Cloud/Vagrant bootstrap script (deploy/cloud/alluxio-bootstrap.sh; reference
integration/emr/alluxio-emr.sh, integration/dataproc/alluxio-dataproc.sh): installs a release
tarball, verifies its manifest and writes the node's site properties (configure-only run)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import release  # noqa: E402


def test_bootstrap_configure_only(tmp_path):
    res = release.make_tarball(str(tmp_path / "dist"), skip_native=True, version="7.7.7")
    prefix = tmp_path / "opt"
    env = dict(os.environ, ALLUXIO_PREFIX=str(prefix), PATH="/usr/bin:/bin")
    r = subprocess.run(["bash", os.path.join(ROOT, "deploy/cloud/alluxio-bootstrap.sh"), "-p", "vagrant",
                        "-t", res["tarball"], "-m", "master-0", "-r", "worker", "-u", "/data/ufs",
                        "-s", "alluxio.user.block.size.bytes.default=32MB", "-n"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "role=worker master=master-0" in r.stdout
    home = prefix / "alluxio-amd"
    assert (home / "bin" / "alluxio").exists() and (home / "lib/python/alluxio_amd/__init__.py").exists()
    site = (home / "conf" / "alluxio-site.properties").read_text()
    assert "alluxio.master.hostname=master-0" in site
    assert "alluxio.master.mount.table.root.ufs=/data/ufs" in site
    assert "alluxio.worker.tieredstore.level0.dirs.path=hbm" in site
    assert "alluxio.user.block.size.bytes.default=32MB" in site
