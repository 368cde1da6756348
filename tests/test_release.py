"""Distribution builder (tools/release.py; reference dev/scripts generate-tarballs + assembly/)."""
import hashlib
import os
import sys
import tarfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import release  # noqa: E402


def test_tarball_layout_and_manifest(tmp_path):
    res = release.make_tarball(str(tmp_path), skip_native=True, version="9.9.9")
    assert os.path.exists(res["tarball"]) and res["version"] == "9.9.9"
    with open(res["tarball"], "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == res["sha256"]
    with tarfile.open(res["tarball"]) as t:
        names = set(t.getnames())
        top = "alluxio-amd-9.9.9/"
        for must in ("bin/alluxio", "conf/alluxio-site.properties.template", "pyproject.toml",
                     "lib/python/alluxio_amd/__init__.py", "lib/python/alluxio_amd/csrc/kernels.hip",
                     "MANIFEST.sha256"):
            assert top + must in names, must
        assert not any("__pycache__" in n for n in names)
        man = t.extractfile(top + "MANIFEST.sha256").read().decode().splitlines()
        entries = dict(reversed(line.split("  ", 1)) for line in man)
        assert len(entries) == len(names) - 1
        data = t.extractfile(top + "bin/alluxio").read()
        assert entries["bin/alluxio"] == hashlib.sha256(data).hexdigest()
        if res["native"]:
            so = [n for n in names if n.endswith(".so")]
            assert len(so) == 1 and release.has_gfx950_code(
                os.path.join(release.ROOT, "alluxio_amd", os.path.basename(so[0])))
