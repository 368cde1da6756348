#!/usr/bin/env python3
"""Build a binary distribution tarball: ``alluxio-amd-<version>-gfx950.tar.gz``.

Parity: dev/scripts/generate-tarballs (+ src/main/java/.../GenerateTarball in dev/scripts) and
assembly/ (the reference's release builder: build the modules, lay out ``bin/ conf/ lib/ libexec/``
plus docs and deploy files under ``alluxio-<version>/``, tar it, print the checksum).

Here the "modules" are the Python package and the native gfx950 extension: the builder compiles
``alluxio_amd._C`` in-tree (``hipcc --offload-arch=gfx950``), verifies the shared object carries a
gfx950 code object, then lays out::

    alluxio-amd-<version>/
      bin/ conf/ deploy/ docs/          launch scripts, templates, Docker/Helm, docs
      lib/python/alluxio_amd/           the package (sources + the built _C*.so)
      pyproject.toml README.md
      MANIFEST.sha256                   sha256 of every file in the tarball

``--skip-native`` packages whatever ``_C*.so`` is present (or none: a pure-Python client tarball).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import io
import os
import subprocess
import sys
import tarfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TOP_DIRS = ("bin", "conf", "deploy", "docs")
TOP_FILES = ("pyproject.toml", "setup.py", "README.md")
EXCLUDE_DIRS = {"__pycache__", ".pytest_cache", "build", "gpurun_out"}


def _files(base: str, rel: str):
    start = os.path.join(base, rel)
    if os.path.isfile(start):
        yield rel
        return
    for d, dirs, files in os.walk(start):
        dirs[:] = sorted(x for x in dirs if x not in EXCLUDE_DIRS)
        for f in sorted(files):
            if f.endswith((".pyc", ".o")):
                continue
            yield os.path.relpath(os.path.join(d, f), base)


def has_gfx950_code(so_path: str) -> bool:
    """True when the extension embeds an amdgcn gfx950 code object (offload bundle)."""
    with open(so_path, "rb") as f:
        data = f.read()
    return b"gfx950" in data and b"amdgcn" in data


def build_native() -> str:
    from alluxio_amd.ops.build import build
    os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    return build()


def make_tarball(out_dir: str, skip_native: bool = False, version: str | None = None) -> dict:
    from alluxio_amd import __version__
    version = version or __version__
    name = f"alluxio-amd-{version}"
    so = None
    if not skip_native:
        so = build_native()
        if not has_gfx950_code(so):
            raise RuntimeError(f"{so} carries no gfx950 code object")
    else:
        found = glob.glob(os.path.join(ROOT, "alluxio_amd", "_C*.so"))
        so = found[0] if found else None
    entries: list[tuple[str, str]] = []        # (path in tarball, source path)
    for rel in TOP_DIRS + TOP_FILES:
        if os.path.exists(os.path.join(ROOT, rel)):
            entries += [(f"{name}/{p}", os.path.join(ROOT, p)) for p in _files(ROOT, rel)]
    for p in _files(ROOT, "alluxio_amd"):
        if p.endswith(".so") and (so is None or os.path.abspath(os.path.join(ROOT, p)) != os.path.abspath(so)):
            continue                              # stale builds for other interpreters
        entries.append((f"{name}/lib/python/{p}", os.path.join(ROOT, p)))
    os.makedirs(out_dir, exist_ok=True)
    suffix = "gfx950" if so else "noarch"
    tar_path = os.path.join(out_dir, f"{name}-{suffix}.tar.gz")
    manifest = []
    with tarfile.open(tar_path, "w:gz") as tar:
        for arc, src in entries:
            with open(src, "rb") as f:
                data = f.read()
            manifest.append(f"{hashlib.sha256(data).hexdigest()}  {arc[len(name) + 1:]}")
            ti = tarfile.TarInfo(arc)
            ti.size = len(data)
            ti.mode = os.stat(src).st_mode & 0o777
            ti.mtime = int(os.stat(src).st_mtime)
            tar.addfile(ti, io.BytesIO(data))
        body = ("\n".join(manifest) + "\n").encode()
        ti = tarfile.TarInfo(f"{name}/MANIFEST.sha256")
        ti.size, ti.mtime, ti.mode = len(body), int(time.time()), 0o644
        tar.addfile(ti, io.BytesIO(body))
    with open(tar_path, "rb") as f:
        digest = hashlib.sha256(f.read()).hexdigest()
    with open(tar_path + ".sha256", "w") as f:
        f.write(f"{digest}  {os.path.basename(tar_path)}\n")
    return {"tarball": tar_path, "sha256": digest, "files": len(entries) + 1, "native": so is not None,
            "version": version}


def git_describe() -> str | None:
    try:
        return subprocess.run(["git", "-C", ROOT, "describe", "--always", "--dirty"], capture_output=True,
                              text=True, check=True).stdout.strip()
    except Exception:  # noqa: BLE001
        return None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--out", default=os.path.join(ROOT, "build", "dist"))
    ap.add_argument("--skip-native", action="store_true", help="do not (re)build the gfx950 extension")
    ap.add_argument("--version", default=None)
    a = ap.parse_args(argv)
    res = make_tarball(a.out, a.skip_native, a.version)
    res["git"] = git_describe()
    print(f"Tarball: {res['tarball']}\nsha256: {res['sha256']}\nfiles: {res['files']}  native: {res['native']}"
          f"  git: {res['git']}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
