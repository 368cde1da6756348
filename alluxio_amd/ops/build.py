"""In-tree build of the native extension ``alluxio_amd._C`` for gfx950.

Compiles ``csrc/kernels.hip`` with ``hipcc --offload-arch=gfx950`` and the host C++ (block
store, codecs, pybind11 bindings) with ``hipcc`` in host mode, then links one shared object next
to the package so it travels with the repository snapshot to the GPU box.  Rebuilds only when a
source is newer than the ``.so``.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD = os.path.join(os.path.dirname(PKG_DIR), "build", "native")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

SOURCES = ["kernels.hip", "evict_alloc.hip", "page_cache_put.hip", "block_store.cpp", "cpu_codecs.cpp", "ipc.cpp", "ring_read.cpp", "page_cache.cpp", "meta_codec.cpp", "fuse_server.cpp", "http_blob.cpp",
           "frame_rpc.cpp", "journal_log.cpp", "sigv4.cpp", "numa_host.cpp", "data_server.cpp", "block_source.cpp", "stress_bench.cpp", "hdfs_packets.cpp", "data_path_bind.cpp", "bindings.cpp"]
HEADERS = ["kernels.h", "block_store.h", "cpu_codecs.h", "ipc.h", "ring_read.h", "page_cache.h", "page_cache_bind.h", "seg_ring.h", "frame_rpc.h", "journal_log.h", "meta_codec.h", "fuse_server.h", "h2_abi.h", "data_server.h", "sigv4.h", "numa_host.h", "http_blob.h",
           "block_source.h", "stress_bench.h", "hdfs_packets.h"]


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG_DIR, "_C" + suffix)


def _includes() -> list[str]:
    import pybind11
    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"], "-I" + CSRC]


def _needs_build(target: str) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    for f in SOURCES + HEADERS:
        if os.path.getmtime(os.path.join(CSRC, f)) > t:
            return True
    return os.path.getmtime(os.path.abspath(__file__)) > t


def _local_includes(path: str, seen: set | None = None) -> set:
    """Headers of csrc/ that ``path`` includes, transitively (``#include "x.h"``)."""
    import re
    seen = set() if seen is None else seen
    try:
        text = open(path).read()
    except OSError:
        return seen
    for h in re.findall(r'^\s*#\s*include\s+"([^"]+)"', text, re.M):
        hp = os.path.join(CSRC, h)
        if hp not in seen and os.path.exists(hp):
            seen.add(hp)
            _local_includes(hp, seen)
    return seen


def _obj_stale(src_path: str, obj: str) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src_path, os.path.abspath(__file__), *_local_includes(src_path)]
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"native build failed: {os.path.basename(cmd[-1])}")


def build(force: bool = False, verbose: bool = False) -> str:
    target = ext_path()
    if not force and not _needs_build(target):
        return target
    os.makedirs(BUILD, exist_ok=True)
    common = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-Wno-unused-result",
              "-Wno-unused-variable", "-fvisibility=hidden"] + _includes()
    jobs = []
    objs = []
    for src in SOURCES:
        obj = os.path.join(BUILD, src.replace(".", "_") + ".o")
        objs.append(obj)
        path = os.path.join(CSRC, src)
        if src.endswith(".hip"):
            cmd = [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *common,
                   "-c", path, "-o", obj]
        else:
            cmd = [HIPCC, "-x", "c++", "-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include", *common, "-c", path,
                   "-o", obj]
        if force or _obj_stale(path, obj):      # objects whose source and headers did not change are kept
            jobs.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=max(1, min(6, len(jobs)))) as ex:
        for fut in [ex.submit(_run, j) for j in jobs]:
            fut.result()
    tmp = target + ".tmp"
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp,
          f"-L{ROCM}/lib", "-lamdhip64", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{ROCM}/lib"])
    os.replace(tmp, target)
    if verbose:
        print("built", target)
    return target


SANITIZERS = {
    # host code only: the HIP kernels are compiled as usual (GPU sanitizers are not available on
    # the pool); the runtime is loaded into the (uninstrumented) interpreter with LD_PRELOAD
    "asan": (["-fsanitize=address,undefined", "-fno-gpu-sanitize", "-fno-sanitize-recover=undefined",
              "-shared-libasan"], "libclang_rt.asan-x86_64.so"),
    "tsan": (["-fsanitize=thread", "-fno-gpu-sanitize"], "libclang_rt.tsan-x86_64.so"),
}


def sanitizer_runtime(kind: str) -> str:
    import glob
    name = SANITIZERS[kind][1]
    hits = glob.glob(os.path.join(ROCM, "lib", "llvm", "lib", "clang", "*", "lib", "linux", name))
    if not hits:
        raise RuntimeError(f"{name} not found under {ROCM}/lib/llvm")
    return hits[0]


def build_sanitized(kind: str, out_dir: str | None = None) -> str:
    """A host-sanitizer build of the extension (CPU test runs only) into
    ``build/sanitize/<kind>/alluxio_amd/_C*.so``; load it with ``ALLUXIO_AMD_NATIVE_SO`` and the
    runtime from :func:`sanitizer_runtime` in ``LD_PRELOAD`` (tools/sanitize.sh)."""
    flags = SANITIZERS[kind][0]
    out_dir = out_dir or os.path.join(os.path.dirname(PKG_DIR), "build", "sanitize", kind)
    objdir = os.path.join(out_dir, "obj")
    os.makedirs(objdir, exist_ok=True)
    common = ["-O1", "-g", "-fno-omit-frame-pointer", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
              "-Wno-unused-result", "-Wno-unused-variable", "-fvisibility=hidden"] + _includes()
    jobs, objs = [], []
    for src in SOURCES:
        obj = os.path.join(objdir, src.replace(".", "_") + ".o")
        objs.append(obj)
        path = os.path.join(CSRC, src)
        if src.endswith(".hip"):
            # the host half of each .hip file (launchers, page-cache put/get bookkeeping) is
            # instrumented too; the device half is not (-Xarch_host scopes the sanitizer flags)
            host = []
            for f in flags:
                if f.startswith(("-fsanitize", "-fno-sanitize")):
                    host += ["-Xarch_host", f]
            cmd = [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *common, *host,
                   "-fno-gpu-sanitize", "-c", path, "-o", obj]
        else:
            cmd = [HIPCC, "-x", "c++", "-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include", *common,
                   *[f for f in flags if f != "-shared-libasan"], "-c", path, "-o", obj]
        jobs.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        for fut in [ex.submit(_run, j) for j in jobs]:
            fut.result()
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    target = os.path.join(out_dir, "_C" + suffix)
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *flags, *objs, "-o", target, f"-L{ROCM}/lib",
          "-lamdhip64", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{ROCM}/lib"])
    return target


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--sanitize":
        print(build_sanitized(sys.argv[2]))
    else:
        build(force="--force" in sys.argv, verbose=True)
