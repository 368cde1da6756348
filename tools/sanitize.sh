#!/bin/bash
# Host-sanitizer runs of the native extension: build csrc/ host code with
# ASan+UBSan and, separately, TSan (the HIP kernels compile as usual; GPU sanitizers are not
# available on the pool), then run the CPU test suite against each build by loading it through
# ALLUXIO_AMD_NATIVE_SO with the sanitizer runtime preloaded into the interpreter.
#   usage: tools/sanitize.sh [asan|tsan|all] [pytest args...]
set -euo pipefail
cd "$(dirname "$0")/.."
KIND=${1:-all}; shift || true
ARGS=("$@")
# TSan: the suites that drive this project's native threads (store locks, frame-RPC I/O
# threads, page cache, ring readers); tests that fork helper processes or load pyarrow's
# jemalloc are left to the ASan run (TSan cannot follow a multi-threaded fork)
TSAN_TESTS=(tests/test_native_store.py tests/test_native_rpc.py tests/test_page_cache_native.py
            tests/test_concurrency.py tests/test_cluster.py tests/test_tier_management.py
            tests/test_client_cache.py tests/test_ring_reader.py tests/test_marshal.py tests/test_master.py
            tests/test_journal.py tests/test_raft.py tests/test_ha.py tests/test_job_stress.py
            tests/test_proxy.py tests/test_fuse.py tests/test_metastore.py
            tests/test_grpc_native.py tests/test_fuse_native.py tests/test_s3_native.py tests/test_hdfs_native.py
            tests/test_data_server.py tests/test_hdfs_gateway.py)
if [ ${#ARGS[@]} -eq 0 ]; then
  if [ "$KIND" = tsan ]; then ARGS=("${TSAN_TESTS[@]}" -q -m "not gpu" -p no:cacheprovider -n 4)
  else ARGS=(tests -q -m "not gpu" -p no:cacheprovider -n 4); fi
fi
SUFFIX=$(python -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
run() {
  local k=$1
  python -m alluxio_amd.ops.build --sanitize "$k" > /dev/null
  rm -f build/sanitize/"$k"/report.*
  local rt; rt=$(python -c "from alluxio_amd.ops.build import sanitizer_runtime as s; print(s('$k'))")
  echo "=== $k: $rt"
  env LD_PRELOAD="$rt" ALLUXIO_AMD_NATIVE_SO="$PWD/build/sanitize/$k/_C$SUFFIX" \
      GRPC_ENABLE_FORK_SUPPORT=0 ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1" \
      UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1" \
      TSAN_OPTIONS="halt_on_error=1:die_after_fork=0:second_deadlock_stack=1:report_signal_unsafe=0:suppressions=$PWD/tools/tsan.supp:log_path=$PWD/build/sanitize/$k/report" \
      python -m pytest "${ARGS[@]}" || { cat build/sanitize/"$k"/report.* 2>/dev/null | head -80; return 1; }
  if ls build/sanitize/"$k"/report.* > /dev/null 2>&1; then
    echo "sanitizer reports:"; cat build/sanitize/"$k"/report.* | head -80; return 1
  fi
}
case $KIND in
  asan|tsan) run "$KIND" ;;
  all) run asan && ARGS=("${TSAN_TESTS[@]}" -q -m "not gpu" -p no:cacheprovider -n 4) && run tsan ;;
  *) echo "unknown sanitizer $KIND" >&2; exit 2 ;;
esac
