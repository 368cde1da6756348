"""The native StressWorkerBench client (csrc/stress_bench.cpp, ``worker_bench --mode native-threads``).

Reference shape pinned here: StressWorkerBench.java:251-276 -- every thread loops read(buf) over
the whole file and re-opens it at EOF; WorkerBenchSummary.java:59-71 -- only bytes read after the
warmup count, over the duration.
"""
import os

import numpy as np
import pytest

from alluxio_amd.ops.native import lib
from alluxio_amd.stress.worker_bench import main as worker_bench

from test_data_server import _cluster, _remote_fs

pytestmark = pytest.mark.skipif(not lib().FrameRpcServer.grpc_available(), reason="libnghttp2 not present")


@pytest.mark.parametrize("short_circuit", [False, True])
def test_native_threads_read_the_file_over_and_over(tmp_path, short_circuit):
    with _cluster(tmp_path) as c:
        fs = c.client()
        fs.create_directory("/stress-worker-base", recursive=True, allow_exists=True)
        fs.write_file("/stress-worker-base/data", np.full(3 << 20, ord("A"), dtype=np.uint8),
                      write_type="MUST_CACHE", block_size=1 << 20)
        rfs = _remote_fs(c, **{"alluxio.user.short.circuit.enabled": str(short_circuit).lower(),
                               "alluxio.user.native.reader.buffer.size": "256KB"})
        st = c.workers[0].data_server.stats
        s0 = st.streams
        # a sanitizer build (tools/sanitize.sh) runs the readers ~10x slower: give them the time to
        # go round the file
        slow = bool(os.environ.get("ALLUXIO_AMD_NATIVE_SO"))
        r = worker_bench(["--threads", "8", "--file-size", "3m", "--buffer-size", "4k", "--block-size", "1m",
                          "--duration", "4s" if slow else "400ms", "--warmup", "100ms", "--mode", "native-threads"],
                         fs=rfs, print_result=False)
        assert not r["errors"], r["errors"]
        n = r["native"]
        assert r["bytes"] > 0 and r["bytes"] == n["reads"] * 4096
        assert n["file_opens"] > 8                    # every thread went round the file and re-opened it
        assert n["block_opens"] >= 3 * 8
        if short_circuit:
            assert n["transport"] == "ipc" or n["transport"] == "grpc-uds"
        else:
            assert n["transport"].startswith("grpc")
            assert st.streams - s0 >= n["block_opens"] - 8   # a ReadBlock call per block per pass
        rfs.close()
        fs.close()
