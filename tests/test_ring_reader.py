"""Device-cursor ring reader (RingReadSession + seq_read_kernel) vs the byte-level expectation of
StressWorkerBench's read(buf)/reopen loop (numpy reference of every sampled call)."""
import numpy as np
import pytest

from alluxio_amd.client.batch_reader import RingStreamReader
from alluxio_amd.minicluster import LocalAlluxioCluster


def _run(path, device):
    import torch
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": path,
                                                  "alluxio.worker.hbm.page.size": "64KB",
                                                  "alluxio.user.block.size.bytes.default": "256KB"}) as c:
        fs = c.client(metadata_cache=True)
        n = 1_000_003
        data = np.random.default_rng(0).integers(0, 256, n, dtype=np.uint8)
        fs.write_file("/r", data, write_type="MUST_CACHE")
        S, D, B = 16, 37, 4096
        ring = torch.zeros((S, D, B), dtype=torch.uint8, device=device)
        r = RingStreamReader(fs, "/r", ring, start_offsets=[i * 8192 for i in range(S)])
        total = 0
        for step in range(30):
            total += r.step()
            host = ring.cpu().numpy()
            for s in range(S):
                for k in range(D):
                    off, ln = r.last_call(s, k)
                    if ln:
                        assert np.array_equal(host[s, k, :ln], data[off:off + ln]), (step, s, k, off, ln)
        calls = 30 * D
        cycle = -(-n // B) + 1
        expect = 0
        for s in range(S):
            g0 = (s * 8192) // B
            for g in range(g0, g0 + calls):
                c_ = g % cycle
                if c_ != cycle - 1:
                    expect += min(B, n - c_ * B)
        assert total == expect == r.total_bytes
        assert r.reopens == sum((g0 + calls) // cycle - g0 // cycle for g0 in [(s * 8192) // B for s in range(S)])
        r.close()
        fs.close()


def test_ring_reader_cpu():
    _run("dram", "cpu")


@pytest.mark.gpu
def test_ring_reader_gpu(gpu):
    _run("hbm:0", "cuda")
