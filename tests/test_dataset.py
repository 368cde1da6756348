"""HBM dataset loader: batches of random records gathered by one launch (CPU: DRAM tier + host
tensors; GPU: HBM tier + device tensors, compared with a numpy reference of the same records)."""
import numpy as np
import pytest

from alluxio_amd.minicluster import LocalAlluxioCluster
from alluxio_amd.models import DeviceBatchLoader, FixedRecordDataset

REC = 3000  # not a divisor of the 64KB-ish block size: records straddle blocks


def _cluster(path):
    return LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": path,
                                                    "alluxio.worker.hbm.page.size": "64KB",
                                                    "alluxio.user.block.size.bytes.default": "256KB"})


def _check(c, device):
    import torch
    fs = c.client()
    rng = np.random.default_rng(3)
    files = []
    for k in range(2):
        d = rng.integers(0, 256, REC * (200 + 37 * k) + 17, dtype=np.uint8)  # trailing partial record
        fs.write_file(f"/ds/part-{k}", d, write_type="MUST_CACHE")
        files.append(d)
    ds = FixedRecordDataset(fs, ["/ds/part-0", "/ds/part-1"], REC, device=device)
    assert len(ds) == 200 + 237
    flat = [f[i * REC:(i + 1) * REC] for f in files for i in range(len(f) // REC)]
    assert np.array_equal(ds[5].cpu().numpy(), flat[5])
    assert np.array_equal(ds[250].cpu().numpy(), flat[250])
    with DeviceBatchLoader(ds, batch_size=64, shuffle=True, seed=1, device=device) as dl:
        seen = 0
        order = np.random.default_rng(1).permutation(len(ds))
        for b, batch in enumerate(dl):
            assert batch.device.type == torch.device(device).type
            idx = order[b * 64:(b + 1) * 64]
            ref = np.stack([flat[i] for i in idx])
            assert np.array_equal(batch.cpu().numpy(), ref)
            seen += batch.shape[0]
        assert seen == len(ds) and len(dl) == -(-len(ds) // 64)
    fs.close()


def test_loader_cpu():
    with _cluster("dram") as c:
        _check(c, "cpu")


@pytest.mark.gpu
def test_loader_gpu(gpu):
    with _cluster("hbm:0") as c:
        _check(c, "cuda")


def test_file_list_dataset_one_listing(tmp_path):
    """Config-4 shape: one record per file, metadata from one listStatus, batches gathered by one
    array-planned read per batch (short files zero-padded)."""
    import numpy as np
    import torch

    from alluxio_amd.minicluster import LocalAlluxioCluster
    from alluxio_amd.models.dataset import DeviceBatchLoader, FileListDataset
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram",
                                                   "alluxio.user.block.size.bytes.default": "1MB"}) as c:
        fs = c.client()
        rng = np.random.default_rng(0)
        files = {}
        for i in range(40):
            n = 4096 if i % 7 else 1000          # a few short files
            files[i] = rng.integers(0, 256, n, dtype=np.uint8)
            fs.write_file(f"/img/{i:05d}", files[i], write_type="MUST_CACHE")
        ds = FileListDataset(fs, "/img", record_bytes=4096)
        assert len(ds) == 40 and ds.single_block
        seen = 0
        with DeviceBatchLoader(ds, batch_size=16, shuffle=True, seed=3, device="cpu") as dl:
            order = np.random.default_rng(3).permutation(40)
            for b, batch in enumerate(dl):
                for r in range(batch.shape[0]):
                    i = int(order[b * 16 + r])
                    want = np.zeros(4096, dtype=np.uint8)
                    want[:len(files[i])] = files[i]
                    assert np.array_equal(batch[r].numpy(), want)
                    seen += 1
            assert dl._one_worker is not None
        assert seen == 40
        fs.close()
