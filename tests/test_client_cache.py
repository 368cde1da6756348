"""Client local page cache (reference core/client/fs/src/test/.../cache/LocalCacheManagerTest,
LocalCacheFileInStreamTest, evictor tests): hits/misses, eviction order, restore, stream reads."""
import os

import numpy as np
import pytest

from alluxio_amd.client.cache import (LFUCacheEvictor, LocalCacheManager, LRUCacheEvictor, MemPageStore,
                                      PageId)
from alluxio_amd.conf import Configuration
from alluxio_amd.minicluster import LocalAlluxioCluster


def _conf(tmp_path, **kw):
    c = {"alluxio.user.client.cache.enabled": "true", "alluxio.user.client.cache.dir": str(tmp_path / "cache"),
         "alluxio.user.client.cache.page.size": "4KB", "alluxio.user.client.cache.size": "16KB"}
    c.update(kw)
    return Configuration(c)


def test_evictors():
    lru = LRUCacheEvictor()
    for i in range(3):
        lru.update_on_put(PageId("f", i))
    lru.update_on_get(PageId("f", 0))
    assert lru.evict() == PageId("f", 1)
    lfu = LFUCacheEvictor(Configuration())
    for i in range(3):
        lfu.update_on_put(PageId("f", i))
    for _ in range(4):
        lfu.update_on_get(PageId("f", 0))
        lfu.update_on_get(PageId("f", 2))
    assert lfu.evict() == PageId("f", 1)


def test_manager_put_get_evict_restore(tmp_path):
    m = LocalCacheManager(_conf(tmp_path))
    pages = {i: os.urandom(4096) for i in range(5)}
    for i in range(4):
        assert m.put(PageId("f", i), pages[i])
    assert m.get(PageId("f", 0), 10, 100) == pages[0][10:110]   # touch 0: LRU victim is now 1
    assert m.put(PageId("f", 4), pages[4])
    assert not m.has(PageId("f", 1)) and m.has(PageId("f", 0)) and m.bytes == 16384
    assert not m.put(PageId("f", 9), b"x" * 5000)               # larger than a page
    # LOCAL store restores its pages on restart
    m2 = LocalCacheManager(_conf(tmp_path))
    assert m2.bytes == 16384 and m2.get(PageId("f", 4), 0, 4096) == pages[4]
    mm = LocalCacheManager(_conf(tmp_path), store=MemPageStore())
    mm.put(PageId("g", 0), b"abc")
    assert mm.delete(PageId("g", 0)) and not mm.has(PageId("g", 0))


def test_cached_stream_through_filesystem(tmp_path):
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"}) as c:
        data = np.random.default_rng(1).integers(0, 256, 50_000, dtype=np.uint8).tobytes()
        plain = c.client()
        plain.write_file("/cc/f", data, write_type="MUST_CACHE")
        from alluxio_amd.client.file_system import FileSystem
        fs = FileSystem(conf=_conf(tmp_path, **{"alluxio.user.client.cache.size": "1MB"}),
                        master_address=c.master.address)
        with fs.open_file("/cc/f") as f:
            assert f.read() == data
        assert fs.local_cache.bytes == len(data)
        hits0 = fs.local_cache.metrics.counter("ClientCacheBytesReadCache").count
        with fs.open_file("/cc/f") as f:
            f.seek(12_345)
            assert f.read(9_999) == data[12_345:22_344]
            buf = bytearray(100)
            assert f.pread(40_000, buf) == 100 and bytes(buf) == data[40_000:40_100]
        assert fs.local_cache.metrics.counter("ClientCacheBytesReadCache").count - hits0 >= 10_099
        fs.close()
        plain.close()


@pytest.mark.gpu
def test_hbm_page_store_device_reads(gpu, tmp_path):
    import torch
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"}) as c:
        data = np.random.default_rng(2).integers(0, 256, 300_000, dtype=np.uint8)
        c.client().write_file("/hc/f", data, write_type="MUST_CACHE")
        from alluxio_amd.client.file_system import FileSystem
        fs = FileSystem(conf=_conf(tmp_path, **{"alluxio.user.client.cache.store.type": "HBM",
                                                "alluxio.user.client.cache.page.size": "64KB",
                                                "alluxio.user.client.cache.size": "8MB"}),
                        master_address=c.master.address)
        out = torch.empty(250_000, dtype=torch.uint8, device="cuda")
        with fs.open_file("/hc/f") as f:
            f.seek(17)
            assert f.read_into(out) == 250_000
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), data[17:250_017])
        with fs.open_file("/hc/f") as f:   # second pass: all hits, one gather launch
            f.seek(17)
            f.read_into(out)
        assert np.array_equal(out.cpu().numpy(), data[17:250_017])
        fs.close()


def test_local_page_store_options_mismatch_discards(tmp_path):
    from alluxio_amd.client.cache import LocalPageStore, PageId
    st = LocalPageStore(str(tmp_path), 4096, buckets=4, cache_size=1 << 20)
    st.put(PageId("f1", 0), b"a" * 10)
    assert [p for p, _ in LocalPageStore(str(tmp_path), 4096, 4, 1 << 20).restore()] == [PageId("f1", 0)]
    opts = tmp_path / "4096" / "options.pb"
    from alluxio_amd.proto import pb
    opts.write_bytes(pb.client_cache.PPageStoreCommonOptions(pageSize=4096, alluxioVersion="0.0.0-old")
                     .SerializeToString())
    assert LocalPageStore(str(tmp_path), 4096, 4, 1 << 20).restore() == []   # other version: wiped


def test_hbm_store_host_mode_slot_pressure(tmp_path):
    """HBM store on the native page table (host mode here): short pages use up the slots before
    the byte budget; the store's own LRU evictions reach the manager's metastore."""
    import torch
    from alluxio_amd.client.cache import HbmPageStore
    m = LocalCacheManager(_conf(tmp_path), store=HbmPageStore(16384, 4096, use_device=False))
    for i in range(6):
        assert m.put(PageId("f", i), bytes([i]) * 100)
    assert len(m.meta) == 4 == m.store.cache.used and m.bytes == 400
    assert not m.has(PageId("f", 0)) and not m.has(PageId("f", 1)) and m.has(PageId("f", 5))
    assert m.get(PageId("f", 5), 10, 20) == bytes([5]) * 20
    out = torch.zeros((3, 4096), dtype=torch.uint8)
    slots, lens = m.gather("f", torch.tensor([5, 0, 3]), out)
    assert slots.tolist()[1] == -1 and lens.tolist() == [100, 0, 100]
    assert bytes(out[0, :100].numpy()) == bytes([5]) * 100 and bytes(out[2, :100].numpy()) == bytes([3]) * 100


def test_read_pages_through_filesystem(tmp_path):
    _read_pages_body(tmp_path)


@pytest.mark.gpu
def test_read_pages_device_store(gpu, tmp_path):
    """Same reads with the store in HBM: GPU page indices, the small-page gather kernel (4 KiB
    pages, one 77-byte tail page)."""
    _read_pages_body(tmp_path)


def _read_pages_body(tmp_path):
    import torch
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"}) as c:
        data = np.random.default_rng(3).integers(0, 256, 10 * 4096 + 77, dtype=np.uint8)
        c.client().write_file("/rp/f", data, write_type="MUST_CACHE")
        from alluxio_amd.client.file_system import FileSystem
        fs = FileSystem(conf=_conf(tmp_path, **{"alluxio.user.client.cache.store.type": "HBM",
                                                "alluxio.user.client.cache.size": "1MB"}),
                        master_address=c.master.address)
        dev = fs.local_cache.store.device or torch.device("cpu")
        pages = [3, 10, 0, 3]
        out = torch.zeros((4, 4096), dtype=torch.uint8, device=dev)
        with fs.open_file("/rp/f") as f:
            lens = f.read_pages(torch.tensor(pages, device=dev), out)            # cold: misses filled
            lens2 = f.read_pages(torch.tensor(pages, device=dev), out, fill_misses=False)   # warm
        assert lens.tolist() == lens2.tolist() == [4096, 77, 4096, 4096]
        host = out.cpu().numpy()
        for r, p in enumerate(pages):
            n = int(lens[r])
            assert np.array_equal(host[r, :n], data[p * 4096:p * 4096 + n])
        fs.close()


@pytest.mark.gpu
def test_hbm_read_into_longer_than_cache(gpu, tmp_path):
    """A read_into spanning more pages than the HBM cache holds: every group of pages is filled
    and copied before the next group can evict it (slot reuse before the copy)."""
    import torch
    with LocalAlluxioCluster(num_workers=1, conf={"alluxio.worker.tieredstore.level0.dirs.path": "dram"}) as c:
        data = np.random.default_rng(5).integers(0, 256, 3_000_000, dtype=np.uint8)
        c.client().write_file("/hc/big", data, write_type="MUST_CACHE")
        from alluxio_amd.client.file_system import FileSystem
        fs = FileSystem(conf=_conf(tmp_path, **{"alluxio.user.client.cache.store.type": "HBM",
                                                "alluxio.user.client.cache.page.size": "64KB",
                                                "alluxio.user.client.cache.size": "512KB"}),
                        master_address=c.master.address)
        out = torch.empty(2_900_000, dtype=torch.uint8, device="cuda")
        for _ in range(2):
            with fs.open_file("/hc/big") as f:
                f.seek(33)
                assert f.read_into(out) == 2_900_000
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy(), data[33:2_900_033])
        fs.close()
