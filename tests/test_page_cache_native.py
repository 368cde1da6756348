"""K9 native HBM client page cache (csrc/page_cache.{h,cpp} + page_lookup_gather_kernel).

Parity: core/client/fs/src/main/java/alluxio/client/file/cache/LocalCacheManager.java:249-347 (put with
two-phase evict), :360 (get), evictor/LRUCacheEvictor.java.  The host-mode cache (use_device=False) runs
the same table and eviction logic on the CPU; the GPU tests check the fused device lookup+gather kernel
against a plain PyTorch gather of the same pages.
"""
import numpy as np
import pytest

from alluxio_amd.ops.native import lib


def _key(fid, idx):
    return (fid << 24) | idx


def test_host_put_get_erase_evict():
    C = lib()
    pc = C.PageCache(0, 8 * 4096, 4096, False)
    assert pc.slots == 8 and pc.used == 0
    pages = {i: np.random.default_rng(i).integers(0, 256, 4096, dtype=np.uint8) for i in range(12)}
    for i in range(8):
        assert pc.put_bytes(_key(1, i), pages[i], False) == []
    assert pc.used == 8
    with pytest.raises(Exception):
        pc.put_bytes(_key(1, 8), pages[8], False)          # full, eviction off
    assert pc.get_bytes(_key(1, 3), 100, 50) == pages[3][100:150].tobytes()
    assert pc.get_bytes(_key(2, 3), 0, 10) is None
    # touch 0..6 (host gets bump recency): page 7 is the LRU victim
    for i in range(7):
        assert pc.lookup(_key(1, i))[0] >= 0
    ev = pc.put_bytes(_key(1, 8), pages[8], True)
    assert ev == [_key(1, 7)] and not pc.contains(_key(1, 7)) and pc.contains(_key(1, 8))
    assert pc.erase(_key(1, 0)) and not pc.erase(_key(1, 0)) and pc.used == 7
    # overwrite in place keeps one slot
    pc.put_bytes(_key(1, 1), pages[11][:100], True)
    assert pc.lookup(_key(1, 1))[1] == 100 and pc.used == 7
    pc.clear()
    assert pc.used == 0 and not pc.contains(_key(1, 1))


def test_host_gather_and_tombstone_churn():
    C = lib()
    ps = 256
    pc = C.PageCache(0, 64 * ps, ps, False)
    rng = np.random.default_rng(7)
    live = {}
    for step in range(2000):                   # churn: tombstones force table rebuilds
        k = _key(int(rng.integers(1, 5)), int(rng.integers(0, 40)))
        if rng.random() < 0.3 and live:
            victim = list(live)[int(rng.integers(0, len(live)))]
            assert pc.erase(victim)
            del live[victim]
            continue
        data = rng.integers(0, 256, int(rng.integers(1, ps + 1)), dtype=np.uint8)
        for e in pc.put_bytes(k, data, True):
            live.pop(e, None)
        live[k] = data
    assert pc.used == len(live)
    keys = list(live)[:20] + [_key(99, 1)]
    dst = np.zeros((len(keys), ps), dtype=np.uint8)
    slots = pc.gather_host_keys(keys, dst.ctypes.data, ps, 0)
    assert slots[-1] == -1
    for i, k in enumerate(keys[:-1]):
        assert slots[i] >= 0
        assert np.array_equal(dst[i, :len(live[k])], live[k])


@pytest.mark.gpu
def test_device_gather_matches_torch(gpu):
    import torch
    C = lib()
    ps = 64 << 10
    n_pages = 96
    pc = C.PageCache(0, n_pages * ps, ps, True)
    assert pc.on_device
    src = torch.randint(0, 256, (n_pages, ps), dtype=torch.uint8, device=gpu)
    stream = torch.cuda.current_stream().cuda_stream
    for i in range(n_pages):
        ln = ps if i % 5 else ps - 4096 * (i % 7 + 1)
        pc.put(_key(3, i), src[i].data_ptr(), ln, 1, stream, False)
    torch.cuda.synchronize()
    # device-generated keys (a sampler on the GPU): pages 0..n-1 shuffled + misses
    perm = torch.randperm(n_pages + 8, device=gpu)
    keys = ((torch.full_like(perm, 3) << 24) | perm).to(torch.int64)
    n = keys.numel()
    out = torch.zeros((n, ps), dtype=torch.uint8, device=gpu)
    slot = torch.empty(n, dtype=torch.int32, device=gpu)
    lens = torch.empty(n, dtype=torch.int32, device=gpu)
    pc.gather(keys.data_ptr(), n, out.data_ptr(), ps, slot.data_ptr(), lens.data_ptr(), stream)
    torch.cuda.synchronize()
    p = perm.cpu()
    for r in range(n):
        i = int(p[r])
        if i >= n_pages:
            assert int(slot[r]) == -1 and int(lens[r]) == 0
            continue
        ln = ps if i % 5 else ps - 4096 * (i % 7 + 1)
        assert int(lens[r]) == ln
        assert torch.equal(out[r, :ln], src[i, :ln]), r
    # evict after device gathers: device stamps take part in the LRU choice
    hot = perm[:8].cpu().tolist()
    hot_keys = torch.tensor([(3 << 24) | k for k in hot if k < n_pages], dtype=torch.int64, device=gpu)
    for _ in range(3):
        pc.gather(hot_keys.data_ptr(), hot_keys.numel(), out.data_ptr(), ps, slot.data_ptr(), lens.data_ptr(),
                  stream)
    ev = pc.put(_key(4, 0), src[0].data_ptr(), ps, 1, stream, True)
    assert ev and not (set(ev) & set(hot_keys.cpu().tolist()))
    torch.cuda.synchronize()


def test_host_put_many_matches_put_and_evicts():
    C = lib()
    ps = 4096
    pc = C.PageCache(0, 16 * ps, ps, False)
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, (12, ps), dtype=np.uint8)
    keys = [_key(3, i) for i in range(12)]
    assert pc.put_many(keys, buf.ctypes.data, ps, ps, 0, 0, False) == []
    assert pc.used == 12
    for i in (0, 5, 11):
        assert pc.get_bytes(keys[i], 0, ps) == buf[i].tobytes()
    # stride 0 repeats one source page; overflowing the 16 slots evicts the LRU pages
    more = [_key(4, i) for i in range(8)]
    with pytest.raises(Exception):
        pc.put_many(more, buf.ctypes.data, 0, ps, 0, 0, False)
    ev = pc.put_many([_key(5, i) for i in range(8)], buf[2].ctypes.data, 0, ps, 0, 0, True)
    assert len(ev) >= 4 and all(pc.contains(k) is False for k in ev)
    for i in range(8):
        assert pc.get_bytes(_key(5, i), 0, ps) == buf[2].tobytes()


def test_host_put_many_is_atomic_and_dedups():
    C = lib()
    ps = 4096
    pc = C.PageCache(0, 8 * ps, ps, False)
    rng = np.random.default_rng(8)
    buf = rng.integers(0, 256, (10, ps), dtype=np.uint8)
    assert pc.put_many([_key(1, i) for i in range(6)], buf.ctypes.data, ps, ps, 0, 0, False) == []
    # 4 new keys do not fit the 2 free slots: nothing changes
    with pytest.raises(Exception):
        pc.put_many([_key(2, i) for i in range(4)], buf.ctypes.data, ps, ps, 0, 0, False)
    assert pc.used == 6 and not any(pc.contains(_key(2, i)) for i in range(4))
    # a repeated key keeps its LAST source, and only takes one slot
    assert pc.put_many([_key(3, 0), _key(3, 1), _key(3, 0)], buf.ctypes.data, ps, ps, 0, 0, False) == []
    assert pc.used == 8
    assert pc.get_bytes(_key(3, 0), 0, ps) == buf[2].tobytes()
    assert pc.get_bytes(_key(3, 1), 0, ps) == buf[1].tobytes()


def test_host_read_segments():
    C = lib()
    ps = 4096
    pc = C.PageCache(0, 8 * ps, ps, False)
    rng = np.random.default_rng(9)
    buf = rng.integers(0, 256, (4, ps), dtype=np.uint8)
    pc.put_many([_key(1, i) for i in range(4)], buf.ctypes.data, ps, ps, 0, 0, False)
    pc.put_bytes(_key(1, 9), buf[0][:100], False)
    out = np.zeros(3 * ps, dtype=np.uint8)
    base = out.ctypes.data
    missed = pc.read_segments([_key(1, 2), _key(1, 7), _key(1, 0), _key(1, 9)], [10, 0, 0, 50],
                              [ps - 10, 5, ps, 60], [base, base + 4000, base + ps, base + 2 * ps], 0, 0)
    assert missed == [1, 3]           # absent page; range past a short page's valid bytes
    assert np.array_equal(out[:ps - 10], buf[2][10:]) and np.array_equal(out[ps:2 * ps], buf[0])
    assert not out[2 * ps:].any()


@pytest.mark.gpu
def test_device_put_many_matches_torch(gpu):
    import torch
    C = lib()
    ps, n = 8192, 300
    pc = C.PageCache(0, 512 * ps, ps, True)
    src = torch.randint(0, 256, (n, ps), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    keys = [_key(9, i) for i in range(n)]
    assert pc.put_many(keys, src.data_ptr(), ps, ps, 1, stream, False) == []
    out = torch.empty_like(src)
    kd = torch.tensor(keys, dtype=torch.int64, device="cuda")
    so = torch.empty(n, dtype=torch.int32, device="cuda")
    lo = torch.empty(n, dtype=torch.int32, device="cuda")
    pc.gather(kd.data_ptr(), n, out.data_ptr(), ps, so.data_ptr(), lo.data_ptr(), stream)
    torch.cuda.synchronize()
    assert bool((so >= 0).all()) and torch.equal(out, src)


def _ref_check(pc, src_rows, expect: dict, ps, gpu):
    """Every expected key gathers to its source row (byte-exact, device lookup) and reads back
    through the host mirror (pulled from the device table)."""
    import torch
    keys = list(expect)
    kd = torch.tensor(keys, dtype=torch.int64, device=gpu)
    out = torch.empty((len(keys), ps), dtype=torch.uint8, device=gpu)
    so = torch.empty(len(keys), dtype=torch.int32, device=gpu)
    lo = torch.empty(len(keys), dtype=torch.int32, device=gpu)
    stream = torch.cuda.current_stream().cuda_stream
    pc.gather(kd.data_ptr(), len(keys), out.data_ptr(), ps, so.data_ptr(), lo.data_ptr(), stream)
    torch.cuda.synchronize()
    assert bool((so >= 0).all()) and bool((lo == ps).all())
    rows = torch.tensor([expect[k] for k in keys], device=gpu)
    assert torch.equal(out, src_rows[rows])
    for k in keys[:5]:
        assert pc.get_bytes(k, 0, 64) == src_rows[expect[k], :64].cpu().numpy().tobytes()


@pytest.mark.gpu
def test_device_put_many_device_keys_matches_reference(gpu):
    """K9 device put path (page_cache_put.hip): device-resident keys are probed/claimed, assigned
    (free stack, then CLOCK eviction) and filled on the GPU; checked byte-for-byte against a
    Python model of the cache, including duplicates (last wins), all-or-nothing overflow with
    evict=false, eviction of a full cache, and CLOCK's second chance for pages touched after
    insertion."""
    import torch
    C = lib()
    ps, nslots = 4096, 256
    pc = C.PageCache(0, nslots * ps, ps, True)
    src = torch.randint(0, 256, (1024, ps), dtype=torch.uint8, device=gpu)
    stream = torch.cuda.current_stream().cuda_stream
    model = {}

    def put(keys, rows, evict):
        kd = torch.tensor(keys, dtype=torch.int64, device=gpu)
        rowsel = src[torch.tensor(rows, device=gpu)].contiguous()
        ev = pc.put_many_device(kd.data_ptr(), len(keys), rowsel.data_ptr(), ps, ps, 1, stream, evict)
        torch.cuda.synchronize()
        for k, r in zip(keys, rows):
            model[k] = r
        for k in ev:
            model.pop(k, None)
        return ev

    assert put([_key(1, i) for i in range(200)], list(range(200)), False) == []
    assert pc.device_owned and pc.used == 200
    _ref_check(pc, src, model, ps, gpu)
    # duplicates: the last occurrence wins and takes one slot
    assert put([_key(2, 0), _key(2, 1), _key(2, 0)], [300, 301, 302], False) == []
    assert model[_key(2, 0)] == 302 and pc.used == 202
    _ref_check(pc, src, model, ps, gpu)
    # evict=false overflow: 100 fresh keys, 54 free slots -> nothing changes
    kd = torch.tensor([_key(3, i) for i in range(100)], dtype=torch.int64, device=gpu)
    with pytest.raises(Exception):
        pc.put_many_device(kd.data_ptr(), 100, src.data_ptr(), ps, ps, 1, stream, False)
    assert pc.used == 202 and not any(pc.contains(_key(3, i)) for i in range(100))
    _ref_check(pc, src, model, ps, gpu)
    # hot pages: touched (gathered) after insertion -> CLOCK second chance
    hot = [_key(1, i) for i in range(0, 200, 10)]
    hk = torch.tensor(hot, dtype=torch.int64, device=gpu)
    o = torch.empty((len(hot), ps), dtype=torch.uint8, device=gpu)
    so = torch.empty(len(hot), dtype=torch.int32, device=gpu)
    pc.gather(hk.data_ptr(), len(hot), o.data_ptr(), ps, so.data_ptr(), so.data_ptr(), stream)
    torch.cuda.synchronize()
    ev = put([_key(4, i) for i in range(100)], list(range(400, 500)), True)
    assert len(ev) == 202 + 100 - nslots and pc.used == nslots
    assert not set(ev) & set(hot)
    assert not any(pc.contains(k) for k in ev)
    _ref_check(pc, src, model, ps, gpu)
    # a batch as large as the cache replaces everything
    ev = put([_key(5, i) for i in range(nslots)], list(range(500, 500 + nslots)), True)
    assert len(ev) == nslots and set(model) == {_key(5, i) for i in range(nslots)}
    _ref_check(pc, src, model, ps, gpu)
    # host-side operations after device puts see the device table (mirror pulled back)
    assert pc.erase(_key(5, 3)) and not pc.contains(_key(5, 3))
    model.pop(_key(5, 3))
    assert pc.used == nslots - 1
    pc.put(_key(6, 0), src[7].data_ptr(), ps, 1, stream, False)
    model[_key(6, 0)] = 7
    # ... and a device put after host changes sees them (mirror pushed)
    ev = put([_key(7, i) for i in range(10)], list(range(900, 910)), True)
    assert len(ev) == 10 and pc.used == nslots
    _ref_check(pc, src, model, ps, gpu)
