"""K4-K7 on the device (csrc/evict_alloc.hip): the grid-wide byte-weighted eviction select and the
bitmap page allocator against host references, and the BlockStore's device-resident annotator
driving real evictions at arena scale (~150k blocks, the page count of a 288 GB arena at 2 MiB).

Reference behaviour: TieredBlockStore.freeSpaceInternal walks the annotator order (LRU /
LRFUAnnotator.java:81-95) until enough bytes are free (TieredBlockStore.java:740-815); the
allocator reserves space in a dir (MaxFreeAllocator.java:42-110).
"""
import numpy as np
import pytest

from alluxio_amd.ops.native import lib

pytestmark = pytest.mark.gpu
KB = 1 << 10


def _host_select(keys, nbytes, need):
    """Smallest keys first until >= need bytes (ties: any order) -> (set, bytes)."""
    order = np.argsort(keys, kind="stable")
    csum = np.cumsum(nbytes[order])
    k = int(np.searchsorted(csum, need)) + 1 if need <= csum[-1] else len(order)
    return set(order[:k].tolist()), int(csum[k - 1])


def _keys(crf, last, now, step, att, policy):
    age = (now - last).astype(np.float64)
    if policy == 0:
        return 0xFFFFFFFE - np.minimum(age, 0xFFFFFFFE)
    return crf.astype(np.float64) * np.power(1.0 / att, age * step)


@pytest.mark.parametrize("n", [5000, 150_000])
@pytest.mark.parametrize("policy", [0, 1])
def test_grid_select_matches_host(gpu, n, policy):
    C = lib()
    rng = np.random.default_rng(n + policy)
    crf = (rng.random(n) * 10).astype(np.float32)
    # distinct LRU ages; LRFU ages small enough that decayed CRFs stay distinct (no underflow)
    last = (rng.permutation(n).astype(np.uint64) * 3) if policy == 0 else (100 - rng.integers(0, 40, n)).astype(np.uint64)
    nbytes = (rng.integers(1, 33, n).astype(np.uint64) << 21)   # page-rounded footprints
    ev = (rng.random(n) > 0.2).astype(np.uint8)
    now = int(last.max()) + 10
    need = int(nbytes[ev == 1].sum() // 3)
    got, freed = C.evict_select_device(crf.tolist(), last.tolist(), nbytes.tolist(), ev.tolist(), now,
                                       0.25, 2.0, policy, need)
    got = set(got)
    assert all(ev[i] for i in got)
    assert freed == int(nbytes[list(got)].sum()) and freed >= need
    idx = np.nonzero(ev)[0]
    want, want_bytes = _host_select(_keys(crf[idx], last[idx], now, 0.25, 2.0, policy), nbytes[idx], need)
    want = {int(idx[i]) for i in want}
    if policy == 0:
        assert got == want          # distinct integer keys: exactly the host set
    else:                           # float keys: same set up to rounding ties at the threshold
        assert len(got ^ want) <= 4 and abs(freed - want_bytes) <= int(nbytes.max()) * 2


def test_grid_select_everything_and_nothing(gpu):
    C = lib()
    n = 3000
    nbytes = [2 << 20] * n
    got, freed = C.evict_select_device([0.0] * n, list(range(n)), nbytes, [1] * n, n, 0.25, 2.0, 0, 10 ** 15)
    assert sorted(got) == list(range(n)) and freed == sum(nbytes)
    got, freed = C.evict_select_device([0.0] * n, list(range(n)), nbytes, [0] * n, n, 0.25, 2.0, 0, 1)
    assert got == [] and freed == 0


@pytest.mark.parametrize("npages,want", [(150_000, 1), (150_000, 37_000), (150_000, 10 ** 6), (64 * 9 + 5, 100)])
def test_page_alloc_matches_host(gpu, npages, want):
    C = lib()
    rng = np.random.default_rng(npages + want)
    free = rng.random(npages) < 0.4
    words = np.zeros((npages + 63) // 64, dtype=np.uint64)
    for p in np.nonzero(free)[0]:
        words[p >> 6] |= np.uint64(1) << np.uint64(p & 63)
    pages, after = C.page_alloc_device(words.tolist(), want)
    expect = np.nonzero(free)[0][:want]
    assert pages == expect.tolist()
    left = free.copy()
    left[expect] = False
    words2 = np.zeros_like(words)
    for p in np.nonzero(left)[0]:
        words2[p >> 6] |= np.uint64(1) << np.uint64(p & 63)
    assert np.array_equal(np.array(after, dtype=np.uint64), words2)


def _device_store(npages, page, policy=0, step=0.25):
    import torch
    C = lib()
    arena = torch.empty(npages * page, dtype=torch.uint8, device="cuda")
    d = C.DirSpec()
    d.tier, d.tier_alias, d.medium, d.kind = 0, "MEM", "HBM", C.DirKind.DEVICE
    d.base, d.capacity, d.page_size, d.device = arena.data_ptr(), arena.numel(), page, 0
    s = C.BlockStore([d], annotator=policy, alloc_policy=0, lrfu_step=step, device=0)
    s._arena = arena
    return s


def test_store_device_eviction_at_arena_scale(gpu):
    """150k one-page blocks created in bulk (K7 claims their pages), committed, a random tenth
    re-accessed; the device select equals the CPU sort and free_space evicts exactly that set."""
    page = 4 * KB
    n = 150_000
    s = _device_store(n + 64, page)
    s.set_use_device_alloc(True, 64)
    ids = list(range(1, n + 1))
    dirs = s.create_blocks(7, ids, 0, "", [page] * n, False)
    assert set(dirs) == {0}
    st = s.evict_stats()
    assert st["device_allocs"] == 1 and st["device_alloc_pages"] == n
    for b in ids:
        s.commit_block(7, b)
    rng = np.random.default_rng(5)
    hot = rng.choice(n, n // 10, replace=False) + 1
    s.access_blocks(hot.tolist())
    need = 20_000 * page
    dev = s.select_for_bench(0, need, True)
    cpu = s.select_for_bench(0, need, False)
    assert len(dev) == 20_000 and set(dev) == set(cpu)
    assert not set(dev) & set(hot.tolist())     # re-accessed blocks are hot
    # lock one of the victims: it must survive a real eviction
    locked = cpu[0]
    lk = s.lock_block(9, locked)
    gone = set(s.free_space(9, (64 + 20_000) * page, 0, -1))
    s.unlock(lk)
    assert locked not in gone and len(gone) >= 20_000
    assert set(cpu[1:]) <= gone
    st = s.evict_stats()
    assert st["device_selections"] >= 2 and st["annotation_updates"] >= n


def test_store_device_lrfu_and_growth(gpu):
    """LRFU on the device annotator; slot arrays grow past their first allocation mid-run.
    (A small step keeps 40k ticks of decay representable: with the default 0.25 every CRF
    underflows to 0 -- as in the reference's double arithmetic -- and the order is all ties.)"""
    page = 4 * KB
    n = 40_000
    s = _device_store(n + 16, page, policy=1, step=1e-4)
    for b in range(1, n + 1):
        s.create_block(1, b, 0, "", page, False, False)
        s.commit_block(1, b)
        if b == 10_000:
            s.select_for_bench(0, page, True)    # first device arrays (16k slots)
    freq = np.random.default_rng(1).integers(0, 4, n)
    for k in range(1, 4):
        s.access_blocks([b + 1 for b in np.nonzero(freq >= k)[0].tolist()])
    need = 5000 * page
    dev, cpu = set(s.select_for_bench(0, need, True)), set(s.select_for_bench(0, need, False))
    assert len(dev ^ cpu) <= 8
    assert all(freq[b - 1] == 0 for b in dev)   # never-re-accessed blocks go first


def test_bulk_create_then_abort_returns_pages(gpu):
    page = 64 * KB
    s = _device_store(1024, page)
    s.set_use_device_alloc(True, 64)
    before = s.dir_available(0)
    s.create_blocks(3, list(range(100, 400)), 0, "", [page * 2] * 300, False)
    assert s.dir_available(0) == before - 600 * page
    s.cleanup_session(3)
    assert s.dir_available(0) == before


def test_tier_order_device_matches_host(gpu):
    """K8: the k coldest / hottest blocks of a tier from the device select (unit weights, dir mask,
    inverted keys for hottest) equal the host's full sort."""
    import torch
    C = lib()
    page = 4 * KB
    arenas, specs = [], []
    for tier in (0, 1):
        a = torch.empty(30_000 * page, dtype=torch.uint8, device="cuda")
        d = C.DirSpec()
        d.tier, d.tier_alias, d.medium, d.kind = tier, ("MEM", "SSD")[tier], "HBM", C.DirKind.DEVICE
        d.base, d.capacity, d.page_size, d.device = a.data_ptr(), a.numel(), page, 0
        arenas.append(a)
        specs.append(d)
    s = C.BlockStore(specs, annotator=0, alloc_policy=0, device=0)
    n = 25_000
    for tier in (0, 1):
        ids = list(range(1 + tier * n, 1 + (tier + 1) * n))
        s.create_blocks(1, ids, tier, "", [page] * n, False)
        for b in ids:
            s.commit_block(1, b)
    rng = np.random.default_rng(9)
    s.access_blocks((rng.choice(2 * n, 5000, replace=False) + 1).tolist())
    for tier in (0, 1):
        for hottest in (False, True):
            dev = s.tier_order(tier, 100, hottest, True)
            host = s.tier_order(tier, 100, hottest, False)
            assert len(dev) == 100 and dev == host, (tier, hottest)
    keys = s.annotator_keys(s.tier_order(1, 10, True, True))
    assert keys == sorted(keys, reverse=True)


def test_bulk_ingest_into_hbm_and_gathered_crc(gpu, tmp_path):
    """BlockStore::ingest_files into an HBM dir (pinned staging halves, async H2D) round-trips the
    file bytes; checksum_blocks' single gathered CRC launch equals per-block checksum() and the
    host CRC32C of every page."""
    import torch
    C = lib()
    page = 128 * KB
    s = _device_store(2048, page)
    rng = np.random.default_rng(4)
    paths, lens, datas = [], [], []
    for i in range(300):
        n = int(rng.integers(1, 3 * page))
        d = rng.integers(0, 256, n, dtype=np.uint8)
        p = tmp_path / f"f{i}"
        p.write_bytes(d.tobytes())
        paths.append(str(p))
        lens.append(n)
        datas.append(d)
    ids = list(range(1000, 1300))
    staging = torch.empty(8 << 20, dtype=torch.uint8, pin_memory=True)
    st = s.ingest_files(5, ids, paths, [0] * 300, lens, staging.data_ptr(), staging.numel(), 8, 0)
    assert st == [0] * 300
    out = torch.empty(3 * page, dtype=torch.uint8, device="cuda")
    for b, d in zip(ids[::37], datas[::37]):
        s.read_batch([(b, 0, d.nbytes, out.data_ptr(), 1)], 0, True)
        assert np.array_equal(out[:d.nbytes].cpu().numpy(), d)
    crcs = s.checksum_blocks(ids + [999999])
    assert crcs[-1] == (0, [])
    assert all(c[0] == page for c in crcs[:-1])
    for b, d, (_, c) in zip(ids, datas, crcs):
        assert c == s.checksum(b, 0)
        assert c == [C.crc32c(d[o:o + page].tobytes()) for o in range(0, d.nbytes, page)]


def test_magazine_ingest_then_host_allocs_keep_pages_disjoint(gpu, tmp_path):
    """K7 device magazine: ingest_files claims its blocks' pages on the GPU (fused claim + scatter,
    no host page lists); host allocations then fill the dir, draining the magazine back into the
    host pool.  Every page ends up owned by exactly one block, the accounting adds up, and the
    ingested bytes are intact."""
    import torch
    C = lib()
    page = 64 * KB
    npages = 512
    s = _device_store(npages, page)
    s.set_use_device_alloc(True, 64)
    rng = np.random.default_rng(11)
    paths, lens, datas = [], [], []
    for i in range(150):
        n = int(rng.integers(1, 2 * page))
        d = rng.integers(0, 256, n, dtype=np.uint8)
        p = tmp_path / f"m{i}"
        p.write_bytes(d.tobytes())
        paths.append(str(p))
        lens.append(n)
        datas.append(d)
    ids = list(range(5000, 5150))
    staging = torch.empty(4 << 20, dtype=torch.uint8, pin_memory=True)
    assert s.ingest_files(5, ids, paths, [0] * 150, lens, staging.data_ptr(), staging.numel(), 4, 0) == [0] * 150
    used = sum((n + page - 1) // page for n in lens)
    st = s.evict_stats()
    assert st["device_alloc_pages"] >= used
    assert s.dir_available(0) == (npages - used) * page
    # host allocations (one page each) until the dir is full: the magazine is drained on demand
    b = 9000
    while True:
        try:
            s.create_block(6, b, 0, "", page, False, False)
        except Exception:
            break
        b += 1
    assert b - 9000 == npages - used and s.dir_available(0) == 0
    owned = []
    for blk in ids + list(range(9000, b)):
        pages = s.block_pages(blk)[0]
        owned += pages
    assert len(owned) == npages and sorted(owned) == list(range(npages))
    out = torch.empty(2 * page, dtype=torch.uint8, device="cuda")
    for blk, d in zip(ids, datas):
        s.read_batch([(blk, 0, d.nbytes, out.data_ptr(), 1)], 0, True)
        assert np.array_equal(out[:d.nbytes].cpu().numpy(), d), blk
    # freeing returns pages to the host pool; a second ingest claims again through a refill
    s.cleanup_session(6)
    assert s.dir_available(0) == (npages - used) * page
    ids2 = list(range(7000, 7040))
    assert s.ingest_files(8, ids2, paths[:40], [0] * 40, lens[:40], staging.data_ptr(), staging.numel(), 4, 0) == [0] * 40
    for blk, d in zip(ids2[::7], datas[:40:7]):
        s.read_batch([(blk, 0, d.nbytes, out.data_ptr(), 1)], 0, True)
        assert np.array_equal(out[:d.nbytes].cpu().numpy(), d)


@pytest.mark.parametrize("npages,nitems,want", [(512, 25, 2), (512, 150, 1), (150_064, 2000, 3), (4096, 4096, 1),
                                                (4096, 300, 20)])
def test_magazine_concurrent_claims_exact(gpu, npages, nitems, want):
    """Many items claiming from one magazine at once (one wave each, CAS on bitmap words): every
    page is handed out at most once, every item gets its pages while the magazine has them, and
    the device bitmap keeps exactly the rest."""
    s = _device_store(npages, 64 * KB)
    moved = s.mag_refill(0, nitems * want)
    assert s.mag_device_count(0) == moved >= min(npages, nitems * want)
    got = s.mag_claim_many(0, [want] * nitems)
    flat = [p for g in got for p in g]
    assert len(flat) == len(set(flat)) and all(0 <= p < npages for p in flat)
    assert len(flat) == min(moved, nitems * want)
    if moved >= nitems * want:
        assert all(len(g) == want for g in got)
    assert s.mag_device_count(0) == moved - len(flat) == s.mag_pages(0)
    assert s.mag_drain(0) == moved - len(flat) and s.mag_device_count(0) == 0


def test_magazine_accounting_mixed_workload(gpu, tmp_path):
    """with the K7 magazine on by default, page accounting must survive a mixed
    workload -- bulk ingests and bulk creates (device claims), single creates (host scan, drains
    the magazine on demand), aborts, removes, evictions that demote into a second HBM tier --
    with check_pages (host pool + magazine bitmap + block page lists partition each arena, the
    device bitmap holds exactly mag_pages) clean after every step, and the ingested bytes intact."""
    import torch
    C = lib()
    page = 64 * KB
    arenas, specs = [], []
    for tier, n in ((0, 1024), (1, 2048)):
        a = torch.empty(n * page, dtype=torch.uint8, device="cuda")
        d = C.DirSpec()
        d.tier, d.tier_alias, d.medium, d.kind = tier, ("MEM", "SSD")[tier], "HBM", C.DirKind.DEVICE
        d.base, d.capacity, d.page_size, d.device = a.data_ptr(), a.numel(), page, 0
        arenas.append(a)
        specs.append(d)
    s = C.BlockStore(specs, annotator=0, alloc_policy=0, device=0)
    s._arenas = arenas
    s.set_use_device_alloc(True, 8)
    s.set_demote_on_evict(True)
    rng = np.random.default_rng(23)
    staging = torch.empty(4 << 20, dtype=torch.uint8, pin_memory=True)
    out = torch.empty(3 * page, dtype=torch.uint8, device="cuda")
    data: dict[int, np.ndarray] = {}
    committed: list[int] = []
    nxt = [100]

    def new_ids(k):
        ids = list(range(nxt[0], nxt[0] + k))
        nxt[0] += k
        return ids

    def check(step):
        for d in range(2):
            assert s.check_pages(d) == "", (step, d, s.check_pages(d))

    for step in range(60):
        op = step % 6
        if op == 0:                                    # bulk UFS ingest (device claim + scatter)
            ids = new_ids(int(rng.integers(20, 80)))
            paths, lens = [], []
            for b in ids:
                n = int(rng.integers(1, 3 * page))
                d = rng.integers(0, 256, n, dtype=np.uint8)
                p = tmp_path / f"b{b}"
                p.write_bytes(d.tobytes())
                paths.append(str(p))
                lens.append(n)
                data[b] = d
            st = s.ingest_files(5, ids, paths, [0] * len(ids), lens, staging.data_ptr(), staging.numel(), 4, 0)
            for b, code in zip(ids, st):
                if code == 0:
                    committed.append(b)
                else:
                    data.pop(b)
        elif op == 1:                                  # bulk create, then commit or abort
            ids = new_ids(int(rng.integers(64, 120)))          # >= kDeviceAllocMinBlocks: K7 claims
            try:
                s.create_blocks(7, ids, 0, "", [page * int(rng.integers(1, 3))] * len(ids), True)
            except Exception:  # noqa: BLE001 - the tier may be full of locked/temp blocks
                pass
            if step % 12 == 1:
                s.cleanup_session(7)
            else:
                for b in ids:
                    if s.has_temp_block(b):
                        s.commit_block(7, b)
                        committed.append(b)
        elif op == 2:                                  # single creates on the host scan
            for b in new_ids(int(rng.integers(5, 30))):
                try:
                    s.create_block(8, b, 0, "", page, True, False)
                    s.commit_block(8, b)
                    committed.append(b)
                except Exception:  # noqa: BLE001
                    break
        elif op == 3 and committed:                    # removes
            for b in rng.choice(committed, min(len(committed), 15), replace=False).tolist():
                if s.has_block(b):
                    s.remove_block(10, b)
                committed.remove(b)
                data.pop(b, None)
        elif op == 4:                                  # eviction (demotes into tier 1)
            s.free_space(9, int(rng.integers(50, 300)) * page, 0, -1)
        elif op == 5 and committed:                    # accesses reorder the victims
            s.access_blocks(rng.choice(committed, min(len(committed), 40), replace=False).tolist())
        check(step)
    live = [b for b in data if s.has_block(b)]
    assert live
    for b in live[::5]:
        d = data[b]
        s.read_batch([(b, 0, d.nbytes, out.data_ptr(), 1)], 0, True)
        assert np.array_equal(out[:d.nbytes].cpu().numpy(), d), b
    assert s.evict_stats()["device_alloc_pages"] > 0


def test_tier_moves_between_hbm_and_mapped_dram_are_byte_exact(gpu):
    """Tier moves between an HBM arena and a GPU-mapped (hipHostRegister) DRAM arena run as one
    batched copy kernel per move on the caller's move stream (not runtime copyBuffer per page
    run); demoted and promoted-back blocks keep their bytes, including a partial last page."""
    import torch
    C = lib()
    page = 64 * KB
    dev = torch.empty(64 * page, dtype=torch.uint8, device="cuda")
    host = np.zeros(256 * page, dtype=np.uint8)
    assert C.host_register(host.ctypes.data, host.nbytes)
    try:
        specs = []
        for tier, (base, cap, kind, medium) in enumerate([(dev.data_ptr(), dev.numel(), C.DirKind.DEVICE, "HBM"),
                                                          (host.ctypes.data, host.nbytes, C.DirKind.HOST, "DRAM")]):
            d = C.DirSpec()
            d.tier, d.tier_alias, d.medium, d.kind = tier, ("MEM", "SSD")[tier], medium, kind
            d.base, d.capacity, d.page_size, d.device = base, cap, page, 0
            specs.append(d)
        s = C.BlockStore(specs, annotator=0, alloc_policy=0, device=0)
        rng = np.random.default_rng(31)
        src = torch.empty(4 * page, dtype=torch.uint8).pin_memory()
        blobs = {}
        ids = list(range(1, 9))
        for b in ids:
            n = 4 * page - (b * 777 if b % 2 else 0)          # odd blocks end mid-page
            data = rng.integers(0, 256, n, dtype=np.uint8)
            src[:n].copy_(torch.from_numpy(data))
            s.create_block(5, b, 0, "", n)
            s.write(5, b, 0, src.data_ptr(), n, 0)
            s.commit_block(5, b)
            blobs[b] = data
        before = s.evict_stats()["batched_moves"]
        moved = s.move_blocks(5, ids[:5], 1)
        assert sorted(moved) == ids[:5]
        assert all(s.block_info(b).tier == 1 for b in ids[:5])
        back = s.move_blocks(5, ids[:3], 0)
        assert sorted(back) == ids[:3]
        out = torch.empty(4 * page, dtype=torch.uint8).pin_memory()
        for b in ids:
            n = len(blobs[b])
            out.zero_()
            s.read(b, 0, n, out.data_ptr(), 0)
            assert np.array_equal(out[:n].numpy(), blobs[b]), b
        assert s.evict_stats()["batched_moves"] >= before + 2
        del s
    finally:
        C.host_unregister(host.ctypes.data)


def test_store_churn_across_a_thread_pool_keeps_hip_streams_flat(gpu):
    """100 stores created, used for tier moves and destroyed across a pool of 4 threads: every
    move runs on the thread's stream of the device (thread_stream_on), so the process creates at
    most one stream per (thread, device) -- not one per store, as the per-store cache did
    (move_stream leaked a stream per store and could reuse a stale one)."""
    import concurrent.futures as cf

    import torch
    C = lib()
    page = 64 * KB
    dev = torch.empty(16 * page, dtype=torch.uint8, device="cuda")
    host = np.zeros(32 * page, dtype=np.uint8)
    assert C.host_register(host.ctypes.data, host.nbytes)
    try:
        src = torch.empty(2 * page, dtype=torch.uint8).pin_memory()
        src.fill_(7)

        def one(i):
            specs = []
            for tier, (base, cap, kind, medium) in enumerate([(dev.data_ptr(), dev.numel(), C.DirKind.DEVICE, "HBM"),
                                                              (host.ctypes.data, host.nbytes, C.DirKind.HOST, "DRAM")]):
                d = C.DirSpec()
                d.tier, d.tier_alias, d.medium, d.kind = tier, ("MEM", "SSD")[tier], medium, kind
                d.base, d.capacity, d.page_size, d.device = base, cap, page, 0
                specs.append(d)
            s = C.BlockStore(specs, annotator=0, alloc_policy=0, device=0)
            s.create_block(5, 1, 0, "", 2 * page)
            s.write(5, 1, 0, src.data_ptr(), 2 * page, 0)
            s.commit_block(5, 1)
            assert s.move_blocks(5, [1], 1) == [1]
            assert s.move_block(5, 1, 0, "", True) >= 0
            del s
            return i

        before = C.thread_streams_created()
        with cf.ThreadPoolExecutor(4) as ex:
            assert sorted(ex.map(one, range(100))) == list(range(100))
        assert C.thread_streams_created() - before <= 4
    finally:
        C.host_unregister(host.ctypes.data)
