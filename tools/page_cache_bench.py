#!/usr/bin/env python3
"""K9 page-cache gather throughput on one MI355X.

Times the fused device hash lookup + page copy (``_C.PageCache.gather`` ->
``page_lookup_gather_kernel`` in csrc/kernels.hip) for random page keys generated on the GPU,
against ``torch.index_select`` over the same arena with the slot indices already resolved (no lookup
at all) and a contiguous ``copy_`` of the same byte count (the HBM copy roof).  The reference's
client cache serves one page per ``get`` call from a file or heap store
(core/client/fs/src/main/java/alluxio/client/file/cache/LocalCacheManager.java:360).

Run: python tools/page_cache_bench.py [--page-sizes 4k,64k,512k,2m] [--cache 8g] [--out f.jsonl]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _DevArray:
    """A raw device allocation exposed to torch (the cache arena, owned by the native cache)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3}


def _time_ms(fn, iters):
    import torch
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--page-sizes", default="4k,64k,512k,2m")
    ap.add_argument("--cache", default="8g", help="arena bytes (capped by --max-pages)")
    ap.add_argument("--max-pages", type=int, default=1 << 18)
    ap.add_argument("--batch-bytes", default="1g", help="bytes gathered per launch")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", choices=["auto", "both"], default="auto",
                    help="both: time the wave-per-request and the chunked kernel at every page size")
    ap.add_argument("--wave-variants", default="0",
                    help="wave-kernel variants timed with --variants both (see set_page_gather_wave_variant)")
    ap.add_argument("--chunk-variants", default="0",
                    help="chunk-kernel variants timed with --variants both (see set_page_gather_chunk_variant)")
    ap.add_argument("--passes", type=int, default=1, help="repeat the whole run list; every pass is reported")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    import torch
    from alluxio_amd.ops.native import lib
    from alluxio_amd.utils.format import parse_space_size
    C = lib()
    assert torch.cuda.is_available(), "needs a HIP device"
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    runs = [(parse_space_size(p), None) for p in a.page_sizes.split(",")]
    if a.variants == "both":
        waves = ["wave%s" % w for w in a.wave_variants.split(",")]
        chunks = ["chunk%s" % c for c in a.chunk_variants.split(",")]
        runs = [(ps, v) for ps, _ in runs for v in waves + chunks]
    # clocks and caches warm before the first timed case, so case order does not bias the sweep
    warm = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    warm2 = torch.empty_like(warm)
    for _ in range(50):
        warm2.copy_(warm)
    torch.cuda.synchronize()
    del warm, warm2
    for pas, (ps, variant) in [(p, r) for p in range(a.passes) for r in runs]:
        if variant is not None:
            C.set_page_gather_small_max(0 if variant.startswith("chunk") else 1 << 40)
            if variant.startswith("chunk"):
                C.set_page_gather_chunk_variant(int(variant[5:] or 0))
            else:
                C.set_page_gather_wave_variant(int(variant[4:]))
        slots = max(1, min(parse_space_size(a.cache) // ps, a.max_pages))
        pc = C.PageCache(0, slots * ps, ps, True)
        src = torch.zeros(ps, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        t_fill = time.perf_counter()
        pc.put_many([(1 << 24) | i for i in range(slots)], src.data_ptr(), 0, ps, 1, stream, False)
        fill_GBps = slots * ps / (time.perf_counter() - t_fill) / 1e9
        # device put path with device-resident keys (page_cache_put.hip): overwrite every page,
        # then replace the whole cache with new keys (CLOCK eviction of every slot)
        src_rows = torch.empty((slots, ps), dtype=torch.uint8, device=dev)    # distinct source pages
        dk = torch.arange(slots, device=dev, dtype=torch.int64) | (1 << 24)
        stride = ps
        torch.cuda.synchronize()
        t_dev = time.perf_counter()
        pc.put_many_device(dk.data_ptr(), slots, src_rows.data_ptr(), stride, ps, 1, stream, False)
        overwrite_GBps = slots * ps / (time.perf_counter() - t_dev) / 1e9
        dk2 = dk | (1 << 40)
        torch.cuda.synchronize()
        t_dev = time.perf_counter()
        ev = pc.put_many_device(dk2.data_ptr(), slots, src_rows.data_ptr(), stride, ps, 1, stream, True, True)
        evict_GBps = slots * ps / (time.perf_counter() - t_dev) / 1e9
        assert len(ev) == slots, len(ev)
        torch.cuda.synchronize()
        t_dev = time.perf_counter()
        pc.put_many_device(dk.data_ptr(), slots, src_rows.data_ptr(), stride, ps, 1, stream, True, True)
        evict2_GBps = slots * ps / (time.perf_counter() - t_dev) / 1e9
        del src_rows, dk2
        C.fill_pattern(pc.arena, slots * ps, 1234, 0, stream)      # distinct bytes in every page
        arena = torch.as_tensor(_DevArray(pc.arena, slots * ps), device=dev).view(slots, ps)
        n = max(1, min(parse_space_size(a.batch_bytes) // ps, 1 << 20))
        g = torch.Generator(device=dev)
        g.manual_seed(0)
        pages = torch.randint(0, slots, (n,), device=dev, generator=g)
        keys = (pages | (1 << 24)).contiguous()
        out = torch.empty((n, ps), dtype=torch.uint8, device=dev)
        so = torch.empty(n, dtype=torch.int32, device=dev)
        lo = torch.empty(n, dtype=torch.int32, device=dev)

        def gather():
            pc.gather(keys.data_ptr(), n, out.data_ptr(), ps, so.data_ptr(), lo.data_ptr(), stream)

        gather()
        torch.cuda.synchronize()
        idx = so.long()
        assert bool((idx >= 0).all()) and bool((lo == ps).all()), "lookup missed a cached page"
        check = min(n, 512)
        assert torch.equal(out[:check], arena.index_select(0, idx[:check])), "gathered bytes differ"
        for _ in range(2):
            gather()
        ms = _time_ms(gather, a.iters)
        out2 = torch.empty_like(out)
        ms_ix = _time_ms(lambda: torch.index_select(arena, 0, idx, out=out2), a.iters)
        flat = arena.view(-1)[: n * ps] if n <= slots else None
        ms_cp = _time_ms(lambda: out2.view(-1).copy_(flat), a.iters) if flat is not None else None
        nbytes = n * ps
        r = {"bench": "page_cache_gather", "pass": pas, "kernel": variant or "auto", "page_size": ps, "pages_cached": slots,
             "batch_pages": n, "batch_bytes": nbytes, "fused_lookup_gather_ms": round(ms, 4),
             "fused_GBps": round(nbytes / ms / 1e6, 1),
             "torch_index_select_resolved_ms": round(ms_ix, 4),
             "torch_index_select_GBps": round(nbytes / ms_ix / 1e6, 1),
             "contiguous_copy_GBps": round(nbytes / ms_cp / 1e6, 1) if ms_cp else None,
             "fill_put_many_GBps": round(fill_GBps, 1),
             "put_device_overwrite_GBps": round(overwrite_GBps, 1),
             "put_device_evict_all_GBps": round(evict_GBps, 1),
             "put_device_evict_all_2_GBps": round(evict2_GBps, 1),
             "verified": True}
        print(json.dumps(r), flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(json.dumps(r) + "\n")
        del arena, out, out2, flat
        del pc
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
