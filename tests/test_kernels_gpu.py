"""Numerics of the CDNA4 kernels against host references (gpu-marked).

Each HIP kernel is compared with a plain host implementation of the same op: byte-exact copy,
CRC32C vs the slicing-by-8 software CRC (itself pinned to the standard check value), LZ4 vs the
host codec (decode of host-encoded data, host-decode of device-encoded data), eviction selection
vs a sorted host reference.
"""
import os

import numpy as np
import pytest

from alluxio_amd.ops.native import lib

pytestmark = pytest.mark.gpu


def _t(nbytes, device, fill=None):
    import torch
    if fill is None:
        return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=device)
    return torch.full((nbytes,), fill, dtype=torch.uint8, device=device)


def test_batched_copy_exact(gpu):
    import torch
    C = lib()
    src = _t(48 << 20, gpu)
    dst = torch.zeros_like(src)
    rng = np.random.default_rng(0)
    segs = []
    off = 0
    # mixture of aligned, 4-B aligned and odd segments, small and large
    for n in [1, 3, 15, 16, 17, 4096, 4097, 65536 + 7, 1 << 20, (3 << 20) + 5, 7 << 20]:
        so = off + int(rng.integers(0, 3))
        segs.append((src.data_ptr() + so, dst.data_ptr() + so, n))
        off = so + n + 64
    C.batched_copy(segs, 0)
    torch.cuda.synchronize()
    for s, d, n in segs:
        o = s - src.data_ptr()
        assert torch.equal(src[o:o + n], dst[o:o + n])


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
def test_crc32c_matches_host(gpu, variant):
    import torch
    C = lib()
    C.set_crc_variant(variant)
    for nbytes, piece in [(1, 0), (15, 0), (1000, 0), (65536, 0), (4111, 0), ((2 << 20) + 13, 1 << 20),
                          (5 << 20, 2 << 20), (3 << 20, 64 << 10), ((1 << 20) + 4097, 300_001)]:
        t = _t(nbytes, gpu)
        host = t.cpu().numpy().tobytes()
        got = C.crc32c_device(t.data_ptr(), nbytes, piece, 0)
        p = piece or nbytes
        want = [C.crc32c(host[i:i + p]) for i in range(0, nbytes, p)]
        assert got == want, (variant, nbytes, piece)
    C.set_crc_variant(4)


def test_crc32c_device_pages_scattered(gpu):
    """The one-launch CRC of a block whose pages are scattered in the arena (the streamed commit
    CRC, BlockStore::checksum_async): page i read at base + pages[i] * page_bytes, the last page
    partial, equal to the host CRC32C of each page."""
    C = lib()
    C.set_crc_variant(4)
    for page_bytes, npages, tail in [(2 << 20, 12, 12345), (1 << 20, 9, 1), (300_001, 7, 77), (4096, 33, 4095)]:
        arena = _t(page_bytes * (npages + 5), gpu)
        host = arena.cpu().numpy().tobytes()
        pages = list(np.random.default_rng(page_bytes).permutation(npages + 5)[:npages])
        length = (npages - 1) * page_bytes + tail
        got = C.crc32c_device_pages(arena.data_ptr(), [int(p) for p in pages], length, page_bytes)
        want = []
        for i, p in enumerate(pages):
            n = min(page_bytes, length - i * page_bytes)
            want.append(C.crc32c(host[int(p) * page_bytes:int(p) * page_bytes + n]))
        assert got == want, (page_bytes, npages)


@pytest.mark.parametrize("variant", [-1] + list(range(27)))
def test_lz4_device_roundtrip(gpu, variant):
    import torch
    C = lib()
    C.set_lz4_decode_variant(variant)
    rng = np.random.default_rng(1)
    chunks = []
    far = os.urandom(20000)
    for i in range(20):
        n = int(rng.integers(1, 65536)) if i < 15 else 65536
        kind = i % 5
        if kind == 0:
            raw = rng.integers(0, 4, n, dtype=np.uint8).tobytes()         # compressible
        elif kind == 1:
            raw = os.urandom(n)                                            # incompressible
        elif kind == 2:
            raw = (b"alluxio-amd-" * (n // 12 + 1))[:n]                    # long matches
        elif kind == 3:
            raw = (far * 4)[:n]                                            # offsets of 20000 (beyond 8/16 KiB rings)
        else:
            raw = b"\x07" * (n // 2) + bytes(rng.integers(0, 3, n - n // 2, dtype=np.uint8))  # offset-1 run
        chunks.append(raw)
    # host-encoded -> device decode
    comp = [C.lz4_compress(c) for c in chunks]
    srcs = [torch.tensor(list(c), dtype=torch.uint8, device=gpu) if c else torch.zeros(1, dtype=torch.uint8, device=gpu)
            for c in comp]
    outs = [torch.zeros(65536, dtype=torch.uint8, device=gpu) for _ in chunks]
    sizes = C.lz4_device([(s.data_ptr(), o.data_ptr(), len(c), 65536) for s, o, c in zip(srcs, outs, comp)],
                         False, 0)
    for raw, o, sz in zip(chunks, outs, sizes):
        assert sz == len(raw)
        assert o[:sz].cpu().numpy().tobytes() == raw
    # truncated / undersized streams fail with a negative status (no fault, no overrun)
    bad = [(srcs[0].data_ptr(), outs[0].data_ptr(), max(1, len(comp[0]) - 3), 65536),
           (srcs[2].data_ptr(), outs[2].data_ptr(), len(comp[2]), max(1, len(chunks[2]) // 2))]
    assert all(sz < 0 for sz in C.lz4_device(bad, False, 0))
    # device encode (every encoder variant) -> host decode
    ins = [torch.tensor(list(c), dtype=torch.uint8, device=gpu) for c in chunks]
    cap = [C.lz4_compress_bound(len(c)) for c in chunks]
    for ev in (0, 1, 2, 3, 4):
        C.set_lz4_encode_variant(ev)
        enc = [torch.zeros(k, dtype=torch.uint8, device=gpu) for k in cap]
        sizes = C.lz4_device([(i.data_ptr(), e.data_ptr(), len(c), k) for i, e, c, k in zip(ins, enc, chunks, cap)],
                             True, 0)
        for raw, e, sz in zip(chunks, enc, sizes):
            assert sz > 0, ev
            assert C.lz4_decompress(e[:sz].cpu().numpy().tobytes(), len(raw)) == raw, ev
        # an output capacity too small for the stream fails cleanly
        small = C.lz4_device([(ins[1].data_ptr(), enc[1].data_ptr(), len(chunks[1]), max(1, len(chunks[1]) // 2))],
                             True, 0)
        assert small[0] < 0, ev
    C.set_lz4_encode_variant(4)
    C.set_lz4_decode_variant(-1)


@pytest.mark.parametrize("variant", [-1, 2, 17, 19, 20, 21, 22, 23, 24, 25, 26])
def test_lz4_device_unaligned_and_text(gpu, variant):
    """Unaligned source/destination addresses, text/CSV-shaped streams (many short sequences with
    small offsets: the window kernels' reference chains), long zero runs and incompressible tails."""
    import torch
    C = lib()
    C.set_lz4_decode_variant(variant)
    rng = np.random.default_rng(7)
    words = [b"alluxio", b"worker", b"block", b"hbm", b"page", b"read", b"\n", b",", b" "]
    text = b"".join(words[i] for i in rng.integers(0, len(words), 30000))
    csv = b"".join(b"%d,%s,%d\n" % (i, [b"GET", b"PUT"][i % 2], int(rng.integers(0, 999))) for i in range(6000))
    chunks = [text[:65536], csv[:65536], bytes(40000) + os.urandom(25536), text[:1000] + bytes(60000),
              os.urandom(3000) + text[:50000], b"ab" * 20000, text[:7], b""]
    comp = [C.lz4_compress(c) for c in chunks]
    base = torch.zeros(sum(len(c) + 64 for c in comp), dtype=torch.uint8, device=gpu)
    outs = torch.zeros(len(chunks) * 70000, dtype=torch.uint8, device=gpu)
    items, pos = [], 0
    for i, c in enumerate(comp):
        so = pos + 1 + i % 15
        if c:
            base[so:so + len(c)] = torch.tensor(list(c), dtype=torch.uint8, device=gpu)
        items.append((base.data_ptr() + so, outs.data_ptr() + i * 70000 + (3 * i) % 16, len(c), 65536))
        pos = so + len(c) + 16
    sizes = C.lz4_device(items, False, 0)
    host = outs.cpu().numpy().tobytes()
    for i, (raw, sz) in enumerate(zip(chunks, sizes)):
        o = i * 70000 + (3 * i) % 16
        assert sz == len(raw), (i, sz, len(raw))
        assert host[o:o + sz] == raw, i
        assert host[o + sz:o + sz + 8] == bytes(8), i   # nothing written past the output
    C.set_lz4_decode_variant(-1)


def _host_select(crf, last, nbytes, ev, now, step, att, policy, need):
    keys = []
    for i in range(len(crf)):
        if not ev[i]:
            continue
        age = max(0, now - last[i])
        if policy == 0:
            k = 0xFFFFFFFE - min(age, 0xFFFFFFFE)
        else:
            k = float(np.float32(crf[i]) * np.float32(np.power(np.float32(1.0 / att), np.float32(age * step))))
        keys.append((k, i))
    keys.sort()
    out, got = [], 0
    for k, i in keys:
        if got >= need:
            break
        out.append(i)
        got += nbytes[i]
    return out


@pytest.mark.parametrize("policy", [0, 1])
def test_evict_select_matches_host(gpu, policy):
    C = lib()
    rng = np.random.default_rng(2 + policy)
    n = 5000
    crf = rng.random(n).astype(np.float32) * 10
    # distinct keys: LRU ages are a permutation; LRFU ages stay small enough that the decayed CRFs
    # (crf * 0.5^(age/4)) do not underflow into ties at zero
    last = (rng.permutation(n).astype(np.uint64) * 3) if policy == 0 else \
        (100 - rng.integers(0, 40, n)).astype(np.uint64)
    nbytes = rng.integers(1, 64, n).astype(np.uint64) << 20
    ev = (rng.random(n) > 0.2).astype(np.uint8)
    now = int(last.max()) + 10
    need = int(nbytes[ev == 1].sum() // 3)
    got, freed = C.evict_select_device(crf.tolist(), last.tolist(), nbytes.tolist(), ev.tolist(), now,
                                       0.25, 2.0, policy, need)
    assert freed >= need
    assert all(ev[i] for i in got)
    want = _host_select(crf, last, nbytes, ev, now, 0.25, 2.0, policy, need)
    # same set up to ties at the threshold: the freed bytes stay within one block of the host set
    assert abs(int(freed) - int(nbytes[want].sum())) <= int(nbytes.max())
    assert len(set(got) ^ set(want)) <= 4


def test_fill_pattern_deterministic(gpu):
    import torch
    C = lib()
    a = torch.zeros(1 << 20, dtype=torch.uint8, device=gpu)
    b = torch.zeros(1 << 20, dtype=torch.uint8, device=gpu)
    C.fill_pattern(a.data_ptr(), a.numel(), 7, 0, 0)
    C.fill_pattern(b.data_ptr(), 1 << 19, 7, 0, 0)
    C.fill_pattern(b.data_ptr() + (1 << 19), 1 << 19, 7, (1 << 19) // 8, 0)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
