"""K7 magazine probe on the GPU: refill, claim for many items at once, check counts/disjointness."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from alluxio_amd.ops.native import lib  # noqa: E402

C = lib()
page = 64 << 10
for npages, nitems, want in ((512, 25, 2), (512, 150, 1), (150064, 2000, 3), (4096, 4096, 1)):
    arena = torch.empty(npages * page, dtype=torch.uint8, device="cuda")
    d = C.DirSpec()
    d.tier, d.tier_alias, d.medium, d.kind = 0, "MEM", "HBM", C.DirKind.DEVICE
    d.base, d.capacity, d.page_size, d.device = arena.data_ptr(), arena.numel(), page, 0
    s = C.BlockStore([d], annotator=0, alloc_policy=0, device=0)
    moved = s.mag_refill(0, nitems * want)
    before = s.mag_device_count(0)
    got = s.mag_claim_many(0, [want] * nitems)
    flat = [p for g in got for p in g]
    after = s.mag_device_count(0)
    r = {"npages": npages, "items": nitems, "want": want, "moved": moved, "dev_before": before,
         "claimed": len(flat), "distinct": len(set(flat)), "short": sum(1 for g in got if len(g) < want),
         "dev_after": after, "mag_pages": s.mag_pages(0), "drained": s.mag_drain(0)}
    print(json.dumps(r), flush=True)
    del s, arena
