"""HIP IPC export/import of HBM arenas (placeholder; filled in with the RCCL data plane)."""
from __future__ import annotations


def export_handle(tensor) -> bytes:
    raise NotImplementedError
