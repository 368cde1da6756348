"""Stress benchmarks (reference stress/ module: StressWorkerBench, StressClientIOBench,
StressMasterBench, UfsIOBench, MaxThroughput suite; results as JSON summaries, runnable locally
or fanned out over job workers with ``--cluster`` via the ``stress`` job plan)."""
from __future__ import annotations

import json


def run_local(bench: str, args: list, fs=None) -> dict:
    if bench == "master":
        from .master_bench import main as m
    elif bench == "worker":
        from .worker_bench import main as m
    elif bench == "client-io":
        from .client_io_bench import main as m
    elif bench == "ufs-io":
        from .ufs_io_bench import main as m
    else:
        raise ValueError(f"unknown bench {bench}")
    return m(list(args), fs=fs, print_result=False)


def merge_results(bench: str, results: list) -> dict:
    """Aggregate per-worker task results (reference *Summary classes: sums throughput, merges
    error lists, keeps per-worker rows)."""
    results = [r if isinstance(r, dict) else json.loads(r) for r in results if r is not None]
    out = {"bench": bench, "workers": len(results), "nodes": results}
    if not results:
        return out
    for k in ("throughput_ops", "throughput_MBps", "bytes", "ops"):
        if k in results[0]:
            out[k] = sum(r.get(k, 0) for r in results)
    errs = [e for r in results for e in r.get("errors", [])]
    out["errors"] = errs
    return out
