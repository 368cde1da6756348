"""MaxThroughput suite: find the highest sustained master op rate (reference
stress/shell/src/main/java/alluxio/stress/cli/suite/MaxThroughput.java — binary search of
``--target-throughput`` for StressMasterBench, accepting a rate when the achieved throughput is
within ``--tolerance`` of the target and no errors occurred)."""
from __future__ import annotations

import argparse
import json

from .master_bench import main as master_bench


def main(argv=None, fs=None, print_result=True) -> dict:
    ap = argparse.ArgumentParser(prog="MaxThroughput")
    ap.add_argument("--operation", default="GetFileStatus")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--duration", default="2s")
    ap.add_argument("--lo", type=int, default=100)
    ap.add_argument("--hi", type=int, default=200_000)
    ap.add_argument("--tolerance", type=float, default=0.95)
    ap.add_argument("--iterations", type=int, default=8)
    a = ap.parse_args(argv or [])
    lo, hi, best, trace = a.lo, a.hi, None, []
    for _ in range(a.iterations):
        target = (lo + hi) // 2
        r = master_bench(["--operation", a.operation, "--threads", str(a.threads), "--duration", a.duration,
                          "--warmup", "0s", "--target-throughput", str(target)], fs=fs, print_result=False)
        ok = not r["errors"] and r["throughput_ops"] >= a.tolerance * target
        trace.append({"target": target, "achieved": r["throughput_ops"], "ok": ok})
        if ok:
            best, lo = r, target
        else:
            hi = target
        if hi - lo <= max(1, lo // 50):
            break
    out = {"bench": "max-throughput", "operation": a.operation, "max_ops": best["throughput_ops"] if best else 0,
           "trace": trace}
    if print_result:
        print(json.dumps(out))
    return out


if __name__ == "__main__":  # pragma: no cover
    main(__import__("sys").argv[1:])
