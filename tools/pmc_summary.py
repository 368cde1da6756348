#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--pmc`` counter_collection.csv per kernel (sum over dispatches).

    python tools/pmc_summary.py gpurun_out/pmc_dram_local/pmc_counter_collection.csv [--bytes-per-req 64]

TCC_EA0_{RD,WR}REQ_DRAM counters count 64-byte requests on gfx950 (a 32B request counts once
too, so this is an upper bound on bytes); the summary also prints the implied byte totals.
"""
import argparse
import collections
import csv
import json


def summarise(path: str, bytes_per_req: int = 64) -> dict:
    agg: dict = collections.defaultdict(lambda: collections.defaultdict(float))
    dispatches: dict = collections.defaultdict(set)
    ns: dict = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        k = k[:k.find("(")] if "(" in k else k
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Dispatch_Id"] not in dispatches[k]:
            dispatches[k].add(r["Dispatch_Id"])
            ns[k] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = {}
    for k, counters in agg.items():
        e = {"dispatches": len(dispatches[k]), "kernel_ns_total": ns[k]}
        for c, v in counters.items():
            e[c] = v
            if "REQ" in c:
                e[c + "_bytes"] = v * bytes_per_req
        out[k] = e
    return out


def per_dispatch(path: str, kernel: str, bytes_per_req: int = 64) -> list:
    """Counters of every dispatch of kernels whose name contains ``kernel``, in dispatch order
    (to split one run's dispatches into bench phases)."""
    rows: dict = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if kernel not in k:
            continue
        d = rows.setdefault(int(r["Dispatch_Id"]), {"dispatch": int(r["Dispatch_Id"]),
                                                     "ns": float(r["End_Timestamp"]) - float(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"]) * bytes_per_req
    return [rows[k] for k in sorted(rows)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--bytes-per-req", type=int, default=64)
    ap.add_argument("--per-dispatch", default=None, help="kernel-name substring: print each dispatch (bytes)")
    a = ap.parse_args()
    for p in a.csv:
        if a.per_dispatch:
            for row in per_dispatch(p, a.per_dispatch, a.bytes_per_req):
                print(json.dumps(row))
        else:
            print(json.dumps({"file": p, "kernels": summarise(p, a.bytes_per_req)}))


if __name__ == "__main__":
    main()
