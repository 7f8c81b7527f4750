#!/usr/bin/env python3
"""FETCH_SIZE calibration summary (tools/diag/fetch_cal.hip): counter per dispatch / the bytes the
program actually read, per load shape, at k_select's concurrency.

usage: fetch_cal_summary.py FETCH_CAL.json PASS1_counter_collection.csv [PASS2_counter_collection.csv] OUT.json

PASS1 holds FETCH_SIZE (KiB per dispatch); PASS2 (optional) TCC_EA0_RDREQ_sum and TCC_EA0_RDREQ_32B_sum.
The k_fetch dispatches are matched to fetch_cal's launch list in dispatch order.
"""
import csv
import json
import sys
from collections import defaultdict


def per_dispatch(path, counter):
    rows = defaultdict(float)
    order = []
    for r in csv.DictReader(open(path)):
        if "k_fetch" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        if d not in rows:
            order.append(d)
        rows[d] += float(r["Counter_Value"])
    return [rows[d] for d in sorted(order)]


def main(cal_json, pass1, *rest):
    out = rest[-1]
    pass2 = rest[0] if len(rest) > 1 else None
    cal = json.load(open(cal_json))
    launches = cal["launches"]
    fetch = per_dispatch(pass1, "FETCH_SIZE")
    if len(fetch) != len(launches):
        raise SystemExit(f"{len(fetch)} k_fetch dispatches with FETCH_SIZE, {len(launches)} launches")
    req = per_dispatch(pass2, "TCC_EA0_RDREQ_sum") if pass2 else None
    req32 = per_dispatch(pass2, "TCC_EA0_RDREQ_32B_sum") if pass2 else None
    by = defaultdict(list)
    for i, l in enumerate(launches):
        f = fetch[i] * 1024.0
        e = {"waves": l["waves"], "bytes_read": l["bytes"], "fetch_size_bytes": f,
             "fetch_over_bytes": f / l["bytes"]}
        if req:
            e["rdreq"] = req[i]
            e["rdreq_32B"] = req32[i]
            e["bytes_per_request"] = l["bytes"] / max(req[i], 1.0)
        by[l["shape"]].append(e)
    res = {"source": "tools/diag/fetch_cal.hip under rocprofv3 --kernel-trace --pmc FETCH_SIZE (pass 1) and "
                     "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum (pass 2); 4 waves per workgroup, one wave per "
                     "'tree', reads at chunk positions that never repeat within a launch (1 GiB buffer)",
           "shapes": {}}
    for shape, es in by.items():
        r = sorted(x["fetch_over_bytes"] for x in es)
        med = r[len(r) // 2]
        res["shapes"][shape] = {"fetch_over_bytes_median": round(med, 4), "fetch_over_bytes_range": [round(r[0], 4), round(r[-1], 4)],
                                "correction_factor": round(1.0 / med, 4), "launches": es}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: {kk: v[kk] for kk in ("fetch_over_bytes_median", "correction_factor")}
                      for k, v in res["shapes"].items()}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
