#!/usr/bin/env python3
"""k_select (or k_apply) HBM traffic per launch from tools/pmc_select.sh output -> profiles/<round>/pmc_select.json.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3); steady state = the
last third of the k_select dispatches of each pass. Raw values: on gfx950
FETCH_SIZE counts 64 B per 128-B read request (MI355X_MICROARCH.md, HBM), i.e.
it can under-report wide coalesced reads by 2x; k_select's reads are 4 B/lane
and uncalibrated, so both the raw and the doubled read figure are kept.

usage: pmc_summary.py PMC_DIR BENCH_LOG OUT.json [KERNEL]   (k_select default, k_apply, or k_round)
"""
import csv
import json
import sys


def per_launch(path, counter, kernel="k_select"):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
         if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    v = v[-max(1, len(v) // 3):]
    return sum(v) / len(v), len(v)


def main(d, bench_log, out, kernel="k_select"):
    fetch, nf = per_launch(f"{d}/p1/t_counter_collection.csv", "FETCH_SIZE", kernel)
    write, nw = per_launch(f"{d}/p2/t_counter_collection.csv", "WRITE_SIZE", kernel)
    rdreq, _ = per_launch(f"{d}/p3/t_counter_collection.csv", "TCC_EA0_RDREQ_sum", kernel)
    bench = json.loads([ln for ln in open(bench_log).read().splitlines() if ln.startswith("{")][-1])
    # k_round (fused hash rounds): the select roofline carries both kernels' algorithmic bytes
    roof = bench["roofline_select"] if kernel in ("k_select", "k_round") else bench["roofline_backup"]
    res = {
        "kernel": kernel,
        "launches_averaged": [nf, nw],
        "trees_per_launch": bench["config"]["games_per_gpu"] // bench["config"].get("lanes_per_gpu", 1),
        "fetch_bytes": fetch * 1024, "write_bytes": write * 1024,
        "tcc_ea0_rdreq_x64_bytes": rdreq * 64,
        "traffic_bytes_raw": (fetch + write) * 1024,
        "traffic_bytes_reads_doubled": (2 * fetch + write) * 1024,
        "algo_bytes_per_launch_bench": roof["algo_bytes_per_launch"],
        "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE, then WRITE_SIZE, then TCC_EA0_RDREQ_sum, "
                  "separate passes of `bench.py --steps 6 --warmup 2 --age " + str(bench["config"]["aged_moves"]) +
                  "`; KiB -> bytes; algorithmic bytes from the first pass's own bench line",
        "aged_moves": bench["config"]["aged_moves"],
        "traffic_over_algo": round((fetch + write) * 1024 / max(roof["algo_bytes_per_launch"], 1), 3),
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
