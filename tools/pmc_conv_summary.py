#!/usr/bin/env python3
"""k_wino3h_conv HBM traffic per board from tools/pmc_conv.sh output -> profiles/<round>/pmc_conv.json.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (rocprofv3); steady state = the last half of the
conv dispatches. On gfx950 FETCH_SIZE counts 64 B per 128-B read request (MI355X_MICROARCH.md,
HBM): the kernel's reads are 16-byte-per-lane streaming loads, so the doubled figure is the
read traffic. Algorithmic bytes per board and conv: read x (41.5 KB), write y (41.5 KB), and on
every second conv read the residual (41.5 KB); the transformed weights (1.6 MB per launch) are
shared by all boards.

usage: pmc_conv_summary.py PMC_DIR N_BOARDS OUT.json [KERNEL [CONVS_PER_DISPATCH]]
(round 6: KERNEL k_wino3t_tower, 32 convs per dispatch: the per-board figures are per conv, as before)
"""
import csv
import json
import sys


def per_launch(path, counter, kernel="k_wino3h_conv"):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
         if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    v = v[len(v) // 2:]
    return sum(v) / len(v), len(v)


def main(d, n, out, kernel="k_wino3h_conv", convs=1):
    n = int(n) * int(convs)  # board-convs per dispatch
    fetch, nf = per_launch(f"{d}/p1/t_counter_collection.csv", "FETCH_SIZE", kernel)
    write, nw = per_launch(f"{d}/p2/t_counter_collection.csv", "WRITE_SIZE", kernel)
    algo = 81 * 128 * 4 * 2.5
    res = {
        "kernel": kernel,
        "convs_per_dispatch": int(convs),
        "boards_per_launch": int(n) // int(convs),
        "launches_averaged": [nf, nw],
        "fetch_bytes_per_board_raw": fetch * 1024 / n,
        "fetch_bytes_per_board_x2": 2 * fetch * 1024 / n,
        "write_bytes_per_board": write * 1024 / n,
        "hbm_bytes_per_board": (2 * fetch + write) * 1024 / n,
        "algo_bytes_per_board": algo,
        "traffic_over_algorithmic": (2 * fetch + write) * 1024 / n / algo,
        "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE, then WRITE_SIZE, separate passes of "
                  "tools/diag/nn_forward_only.py (12 forwards, 32 convs each); KiB -> bytes; reads doubled "
                  "(gfx950 FETCH_SIZE counts half of 16-B/lane streaming reads)",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
