#!/usr/bin/env python3
"""k_wino3h_conv L2 hit rate and fetch per board, in the bench vs alone (tools/pmc_l2.sh output).
Steady state = the last half of the conv dispatches of each pass; boards per dispatch come from
the kernel's grid-independent argument count in the bench log (mean boards per launch).

usage: pmc_l2_summary.py PMC_DIR BENCH_BOARDS_PER_LAUNCH OUT.json"""
import csv
import json
import sys


def per_launch(path, counter, kernel="k_wino3h_conv"):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
         if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    v = v[len(v) // 2:]
    return (sum(v) / len(v) if v else None), len(v)


def main(d, nb, out):
    nb = float(nb)
    res = {"kernel": "k_wino3h_conv"}
    for name, boards in (("bench_hit", nb), ("fwd_hit", 1344.0)):
        hit, n = per_launch(f"{d}/{name}/t_counter_collection.csv", "TCC_HIT_sum")
        miss, _ = per_launch(f"{d}/{name}/t_counter_collection.csv", "TCC_MISS_sum")
        res[name] = {"launches": n, "boards_per_launch": boards, "hit": hit, "miss": miss,
                     "hit_rate": hit / (hit + miss) if hit is not None else None,
                     "miss_per_board": miss / boards if miss is not None else None}
    fetch, n = per_launch(f"{d}/bench_fetch/t_counter_collection.csv", "FETCH_SIZE")
    res["bench_fetch"] = {"launches": n, "fetch_kib_per_launch": fetch,
                          "fetch_bytes_per_board_x2": 2 * fetch * 1024 / nb if fetch else None}
    res["method"] = ("rocprofv3 --kernel-trace --pmc, one pass per counter group: TCC_HIT_sum + TCC_MISS_sum over a "
                     "short headline bench (two lanes) and over one lane's forward alone (1,344 boards), then "
                     "FETCH_SIZE over the bench (x2 per the gfx950 note)")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
