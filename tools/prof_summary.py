#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run of bench.py into profiles/<round>/summary.md.

The bench times only its last `steps` steps; the trace also holds the aging and
warmup launches. The timed window is recovered as the last `launches` k_select
dispatches (the bench reports that count), and every kernel is averaged both
over the whole run and over that window, so the select average can be compared
with the bench's HIP-event average.

usage: prof_summary.py TRACE.csv BENCH_JSON_LOG OUT.md
"""
import csv
import json
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0][:80]


def main(trace, bench_log, out):
    with open(bench_log) as f:
        bench = json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r["VGPR_Count"]), int(r["SGPR_Count"]), int(r["Scratch_Size"])))
    rows.sort()
    rs = bench.get("roofline_select", bench["roofline"])
    # fused hash rounds: the select roofline's launches are k_round, k_select (first rounds) and k_apply (flushes)
    names = ("k_round", "k_select", "k_apply") if rs["kernel"].startswith("k_round") else ("k_select",)
    sel = [r for r in rows if any(n in r[2] for n in names)]
    nwin = rs["launches"]
    t0 = sel[-nwin][0] if len(sel) >= nwin else rows[0][0]
    win = [r for r in rows if r[0] >= t0]
    agg = defaultdict(lambda: [0, 0, 0, 0, 0])
    for s, e, n, v, sg, sc in win:
        a = agg[short(n)]
        a[0] += 1
        a[1] += e - s
        a[2], a[3], a[4] = v, sg, sc
    total = sum(a[1] for a in agg.values())
    span = win[-1][1] - win[0][0]
    lines = [f"# rocprofv3 kernel trace — timed window of `{bench_log}`", "",
             f"bench value (under rocprof): {bench['value']:.0f} sims/s; window = last {nwin} {' / '.join(names)} dispatches "
             f"and everything after; span {span / 1e6:.1f} ms, kernel busy {total / 1e6:.1f} ms", "",
             "| kernel | calls | total ms | % busy | avg us | VGPR | SGPR | scratch |", "|---|---|---|---|---|---|---|---|"]
    for n, a in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        lines.append(f"| `{n}` | {a[0]} | {a[1] / 1e6:.2f} | {100 * a[1] / total:.2f} | {a[1] / a[0] / 1e3:.1f} | "
                     f"{a[2]} | {a[3]} | {a[4]} |")
    lines.append("")
    seen = set()
    for key in ("roofline", "roofline_select", "roofline_backup"):
        rf = bench.get(key)
        if not rf or "unit" not in rf or rf["kernel"].split()[0] in seen:
            continue
        kname = rf["kernel"].split()[0]
        seen.add(kname)
        sw = [r for r in win if kname in r[2]]
        avg = sum(e - s for s, e, *_ in sw) / max(len(sw), 1) / 1e3
        tower = kname == "k_wino3t_tower"  # round 6: one launch = the 32 convs of a forward
        if rf["unit"] == "TFLOP/s":
            work = rf["executed_flop_per_board"] * rf["boards_per_launch"] * (32 if tower else 1)
            rate = f"{work / (avg * 1e-6) / 1e12:.1f} TFLOP/s executed MFMA flops (rocprof time)"
        else:
            work = rf["algo_bytes_per_launch"]
            rate = f"{work / (avg * 1e3):.2f} GB/s algorithmic (rocprof time)"
        ev = rf.get("tower_avg_launch_us") if tower else rf.get("event_avg_launch_us", rf["avg_launch_us"])
        lines.append(f"- `{kname}` in window: {len(sw)} dispatches, avg {avg:.1f} us (rocprof) vs "
                     f"{ev} us (this run's dispatch events, under the profiler; {rf['launches']} launches) -> {rate}")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    # the same window as JSON beside the .md: bench.py reads the rocprof averages of the tree kernels from it
    # (newest_profile), matched to its own configuration
    cfg = bench["config"]
    js = {"trace": trace, "bench_log": bench_log, "bench_value": bench["value"],
          "evaluator": ("hash" if "hash" in cfg.get("evaluator", "") else
                        "fused" if "HIP kernels" in cfg.get("evaluator", "") else "nn"),
          "games_per_gpu": cfg.get("games_per_gpu"),
          "sims_per_move": cfg.get("sims_per_move"), "lanes_per_gpu": cfg.get("lanes_per_gpu"),
          "trees_per_launch": cfg.get("games_per_gpu", 0) // max(cfg.get("lanes_per_gpu", 1), 1),
          "window_dispatches_k_select": nwin, "span_ms": span / 1e6, "busy_ms": total / 1e6,
          "kernels": {n: {"calls": a[0], "avg_us": a[1] / a[0] / 1e3, "total_ms": a[1] / 1e6} for n, a in agg.items()},
          "checks": {}}
    seen = set()
    for key in ("roofline", "roofline_select", "roofline_backup"):
        rf = bench.get(key)
        if not rf or "unit" not in rf or rf["kernel"].split()[0] in seen:
            continue
        kname = rf["kernel"].split()[0]
        seen.add(kname)
        sw = [r for r in win if kname in r[2]]
        tower = kname == "k_wino3t_tower"
        js["checks"][key] = {"kernel": kname, "rocprof_avg_us": sum(e - s for s, e, *_ in sw) / max(len(sw), 1) / 1e3,
                             "rocprof_dispatches": len(sw),
                             "event_avg_us": (rf.get("tower_avg_launch_us") if tower else
                                              rf.get("event_avg_launch_us", rf["avg_launch_us"])),
                             "event_launches": rf.get("tower_launches") if tower else rf["launches"]}
    with open(out.rsplit(".", 1)[0] + ".json", "w") as f:
        json.dump(js, f, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:4])
