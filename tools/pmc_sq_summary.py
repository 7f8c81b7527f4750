#!/usr/bin/env python3
"""Per-dispatch means of the SQ counters tools/pmc_sq.sh / pmc_sq_r5.sh collected, per kernel kind
(conv plain / residual / f16 mode, the lds_ring microbenchmark's two loops), with the shares DESIGN §5
quotes: of the waves' cycles, waiting on counters and barriers (SQ_WAIT_ANY), issue-stalled
(SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY); and the matrix pipe's busy share,
SQ_VALU_MFMA_BUSY_CYCLES (summed over SIMDs) / (1,024 SIMDs x the dispatch's traced duration x 2.4 GHz).
usage: tools/pmc_sq_summary.py DIR  (DIR/p*/t_counter_collection.csv, t_kernel_trace.csv)"""
import csv
import glob
import json
import sys
from collections import defaultdict

SIMDS = 1024
CLOCK_GHZ = 2.4


def kind_of(name):
    # rocprofv3 has reported both mangled (ILb1E) and demangled (<true, ...>) template arguments
    if "k_wino3h_conv" in name:
        k = "residual" if ("ILb1E" in name or "k_wino3h_conv<true" in name) else "plain"
        return k + ("_f16" if "2147483648" in name else "")
    if "k_ring" in name:
        return "ring_ldsdma" if ("k_ringILi1E" in name or "k_ring<1>" in name) else "ring_vector"
    return None


def main(d):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in glob.glob(f"{d}/p*/t_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = kind_of(r["Kernel_Name"])
            if k is not None:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(f"{d}/p*/t_kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            k = kind_of(r["Kernel_Name"])
            if k is not None:
                dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for kind, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in sorted(cs.items())}
        der = {}
        wc = m.get("SQ_WAVE_CYCLES")
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if wc and c in m:
                der[c + "_share"] = round(m[c] / wc, 4)
        if dur[kind]:
            ns = sum(dur[kind]) / len(dur[kind])
            der["traced_us_mean"] = round(ns / 1e3, 2)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                der["mfma_busy_share"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * ns * CLOCK_GHZ), 4)
        m["derived"] = der
        out[kind] = m
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
