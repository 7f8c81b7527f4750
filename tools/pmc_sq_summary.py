#!/usr/bin/env python3
"""Per-dispatch means of the SQ counters tools/pmc_sq.sh collected, per conv kernel (plain / residual)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/p*/t_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_wino3h_conv" not in k:
                continue
            kind = "residual" if "ILb1E" in k else "plain"
            acc[kind][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {kind: {c: sum(v) / len(v) for c, v in sorted(cs.items())} for kind, cs in acc.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
