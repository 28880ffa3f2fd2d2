#!/usr/bin/env python3
"""Summary of the round-3 PMC passes and kernel traces (not product code): per kernel, the median
counter value over its dispatches, converted to bytes per launch as MI355X_MICROARCH.md's HBM section
prescribes (FETCH_SIZE KiB x 1024 x 2 on gfx950, WRITE_SIZE KiB x 1024), against the algorithmic bytes.

    python tools/pmc_r3.py gpurun_out/r3p > profiles/r3/pmc/summary.txt
"""
import csv
import os
import sys
from collections import defaultdict
from statistics import median

ALG = {  # algorithmic bytes per launch: payload read, results written
    "cfg2": (4 << 30, 4 << 20),
    "cfg3": (16 << 30, 1 << 20),
    "cfg4": (5464418334, 131072 * 4),
    "lane36": ((1 << 30) // 36 * 36, (1 << 30) // 36 * 4),
    "walpay": (None, None),
}


def short(name):
    name = name.replace("tkv::(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0]


def main(root):
    for d in sorted(os.listdir(root)):
        p = os.path.join(root, d)
        f = os.path.join(p, "pmc_counter_collection.csv")
        if not os.path.exists(f):
            continue
        cfg = d.split("_")[1]
        per = defaultdict(lambda: defaultdict(list))
        for r in csv.DictReader(open(f)):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f"== {d}")
        for k, ctrs in per.items():
            if not any(x in k for x in ("crc_", "rows_", "lane", "wal_")):
                continue
            for c, vals in ctrs.items():
                m = median(vals)
                line = f"  {k:32s} {c:14s} dispatches {len(vals):4d}  median {m:14.1f}"
                if c == "FETCH_SIZE":
                    b = m * 1024 * 2
                    line += f"  = {b / 1e9:8.4f} GB read per launch"
                elif c == "WRITE_SIZE":
                    b = m * 1024
                    line += f"  = {b / 1e6:8.3f} MB written per launch"
                print(line)
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            tot = sum(median(v[c]) for k, v in per.items() if c in v and any(x in k for x in ("crc_", "rows_")))
            alg = ALG.get(cfg, (None, None))[0 if c == "FETCH_SIZE" else 1]
            if tot and alg:
                b = tot * 1024 * (2 if c == "FETCH_SIZE" else 1)
                print(f"  step total {c}: {b / 1e9:.4f} GB vs algorithmic {alg / 1e9:.4f} GB = {b / alg:.4f}x")
        hit = {k: v for k, v in per.items() if "TCC_HIT_sum" in v}
        for k, v in hit.items():
            if "crc_" in k:
                h, m = median(v["TCC_HIT_sum"]), median(v["TCC_MISS_sum"])
                print(f"  {k}: L2 hit rate {h / (h + m):.4f} (hits {h:.0f}, misses {m:.0f})")


if __name__ == "__main__":
    main(sys.argv[1])
