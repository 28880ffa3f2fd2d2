#!/usr/bin/env python3
"""Summary of the round-4 lane-kernel PMC passes (tools/gpu_r4_lanepmc.sh; not product code): per
workload and kernel, the median of each counter over its dispatches, and the derived figures the
bound is read from (MI355X_MICROARCH.md: SQ_* cycle counters count quad-cycles, per SIMD summed over
the chip; FETCH_SIZE x 1024 x 2 = HBM bytes on gfx950).

    python tools/pmc_r4.py gpurun_out/r4_s2/lanepmc > profiles/r4/lanes_pmc/summary.txt
    python tools/pmc_r4.py gpurun_out/r5_lanepmc r5   (round 5's workloads, tools/gpu_r5_lanepmc.sh)
"""
import csv
import os
import re
import sys
from collections import defaultdict
from statistics import median

WORK = {"w1": "uniform 26 B", "w2": "uniform 36 B", "w3": "uniform 59 B", "w4": "irregular WAL payloads 36 B (8-byte gaps)"}
PAYLOAD = {"w1": (1 << 30) // 26 * 26, "w2": (1 << 30) // 36 * 36, "w3": (1 << 30) // 59 * 59,
           "w4": (1 << 30) // 44 * 36}
LEN = {"w1": 26, "w2": 36, "w3": 59, "w4": 36}
WORK5 = {"w1": "uniform 26 B", "w2": "uniform 36 B", "w3": "uniform 36 B at stride 44 from base + 8",
         "w4": "irregular WAL payloads 36 B (8-byte gaps)"}
PAYLOAD5 = {"w1": (1 << 30) // 26 * 26, "w2": (1 << 30) // 36 * 36, "w3": ((1 << 30) - 8) // 44 * 36,
            "w4": (1 << 30) // 44 * 36}
LEN5 = {"w1": 26, "w2": 36, "w3": 36, "w4": 36}


def short(name):
    name = name.replace("tkv::(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0]


def main(root):
    data = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))  # work -> kernel -> counter -> values
    for d in sorted(os.listdir(root)):
        m = re.match(r"(w\d)_g\d+$", d)
        if not m:
            continue
        for dp, _, files in os.walk(os.path.join(root, d)):
            for f in files:
                if not f.endswith("counter_collection.csv"):
                    continue
                for r in csv.DictReader(open(os.path.join(dp, f))):
                    k = short(r["Kernel_Name"])
                    if any(x in k for x in ("crc_", "rows_", "lane", "group")):
                        data[m.group(1)][k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for w in sorted(data):
        print(f"== {w}: {WORK.get(w, w)} (payload {PAYLOAD.get(w, 0) / 1e9:.3f} GB per launch)")
        for k, ctrs in data[w].items():
            med = {c: median(v) for c, v in ctrs.items()}
            print(f"  {k}")
            for c in sorted(med):
                print(f"    {c:36s} {med[c]:16.1f}  ({len(ctrs[c])} dispatches)")
            if "SQ_WAVE_CYCLES" in med:
                wc = med["SQ_WAVE_CYCLES"]
                for c in ("SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                          "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VMEM"):
                    if c in med:
                        print(f"    {c} / SQ_WAVE_CYCLES = {med[c] / wc:.3f}")
            if "SQ_INSTS_VALU" in med and "SQ_WAVES" in med:
                pass
            n = PAYLOAD.get(w)
            if n and "SQ_INSTS_VALU" in med:
                blocks = n / LEN[w]
                for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SMEM"):
                    if c in med:
                        print(f"    {c} per 64 blocks (one wave step) = {med[c] / (blocks / 64):.1f}")
            if "FETCH_SIZE" in med and n:
                print(f"    HBM read per launch = {med['FETCH_SIZE'] * 2048 / 1e9:.4f} GB = {med['FETCH_SIZE'] * 2048 / n:.3f}x payload")
            if "GRBM_GUI_ACTIVE" in med and "SQ_BUSY_CYCLES" in med:
                print(f"    GRBM_GUI_ACTIVE (sum over 8 XCDs) = {med['GRBM_GUI_ACTIVE']:.0f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "r5":
        WORK, PAYLOAD, LEN = WORK5, PAYLOAD5, LEN5
    main(sys.argv[1])
