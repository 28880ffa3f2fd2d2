#!/usr/bin/env python3
"""Median per-dispatch value of every counter of the crc_rows dispatches in a tools/pmc.sh directory."""
import csv
import glob
import os
import sys
from collections import defaultdict

import numpy as np

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "crc_rows"
vals = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "pmc_counter_collection.csv"))):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (disp, name), v in per.items():
        vals[name].append(v)
for name in sorted(vals):
    print(f"{name:28s} {np.median(vals[name]):16.4g}  (n={len(vals[name])})")
