#!/usr/bin/env python3
"""Effective shader clock per kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass:
clock = GRBM_GUI_ACTIVE / 8 (summed over XCDs) / dispatch duration (MI355X_MICROARCH 'DVFS give-back')."""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
        continue
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    if dur <= 0:
        continue
    rows[r["Kernel_Name"][:70]].append((float(r["Counter_Value"]) / 8 / dur / 1e9, dur * 1e3))
for k, v in rows.items():
    v = np.array(v)
    print(f"{k:70s} n={len(v):3d} clock {np.median(v[:, 0]):.3f} GHz  dur {np.median(v[:, 1]):.3f} ms")
