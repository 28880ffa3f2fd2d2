#!/usr/bin/env python3
"""Per-kernel duration summary (rocprofv3 --stats layout) from a rocprofv3 results database
(the default rocpd/SQLite output): python3 tools/rocpd_stats.py run_results.db > stats.csv"""
import csv, sqlite3, statistics, sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
cols = [d[1] for d in db.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else "kernel_name"
rows = db.execute(f"select {name_col}, start, end from kernels").fetchall()
dur = defaultdict(list)
for n, s, e in rows:
    dur[n].append(e - s)
tot = sum(sum(v) for v in dur.values())
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([n, len(v), sum(v), sum(v) / len(v), round(100 * sum(v) / tot, 2), min(v), max(v),
                statistics.pstdev(v)])
