#!/usr/bin/env python3
"""Table of a lane_probe / rec_probe JSONL file: one row per workload, one column (GB/s) per library
(not product code). python tools/probe_table.py FILE.jsonl"""
import json
import sys

rows, libs = {}, []
for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    key = d.get("work") or d.get("image")
    lib = d["lib"] + (":" + d["call"] if "call" in d else "")
    rows.setdefault(key, {})[lib] = d.get("GBps", d.get("payload_GBps"))
    if lib not in libs:
        libs.append(lib)
w = max(len(k) for k in rows)
print(" " * w, " | ".join(f"{x[:16]:>16s}" for x in libs))
for k, r in rows.items():
    print(f"{k:{w}s}", " | ".join(f"{r.get(x, float('nan')):16.1f}" for x in libs))
