#!/usr/bin/env python3
"""Timed-region summary of a rocprofv3 kernel trace (not product code): the last K dispatches of the
kernel whose name contains PATTERN (a bench's timed steps follow its warm-up and nothing of that
kernel runs after them), their average duration and their span per step, beside the average over
every dispatch (warm-up included, as the --stats summary reports it).

    python tools/trace_timed.py run_kernel_trace.csv 'crc_packed<true>' 200
"""
import csv
import json
import sys


def main():
    path, pat, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    last = rows[-k:]
    span = int(last[-1]["End_Timestamp"]) - int(last[0]["Start_Timestamp"])
    print(json.dumps({"kernel": pat, "dispatches": len(rows), "avg_all_us": round(sum(dur) / len(dur) / 1e3, 2),
                      "timed": len(last), "avg_timed_us": round(sum(dur[-k:]) / len(last) / 1e3, 2),
                      "span_per_step_us": round(span / len(last) / 1e3, 2)}))


if __name__ == "__main__":
    main()
