#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of one bench.py run into its phases and summarise each.

bench.py issues, on one stream, `warm` untimed steps, then `steps` timed steps, then (N=1, unless
--no-pipelined) 20 + `steps` steps alternating two streams. With the bench line of the same run
this gives the trace's own average launch duration over exactly the timed steps, to set beside the
line's HIP-event `kernel_ms`.

usage: trace_phases.py run_kernel_trace.csv bench_line.json [kernel-name-substring]
"""
import csv
import json
import statistics
import sys


def main():
    trace, line_path = sys.argv[1], sys.argv[2]
    sub = sys.argv[3] if len(sys.argv) > 3 else "crc_packed"
    line = json.loads(open(line_path).read().strip().splitlines()[-1])
    warm = line["warmup_run"]["steps"]
    steps = line["steps"]
    rows = [r for r in csv.DictReader(open(trace)) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    phases = {"warmup": (0, warm), "timed": (warm, warm + steps), "pipelined": (warm + steps, len(rows))}
    out = {"kernel_substring": sub, "launches": len(rows), "bench_kernel_ms": line["roofline"]["kernel_ms"],
           "bench_value": line["value"], "phases": {}}
    for name, (a, b) in phases.items():
        d = dur[a:b]
        if not d:
            continue
        ph = {"launches": len(d), "avg_us": round(sum(d) / len(d) / 1e3, 2), "min_us": round(min(d) / 1e3, 2),
              "max_us": round(max(d) / 1e3, 2), "stdev_us": round(statistics.pstdev(d) / 1e3, 2)}
        if name == "timed":
            span = int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])
            ph["span_per_step_us"] = round(span / len(d) / 1e3, 2)
        out["phases"][name] = ph
    # Every kernel of the timed steps: those that start after the last warm-up anchor ends and
    # before the last timed anchor ends, with their mean duration and the idle time between launches.
    allk = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    lo = int(rows[warm - 1]["End_Timestamp"]) if warm else 0
    hi = int(rows[warm + steps - 1]["End_Timestamp"])
    win = [r for r in allk if lo <= int(r["Start_Timestamp"]) < hi]
    per = {}
    for r in win:
        per.setdefault(r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-48:], []).append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out["timed_step_kernels"] = {k: {"launches": len(v), "avg_us": round(sum(v) / len(v) / 1e3, 2),
                                     "min_us": round(min(v) / 1e3, 2)} for k, v in per.items()}
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
    out["timed_idle_us_per_step"] = round(((hi - lo) - busy) / steps / 1e3, 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
