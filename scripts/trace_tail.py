#!/usr/bin/env python3
"""Mean duration of the last N launches of a kernel in a rocprofv3 kernel-trace CSV directory — the
launches of a bench command's timed region (bench.py runs nothing on the GPU after it but a reader), so
that `roofline.launch_ms` can be checked against the trace of the same command.

usage: scripts/trace_tail.py TRACE_DIR KERNEL_SUBSTRING N"""
import csv, glob, json, statistics, sys

d, name, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if name in r["Kernel_Name"])
dur = [(e - s) / 1e3 for s, e in ev]
print(json.dumps({"kernel": name, "launches": len(dur), "last_n": n, "mean_last_n_us": round(statistics.mean(dur[-n:]), 2),
                  "mean_all_us": round(statistics.mean(dur), 2), "min_us": round(min(dur), 2), "max_us": round(max(dur), 2)}))
