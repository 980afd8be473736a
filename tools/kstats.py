"""Per-dispatch durations of one kernel in a rocprofv3 kernel trace: count,
mean, median, min, and the mean of the last N dispatches (the timed calls of a
bench run come last) -- to set the bench line's kernel_ms beside rocprof's.

    python tools/kstats.py <trace dir or kernel_trace.csv> <kernel substring> [last N]"""
import csv
import glob
import json
import os
import statistics
import sys

path = sys.argv[1]
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
name = sys.argv[2]
last = int(sys.argv[3]) if len(sys.argv) > 3 else 0
rows = sorted((x for x in csv.DictReader(open(path)) if name in x["Kernel_Name"]), key=lambda x: int(x["Start_Timestamp"]))
d = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6 for x in rows]
out = dict(kernel=name, dispatches=len(d), mean_ms=statistics.mean(d) if d else None,
           median_ms=statistics.median(d) if d else None, min_ms=min(d) if d else None,
           all_ms=[round(x, 5) for x in d])
if last and d:
    out["last_n"] = last
    out["mean_last_ms"] = statistics.mean(d[-last:])
print(json.dumps(out))
