"""Per-step kernel timeline of the last complete step in a rocprofv3 kernel trace.

    python tools/prof_summary.py gpurun_out/prof/bench_kernel_trace.csv [first-kernel-substring]
"""
import csv
import sys

path = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "arena_init"
r = [x for x in csv.DictReader(open(path)) if "nlp::" in x["Kernel_Name"]]
r.sort(key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if first in x["Kernel_Name"]]
st = r[idx[-2]:idx[-1]]
t0 = int(st[0]["Start_Timestamp"])
prev = t0
busy = 0.0
for x in st:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    busy += (e - s) / 1e3
    print("%8.2f gap %6.2f dur %6.2f  %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3, x["Kernel_Name"][:70]))
    prev = e
print("kernel time %.2f us, step span %.2f us, gap to next step %.2f us"
      % (busy, (prev - t0) / 1e3, (int(r[idx[-1]]["Start_Timestamp"]) - prev) / 1e3))
