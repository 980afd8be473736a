"""Aggregate a rocprofv3 kernel trace per predict call (calls delimited by a
marker kernel): python tools/kagg.py <kernel_trace.csv> [marker]"""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_hp_work"
r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if marker in x["Kernel_Name"]] + [len(r)]
for ci in range(len(idx) - 1):
    seg = r[idx[ci]:idx[ci + 1]]
    agg = {}
    for x in seg:
        n = x["Kernel_Name"].split("(")[0][:60]
        d = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
        a = agg.setdefault(n, [0, 0.0])
        a[0] += 1
        a[1] += d
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
    print("call %d span %.1f ms" % (ci, span))
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:8]:
        print("   %-60s n=%4d  %9.2f ms" % (n, c, t))
