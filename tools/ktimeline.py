"""Kernel timeline of the last call in a rocprofv3 kernel trace, from the last
launch of a marker kernel: python tools/ktimeline.py <trace.csv> <marker>"""
import csv
import sys

r = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if sys.argv[2] in x["Kernel_Name"]]
seg = r[idx[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
prev = t0
for x in seg:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    if (e - s) > 20e3 or (s - prev) > 20e3:
        print("%9.1f gap %7.1f dur %7.1f %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3, x["Kernel_Name"][:60]))
    prev = e
print("span %.1f us" % ((prev - t0) / 1e3))
