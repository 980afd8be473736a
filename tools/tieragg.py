"""Per-kernel launch durations of the path-4 kernels in a rocprofv3 kernel
trace (tools/gpu_tierprof.sh output): python tools/tieragg.py <trace.csv>..."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].split("(")[0]
        if "k_hp_" in n:
            agg[n + " LDS%s VGPR%s" % (r["LDS_Block_Size"], r["VGPR_Count"])].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        if sum(v) > 500:
            print("%3d sum %8.2f ms  %s  %s" % (len(v), sum(v) / 1e3, [round(x) for x in v][:12], k))
