"""Per-call kernel totals of the predict calls in a rocprofv3 kernel trace:
the library's kernels minus the per-graph ones (nlp_graph_create), divided by
the number of calls.  python tools/kagg2.py <trace dir or csv> [calls=2]"""
import csv
import glob
import os
import sys

GRAPH = ("k_in_", "k_del_", "k_degrees", "k_check_keys", "k_row_descents", "k_transpose_keys", "k_toff_split",
         "k_etab_upper", "k_etab_insert", "k_edge_filter", "k_deg_class", "k_sv_pack", "k_hp_tile_rows", "k_hp_xs",
         "k_diff_", "k_sum_deg2", "k_hp_entry_classes")
path = sys.argv[1]
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 2
r = sorted((x for x in csv.DictReader(open(path)) if "nlp::" in x["Kernel_Name"]),
           key=lambda x: int(x["Start_Timestamp"]))
# the graph build's radix sort (k_rs_*) precedes the first predict kernel; the build's last kernels (the
# membership table, the short lists' sort and prefix, which follow its own degree-class compaction) end it
last = max((i for i, x in enumerate(r) if any(g in x["Kernel_Name"] for g in ("k_etab_insert", "k_sl_sort", "k_hp_entry_classes"))),
           default=-1)
first = next(i for i, x in enumerate(r) if i > last and not any(g in x["Kernel_Name"] for g in GRAPH + ("k_rs_", "k_scan")))
r = r[first:]
agg = {}
for x in r:
    n = x["Kernel_Name"].replace("void ", "").split("(")[0][:70]
    d = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
    a = agg.setdefault(n, [0, 0.0])
    a[0] += 1
    a[1] += d
tot = sum(t for _, t in agg.values()) / calls
span = (int(r[-1]["End_Timestamp"]) - int(r[0]["Start_Timestamp"])) / 1e6 / calls
print("per call: kernel time %.2f ms, span %.2f ms (%d calls)" % (tot, span, calls))
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print("  %-70s n=%6.1f  %9.3f ms  %5.1f%%" % (n, c / calls, t / calls, 100 * t / calls / tot))
