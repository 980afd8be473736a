"""Per-kernel SQ counter summary of a rocprofv3 --pmc pass (tools/gpu_r04.sh sweeppmc).

    python tools/sqpmc.py gpurun_out/<tag>/sweeppmc [kernel-substring ...]

Prints per kernel: dispatches, SQ_WAVE_CYCLES split into WAIT_ANY (parked on
s_waitcnt / barrier), WAIT_INST_ANY (issue stalls) and ACTIVE_INST_ANY, the VALU
share, VALU instructions per wave-cycle and LDS bank-conflict cycles per LDS
cycle (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES).
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    src = sys.argv[1]
    want = sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for fn in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                m = re.search(r"(k_[a-z0-9_]+(<[^(]*>)?)", row["Kernel_Name"])
                k = m.group(1) if m else row["Kernel_Name"][:40]
                if want and not any(w in k for w in want):
                    continue
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        parts = ["%-44s n=%3d" % (k[:44], len(disp[k]))]
        for name, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "stall"), ("SQ_ACTIVE_INST_ANY", "active"),
                          ("SQ_ACTIVE_INST_VALU", "valu")):
            if name in c:
                parts.append("%s %4.1f%%" % (lab, 100 * c[name] / wc))
        if "SQ_INSTS_VALU" in c:
            parts.append("valu/wcyc %.3f" % (c["SQ_INSTS_VALU"] / wc))
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            parts.append("lds-conf %4.1f%%" % (100 * c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]))
        print("  ".join(parts))


if __name__ == "__main__":
    main()
