"""Summarise tools/gpu_pmc.sh's counter passes into profiles/pmc_traffic.json.

    python tools/pmc_summary.py gpurun_out/pmc <round-tag> [--config C4-sk-2005] [--hot k_sp_grouprun]
        [--fetch DIR --write DIR] [--metric JAC --hub 4]

HBM bytes per launch, following MI355X_MICROARCH.md ("HBM [CDNA4]"):
FETCH_SIZE and WRITE_SIZE come from separate --pmc passes (they do not fit one
pass), both in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
streaming read, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch.
The guide calls other access widths uncalibrated: the figure is an upper-bound
style estimate for the gather-heavy kernels here, and ratios between variants
of one kernel are what it is used for.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ["k_sp_order_rank", "k_sp_cpass0", "k_sp_cpass", "k_sp_grouprun", "k_sp_exbucket", "k_sp_gather", "k_sp_arena_init", "k_sp_runs", "k_sp_bucket", "k_sp_survivors", "k_sp_expand", "k_sp_pass", "k_group_tiles", "k_p1_pass", "k_rts_scan", "k_rts_reduce", "k_os_pass", "k_score_runs", "k_gather_sel",
           "k_desc_keys_sel", "k_sel_hist"]


def short(name):
    hits = [k for k in KERNELS if k + "(" in name or k + "<" in name or name.endswith(k)]
    return max(hits, key=len) if hits else None


def per_kernel(path, counter):
    acc = defaultdict(list)
    for fn in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != counter:
                    continue
                k = short(row["Kernel_Name"])
                if k:
                    acc[k].append(float(row["Counter_Value"]))
    return acc


def main():
    src = sys.argv[1]
    tag = sys.argv[2] if len(sys.argv) > 2 else "r01"
    def opt(name, default):
        return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default
    config = opt("--config", "C4-sk-2005")
    fetch = per_kernel(opt("--fetch", os.path.join(src, "p1")), "FETCH_SIZE")
    write = per_kernel(opt("--write", os.path.join(src, "p2")), "WRITE_SIZE")
    hot = "k_sp_grouprun"
    if "--hot" in sys.argv:
        hot = sys.argv[sys.argv.index("--hot") + 1]
    out = {"config": config, "n_gpus": 1, "metric": opt("--metric", "JAC"), "hub": int(opt("--hub", "4")),
           "hot_kernel": hot,
           "source": "profiles/%s (rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE in separate passes, "
                     "bench.py --steps 5 --warmup 2 --no-cpu-baseline --sweep =); traffic = (2*FETCH_SIZE + "
                     "WRITE_SIZE) KiB * 1024 per dispatch" % tag,
           "kernels": {}}
    for k in KERNELS:
        if k not in fetch or k not in write:
            continue
        f = sum(fetch[k]) / len(fetch[k])
        w = sum(write[k]) / len(write[k])
        out["kernels"][k] = {"dispatches": len(fetch[k]), "fetch_kib": f, "write_kib": w,
                             "traffic_bytes": int((2 * f + w) * 1024)}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(root, "profiles", "pmc_traffic.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
