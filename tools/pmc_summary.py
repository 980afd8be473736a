"""Summarise FETCH_SIZE / WRITE_SIZE counter passes into profiles/pmc_traffic.json.

    python tools/pmc_summary.py --fetch DIR --write DIR --tag r04 \
        --record C4-sk-2005:JAC:4:k_sp_grouprun --record C4-sk-2005:JAC:16:k_hp_batch [--calls 16=5]

HBM bytes per launch, following MI355X_MICROARCH.md ("HBM [CDNA4]"):
FETCH_SIZE and WRITE_SIZE come from separate --pmc passes (they do not fit one
pass), both in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
streaming read, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch.
The guide calls other access widths uncalibrated: the figure is an upper-bound
style estimate for the gather-heavy kernels here, and ratios between variants
of one kernel are what it is used for.

One record per --record config:metric:hub:hot_kernel.  A record takes the
kernels of its own path: path 1 (k_sp_*) for hub thresholds whose calls run
the sort path, path 4 (k_hp_*, k_hh_*, k_es_*, selection) otherwise -- in the
bench command the headline call (H = 4) is path 1 and the work point (H >= 8)
path 4, so no dispatch is claimed by two records.  --calls H=N gives the
profiled calls of that record (launches_per_call = dispatches / N).  Records
already in the file for other (config, n_gpus, metric, hub) keys are kept.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH1 = re.compile(r"^(k_sp_\w+|k_group_tiles|k_p1_pass|k_rts_\w+|k_score_runs|k_gather_sel|k_desc_keys_sel)$")
PATH4 = re.compile(r"^(k_hp_\w+|k_hh_\w+|k_es_\w+|k_sel_\w+|k_ts_\w+|k_scan_\w+)$")


def short(name):
    """nlp::k_hp_batch<false, 1024, ...>(...) -> k_hp_batch"""
    m = re.search(r"(k_[a-z0-9_]+)", name)
    return m.group(1) if m else None


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--tag", required=True)
    ap.add_argument("--record", action="append", required=True, help="config:metric:hub:hot_kernel")
    ap.add_argument("--calls", action="append", default=[], help="hub=profiled calls")
    ap.add_argument("--cmd", default="bench.py --steps 5 --warmup 2 --no-cpu-baseline --sweep = --wp-steps 3 --work-point 16")
    args = ap.parse_args()
    fetch = per_kernel(args.fetch, "FETCH_SIZE")
    write = per_kernel(args.write, "WRITE_SIZE")
    calls = {int(h): int(n) for h, n in (c.split("=") for c in args.calls)}
    dst = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(dst) as f:
            old = json.load(f)
        records = old.get("records", [old])
    except (OSError, ValueError):
        records = []
    for spec in args.record:
        config, metric, hub, hot = spec.split(":")
        hub = int(hub)
        pat = PATH1 if hub <= 4 else PATH4
        rec = {"config": config, "n_gpus": 1, "metric": metric, "hub": hub, "hot_kernel": hot,
               "source": "profiles/%s (rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE in separate passes, "
                         "%s); traffic = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 per dispatch" % (args.tag, args.cmd),
               "kernels": {}}
        for k in sorted(set(fetch) & set(write)):
            if not pat.match(k):
                continue
            f = sum(fetch[k]) / len(fetch[k])
            w = sum(write[k]) / len(write[k])
            kr = {"dispatches": len(fetch[k]), "fetch_kib": f, "write_kib": w, "traffic_bytes": int((2 * f + w) * 1024)}
            if hub in calls:
                kr["launches_per_call"] = len(fetch[k]) / calls[hub]
            rec["kernels"][k] = kr
        key = (config, 1, metric, hub)
        records = [r for r in records if (r.get("config"), r.get("n_gpus"), r.get("metric"), r.get("hub")) != key]
        records.append(rec)
    with open(dst, "w") as fh:
        json.dump({"records": records}, fh, indent=1)
    print(json.dumps({"records": records}, indent=1)[:4000])


if __name__ == "__main__":
    main()
