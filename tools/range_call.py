"""One source-range prediction on a full-size stand-in, for kernel traces and
PMC passes of the IHub path: the same bounded range as
tests/test_gpu_c5.py (sources from span/3 on, until their IHub work
sum_{v in N(u)} deg v reaches --wedges), a warm call, then --reps timed
calls.  One JSON line on stdout (wedges/s of w > u, the extrapolated full call).

    python tools/range_call.py [--config C5-sk-2005-ihub] [--metric CN] [--hub 0] [--wedges 1.5e9] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nlp_loader  # noqa: E402


def source_work(off, keys):
    """IHub work per source, W(u) = sum of deg v over N(u), on the device."""
    deg = off[1:] - off[:-1]
    m = keys.numel()
    pref = torch.zeros(m + 1, dtype=torch.int64, device=keys.device)
    carry = torch.zeros((), dtype=torch.int64, device=keys.device)
    for b in range(0, m, 1 << 27):
        e = min(m, b + (1 << 27))
        pref[b + 1:e + 1] = torch.cumsum(deg[keys[b:e].long()], 0) + carry
        carry = pref[e]
    W = (pref[off[1:]] - pref[off[:-1]]).cpu().numpy()
    return W, float(torch.sum(deg.double() ** 2))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5-sk-2005-ihub")
    ap.add_argument("--metric", default="CN")
    ap.add_argument("--hub", type=int, default=0)
    ap.add_argument("--wedges", type=float, default=1.5e9)
    ap.add_argument("--start", type=float, default=1.0 / 3)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    nlp = nlp_loader.load()
    gg = nlp_loader.load_sub("graphgen")
    off, keys, du, dw, info = gg.make_workload(gg.CONFIGS[args.config], "cuda")
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    k = info["k"]
    W, total = source_work(off, keys)
    span = len(W)
    ua = int(span * args.start)
    ub = min(span, ua + int(np.searchsorted(np.cumsum(W[ua:].astype(np.float64)), args.wedges)) + 1)
    G = nlp.Graph.from_device(off, keys)
    out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
    mid = nlp.METRICS.index(args.metric)
    G.predict_device(mid, args.hub, k, out, ua, ub)  # warm
    torch.cuda.synchronize()
    best = None
    for _ in range(args.reps):
        t0 = time.perf_counter()
        n, t = G.predict_device(mid, args.hub, k, out, ua, ub)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        best = ms if best is None else min(best, ms)
    rate = t["wedges"] / (best * 1e-3)
    print(json.dumps(dict(config=args.config, metric=args.metric, H=args.hub, range=[ua, ub], sources=ub - ua,
                          range_work_all=int(W[ua:ub].sum()), wedges_gt=t["wedges"], candidates=t["candidates"],
                          predicted=n, gpu_ms=best, score_ms=t["score_ms"], select_ms=t["select_ms"],
                          chunks=t["chunks"], path=t["path"], wedges_per_s=rate, total_wedges_all=total,
                          full_call_estimate_s_1gpu=0.5 * total / rate,
                          full_call_estimate_s_8gpu=0.5 * total / rate / 8)), flush=True)
    G.close()


if __name__ == "__main__":
    main()
