"""The whole C5 call (sk-2005 stand-in, IHub Common Neighbours, 0.01|E| removed;
SURVEY §8(d) C5, BASELINE configs[4]) as the 8 wedge-balanced source shards of
the 8-GPU design (dist.py), run back to back on ONE GPU.

    python tools/c5_shards.py --shards 8 --which 0,1,2,3 > part0.jsonl
    python tools/c5_shards.py --merge part0.jsonl part1.jsonl > c5_call.json

Each shard is one nlp_predict_device call on its source range (the shard's
canonical local top-k, k = |deletions| / 2 of the whole call), timed on its
own.  A shard's line carries its time, wedges, candidates, local count and the
histogram of its result's score keys (CN scores are small integers: a few
hundred distinct keys), which is exactly what the exchange step needs:
--merge runs the histogram-first selection of dist.select_quota over the
shards' histograms (the k-th key, every shard's count above it, the tie quota
handed out in shard = u order) and reports the merged count, every shard's
share, the sum of the shard times (the one-GPU call) and their maximum (the
8-GPU call's predict phase).  A heartbeat on stderr every minute keeps a long
shard visibly alive.
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def heartbeat(stop, t0, what):
    while not stop.wait(60):
        print("[c5_shards] %s: %.0f s" % (what[0], time.time() - t0), file=sys.stderr, flush=True)


def run(args):
    import torch
    import nlp_loader
    nlp = nlp_loader.load()
    gg = nlp_loader.load_sub("graphgen")
    dmod = nlp_loader.load_sub("dist")
    t0 = time.time()
    off, keys, du, dw, info = gg.make_workload(gg.CONFIGS[args.config], "cuda")
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    gen_s = time.time() - t0
    k = info["k"]
    span = off.numel() - 1
    w = dmod.source_weights(off, keys, args.hub)
    ranges = dmod.shard_ranges(span, args.shards, w)
    deg = (off[1:] - off[:-1]).double()
    total_w = float(torch.sum(deg * deg))  # every wedge (u, v, w), w > u or not: IHub sum of deg v^2
    t0 = time.time()
    G = nlp.Graph.from_device(off, keys)
    torch.cuda.synchronize()
    create_s = time.time() - t0
    out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
    mid = nlp.METRICS.index(args.metric)
    which = [int(x) for x in args.which.split(",")] if args.which else list(range(args.shards))
    what = ["setup"]
    stop = threading.Event()
    th = threading.Thread(target=heartbeat, args=(stop, time.time(), what), daemon=True)
    th.start()
    print(json.dumps(dict(kind="setup", config=args.config, metric=args.metric, H=args.hub, k=k, span=span,
                          M=int(keys.numel()), shards=args.shards, ranges=ranges, gen_s=gen_s, create_s=create_s,
                          total_wedges_all=total_w)), flush=True)
    for s in which:
        ua, ub = ranges[s]
        what[0] = "shard %d [%d, %d)" % (s, ua, ub)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        n, t = G.predict_device(mid, args.hub, k, out, ua, ub)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t1) * 1e3
        kk = out[:n, 2].contiguous().view(torch.float32)
        b = kk.view(torch.int32).long() & 0xffffffff
        key = torch.where(b >= 0x80000000, 0xffffffff - b, b | 0x80000000)
        key[torch.isnan(kk)] = 0
        uk, cnt = torch.unique(key, return_counts=True)
        # canonical order check of the shard's list (score key desc, u asc, w asc)
        u = out[:n, 0].long() & 0xffffffff
        ww = out[:n, 1].long() & 0xffffffff
        dk, duu, dww = key[1:] - key[:-1], u[1:] - u[:-1], ww[1:] - ww[:-1]
        ordered = bool(((dk < 0) | ((dk == 0) & ((duu > 0) | ((duu == 0) & (dww > 0))))).all()) if n > 1 else True
        in_range = bool(((u >= ua) & (u < ub) & (u < ww)).all()) if n else True
        print(json.dumps(dict(kind="shard", shard=s, range=[ua, ub], ms=ms, predicted=n, wedges=t["wedges"],
                              candidates=t["candidates"], nan=t["nan_candidates"], chunks=t["chunks"], path=t["path"],
                              score_ms=t["score_ms"], select_ms=t["select_ms"],
                              wedges_per_s=t["wedges"] / (ms * 1e-3), canonical_order=ordered, in_range=in_range,
                              key_hist=[[int(a), int(c)] for a, c in zip(uk.tolist(), cnt.tolist())])), flush=True)
    stop.set()
    G.close()


def merge(files):
    setup, shards = None, {}
    for fn in files:
        for ln in open(fn):
            ln = ln.strip()
            if not ln.startswith("{"):
                continue
            d = json.loads(ln)
            if d["kind"] == "setup":
                setup = d
            else:
                shards[d["shard"]] = d
    P, k = setup["shards"], setup["k"]
    missing = [s for s in range(P) if s not in shards]
    # histogram-first selection (dist.select_quota) over the shards' key histograms
    hist = [dict((a, c) for a, c in shards[s]["key_hist"]) for s in range(P) if s in shards]
    allk = sorted({a for h in hist for a in h}, reverse=True)
    total = sum(sum(h.values()) for h in hist)
    take = min(total, k)
    acc, kth = 0, None
    for a in allk:
        c = sum(h.get(a, 0) for h in hist)
        if acc + c >= take:
            kth = a
            break
        acc += c
    above = [sum(c for a, c in h.items() if a > kth) for h in hist]
    ties = [h.get(kth, 0) for h in hist]
    quota = take - sum(above)
    shares, before = [], 0
    for s in range(len(hist)):
        q = min(ties[s], max(quota - before, 0))
        shares.append(above[s] + q)
        before += ties[s]
    ms = [shards[s]["ms"] for s in sorted(shards)]
    wed = sum(shards[s]["wedges"] for s in shards)
    return dict(config=setup["config"], metric=setup["metric"], H=setup["H"], k=k, shards=P, missing=missing,
                merged_count=sum(shares), kth_key=kth, shares=shares, above=above, ties=ties,
                shard_ms=ms, one_gpu_ms=sum(ms), eight_gpu_predict_ms=max(ms) if ms else None,
                wedges=wed, wedges_per_s_one_gpu=wed / (sum(ms) * 1e-3) if ms else None,
                candidates=sum(shards[s]["candidates"] for s in shards),
                all_canonical=all(shards[s]["canonical_order"] and shards[s]["in_range"] for s in shards),
                predicted_per_s_one_gpu=sum(shares) / (sum(ms) * 1e-3) if ms else None,
                predicted_per_s_eight_gpu_predict=sum(shares) / (max(ms) * 1e-3) if ms else None,
                ranges=setup["ranges"], gen_s=setup["gen_s"], create_s=setup["create_s"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5-sk-2005-ihub")
    ap.add_argument("--metric", default="CN")
    ap.add_argument("--hub", type=int, default=0)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--which", default="")
    ap.add_argument("--merge", nargs="*")
    args = ap.parse_args()
    if args.merge:
        print(json.dumps(merge(args.merge)))
    else:
        run(args)


if __name__ == "__main__":
    main()
