"""One-GPU rehearsal of the N-rank bench step (bench.py --gpus N): the N x
configs[1] graph, every rank's source-range prediction run one after another on
this GPU, the all_gather replaced by device copies into the block layout, then
the block merge.  Reports per-rank predict time, the merge time, and checks the
merged result against the single-range prediction (canonical order, bit-exact).

    python tools/shard_emul.py --ranks 8 [--steps 5]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nlp_loader  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--config", default="C2-soc-LiveJournal1")
    args = ap.parse_args()
    nlp = nlp_loader.load()
    gg = nlp_loader.load_sub("graphgen")
    dmod = nlp_loader.load_sub("dist")
    N = args.ranks
    n, m, alpha, seed, d, metric, hub = gg.CONFIGS[args.config]
    off, keys, du, dw, info = gg.make_workload((n * N, m * N, alpha, seed, d, metric, hub), "cuda")
    k = info["k"]
    mid = nlp.METRICS.index(metric)
    st = torch.cuda.current_stream()
    res = {"ranks": N, "k": k}
    with nlp.Graph.from_device(off, keys) as G:
        span = G.info()["span"]
        ranges = dmod.shard_ranges(span, N, dmod.source_weights(off, keys, hub) if os.environ.get("BALANCE", "1") == "1"
                                   else None)
        local = [torch.empty((k + 1, 3), dtype=torch.int32, device="cuda") for _ in range(N)]
        out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
        full = torch.empty((k, 3), dtype=torch.int32, device="cuda")
        nf, _ = G.predict_device(mid, hub, k, full)  # warm + the single-range answer
        # each rank's steps back to back on its own range (a rank keeps one range,
        # so its per-range state -- the range index, captured graphs -- stays warm)
        pred_ms, counts = [], []
        for r, (ub, ue) in enumerate(ranges):
            ts = []
            for step in range(args.steps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                c, _ = G.predict_device(mid, hub, k, local[r][1:], ub, ue, stream=st)
                dmod.write_header(local[r], c)
                e1.record(st)
                torch.cuda.synchronize()
                if step:
                    ts.append(e0.elapsed_time(e1))
            pred_ms.append(float(np.mean(ts)))
            counts.append(c)
        stride = dmod._grow(max(counts), k) + 1
        merge_ms, copy_ms = [], []
        for step in range(args.steps + 1):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(st)
            blocks = torch.stack([b[:stride] for b in local])  # stands in for the all_gather
            ev[1].record(st)
            kk = G.merge_blocks_device(blocks, k, out, stream=st)
            ev[2].record(st)
            torch.cuda.synchronize()
            if step:
                copy_ms.append(ev[0].elapsed_time(ev[1]))
                merge_ms.append(ev[1].elapsed_time(ev[2]))
        ok = kk == nf and torch.equal(out[:kk], full[:nf])
        if not ok:  # diagnose: each rank's block against the single-range result restricted to its range
            fa = full[:nf].cpu().numpy()
            fu = fa[:, 0].view(np.uint32)
            diag = {"single": nf}
            for r, (ub, ue) in enumerate(ranges):
                want = fa[(fu >= ub) & (fu < ue)]
                got = local[r][1:1 + counts[r]].cpu().numpy()
                same = want.shape == got.shape and np.array_equal(want, got)
                diag["rank%d" % r] = {"want": len(want), "got": len(got), "equal": bool(same)}
                if not same and want.shape == got.shape:
                    i = int(np.argmax((want != got).any(axis=1)))
                    diag["rank%d" % r]["first_diff"] = [i, want[i].view(np.uint32).tolist(), got[i].view(np.uint32).tolist()]
            mo = out[:kk].cpu().numpy()
            if mo.shape == fa.shape:
                i = int(np.argmax((mo != fa).any(axis=1)))
                diag["merge_first_diff"] = [i, fa[i].view(np.uint32).tolist(), mo[i].view(np.uint32).tolist()]
            res["diag"] = diag
        res.update(counts=counts, stride=stride, merged=kk, equal_single_range=bool(ok),
                   predict_ms_per_rank=pred_ms,
                   block_copy_ms=float(np.mean(copy_ms)), merge_ms=float(np.mean(merge_ms)))
    print(json.dumps(res), flush=True)
    if not res["equal_single_range"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
