"""bench.py -- predicted edges/s of the link-prediction hot path on MI355X.

BASELINE.json metric: "predicted edges/sec + F1, LHub Jaccard, 0.1|E| removed,
1/2/4/8 MI355X".  Workload (N=1): configs[1], the soc-LiveJournal1-shaped
Chung-Lu stand-in (n = 4,847,571, m = 68,993,773, alpha 0.6, seed 12; SURVEY
§8(d) C2), symmetrized, 0.1|E| undirected edges deleted, then
predictLinksJaccardCoefficient<4> with maxEdges = |deletions| / 2
(main.cxx:50).  A step = one full prediction (score + top-k select + order)
with the graph resident in HBM; for N > 1 it also includes the RCCL exchange
and merge.  Scaling is weak: at N GPUs the graph is N x configs[1] (n and m
scaled) and each rank owns 1/N of the source vertices.

At N = 1 the K timed calls are enqueued back to back (nlp_predict_device_async,
one nlp_sync at the end: every call recomputes the whole prediction, only the
host wait between calls is gone -- a serving loop); the synchronous per-call
latency of the drop-in API is reported beside it (sync_call_ms), and --sync
times the synchronous calls instead.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--sync]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import nlp_loader  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (spec)
HOT_KERNELS = {1: "k_sp_bucket", 2: "k_sp_scan<F_Runs>", 3: "k_group_tiles", 4: "k_sp_survivors",
               5: "k_sp_expand", 6: "k_sp_pass", 7: "k_sp_runs", 8: "k_sp_group",
               9: "k_sp_grouprun"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def f1_on_device(G, out, n, du, dw):
    """main.cxx:48-57,199-206: P = |ins1 ∩ del0| / |ins1|, R = ... / |del0|, with
    |ins1 ∩ del0| counted by the library's evaluation kernel (nlp_set_truth,
    nlp_count_common_device); |ins1| = 2n (both directions of n distinct links)."""
    G.set_truth(du.cpu().numpy().astype(np.uint32), dw.cpu().numpy().astype(np.uint32))
    common = G.count_common_device(out, n)
    p = common / max(2 * n, 1)
    r = common / max(int(du.numel()), 1)
    return p, r, (0.0 if p + r == 0 else 2 * p * r / (p + r))


def cpu_baseline(off, keys, metric, hub, k, ncand, threads=None):
    """The reference's own OpenMP path (oracle/_ref/ref_driver, compiled from
    /root/reference/inc by oracle/Makefile) on this host's cores, same graph.
    maxEdges is capped at the candidate count: above it the reference's
    OpenMP merge reads past its per-thread lists."""
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)), 16))
    if threads:
        cores = threads
    metric_id = ["CN", "JAC", "SOR", "SAL", "HPI", "HDI", "LHN", "AA", "RA"].index(metric)
    me = min(k, ncand) if ncand else k
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "g.csr")
        with open(path, "wb") as f:
            np.array([len(off) - 1, len(keys)], np.uint64).tofile(f)
            off.astype(np.uint64).tofile(f)
            keys.astype(np.uint32).tofile(f)
        if os.path.exists(drv):
            env = dict(os.environ, OMP_NUM_THREADS=str(cores))
            r = subprocess.run([drv, "time", path, str(metric_id), str(hub), str(me), str(cores), "3"],
                               capture_output=True, text=True, env=env, timeout=900)
            if r.returncode == 0:
                t_ms, ts_ms, n = r.stdout.split()
                t_ms = float(t_ms)
                return dict(value=int(n) / (t_ms / 1e3) if t_ms > 0 else None, unit="predicted edges/s",
                            cores=cores, kind="reference", time_ms=t_ms, scoring_ms=float(ts_ms),
                            sample="full workload, predictLinks%sOmp<%d> repeat=3, maxEdges=%d"
                                   % (metric, hub, me))
    # fallback: the single-threaded C restatement (port)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    t0 = time.perf_counter()
    u, _, _, _ = pyoracle.predict(off, keys, metric, hub, max_edges=k)
    dt = time.perf_counter() - t0
    return dict(value=len(u) / dt, unit="predicted edges/s", cores=1, kind="port", time_ms=dt * 1e3,
                sample="full workload, oracle/nlp_oracle.c single thread")


def pmc_traffic(config, world, metric, hub):
    """HBM bytes per launch of the dominant kernel from the committed PMC
    summary (tools/pmc_summary.py over tools/gpu_pmc.sh's separate FETCH_SIZE /
    WRITE_SIZE passes of this same bench command, corrected as
    MI355X_MICROARCH.md's HBM section prescribes).  None when absent or for
    another workload."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("config") != config or d.get("n_gpus") != world or d.get("metric") != metric or d.get("hub") != hub:
        return None
    k = d.get("hot_kernel", "k_sp_bucket")
    if k not in d.get("kernels", {}):
        return None
    return {"bytes_per_launch": d["kernels"][k]["traffic_bytes"], "source": d.get("source"), "kernel": k}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2-soc-LiveJournal1")
    ap.add_argument("--metric", default=None)
    ap.add_argument("--hub", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sync", action="store_true", help="N = 1: time synchronous calls (no pipelining)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    nlp = nlp_loader.load()
    gg = nlp_loader.load_sub("graphgen")
    dmod = nlp_loader.load_sub("dist")
    nlp.lib()

    n, m, alpha, seed, d, metric, hub = gg.CONFIGS[args.config]
    metric = args.metric or metric
    hub = hub if args.hub is None else args.hub
    spec = (n * world, m * world, alpha, seed, d, metric, hub)
    t0 = time.time()
    off, keys, du, dw, info = gg.make_workload(spec, "cuda")
    torch.cuda.empty_cache()  # hand the generator's cached blocks back: libnlp allocates with hipMalloc
    torch.cuda.synchronize()
    gen_s = time.time() - t0
    t0 = time.time()
    G = nlp.Graph.from_device(off, keys)
    torch.cuda.synchronize()
    create_s = time.time() - t0
    ginfo = G.info()
    span = ginfo["span"]
    k = info["k"]
    stream = torch.cuda.current_stream()
    out_local = torch.empty((k + 1, 3), dtype=torch.int32, device="cuda")  # block: header + local top-k
    out = torch.empty((max(k, 1), 3), dtype=torch.int32, device="cuda")
    mid = nlp.METRICS.index(metric)
    last = {}
    xstate = dmod.Exchange()  # all_gather stride, learnt by the first (warmup) step
    # shard bounds balanced by the per-source wedge estimate, once per graph
    weights = dmod.source_weights(off, keys, hub) if world > 1 else None

    def step():
        if world == 1:
            cnt, t = G.predict_device(mid, hub, k, out, stream=stream)
            last.update(t)
            return cnt
        res, cnt, inf = dmod.predict_sharded(dmod.hip_local_predict(G, mid, hub, k, out_local, stream),
                                             dmod.hip_merge(G, out, stream), span, k, state=xstate,
                                             weights=weights)
        last.update(inf)
        return cnt

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # per-phase device time of the library's own events, averaged over the timed steps
    score_ms = select_ms = hot_ms = 0.0
    hot_bytes = replays = 0
    pipelined = world == 1 and not args.sync
    t0 = time.perf_counter()
    if pipelined:
        for _ in range(args.steps):
            G.predict_device_async(mid, hub, k, out, stream=stream)
        try:
            cnt, t = G.sync()
        except nlp.NlpError as e:  # a call of the batch needs a synchronous redo: time synchronous calls
            if e.status != 6:
                raise
            log("bench: asynchronous batch needs a redo (%s); timing synchronous calls" % e)
            pipelined = False
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        else:
            last.update(t)
            score_ms, select_ms, hot_ms = (args.steps * last.get(x, 0.0) for x in ("score_ms", "select_ms", "hot_ms"))
            hot_bytes = args.steps * int(last.get("hot_bytes", 0))
            replays = args.steps * int(last.get("graph_replay", 0))
    if not pipelined:
        for _ in range(args.steps):
            cnt = step()
            score_ms += last.get("score_ms", 0.0)
            select_ms += last.get("select_ms", 0.0)
            hot_ms += last.get("hot_ms", 0.0)
            hot_bytes += int(last.get("hot_bytes", 0))
            replays += int(last.get("graph_replay", 0))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = cnt / (elapsed / args.steps)

    sync_call_ms = None
    if world == 1:  # the drop-in API's synchronous call latency (outside the timed region)
        t1 = time.perf_counter()
        for _ in range(max(5, min(args.steps, 50))):
            step()
        sync_call_ms = (time.perf_counter() - t1) / max(5, min(args.steps, 50)) * 1e3
    if rank == 0:
        p, r, f1 = f1_on_device(G, out, cnt, du, dw)
        score_ms /= args.steps
        select_ms /= args.steps
        # Roofline of the dominant kernel, k_group_tiles: its
        # algorithmic bytes per launch (4*nU bucket counts + 8*W records + 4*W
        # run flags + 12*C runs, from the call's own counters) over its device
        # time, from the HIP events the library records around that launch on
        # the stream it runs on, averaged over the timed steps.
        wedges = int(last.get("wedges", 0))
        cands = int(last.get("candidates", 0))
        hot_ms /= args.steps
        hot_bytes //= args.steps
        achieved = hot_bytes / (hot_ms * 1e-3) / 1e9 if hot_ms > 0 else None
        traffic = pmc_traffic(args.config, world, metric, hub)
        # Whole-call effective bandwidth against SURVEY.md §8(d)'s algorithmic
        # bytes of the reference's wedge scan: B_alg(H) = 8(S+1) + 4M + 4M + 8 P_H
        # + 4 W_H + 12 k_out, with P_H = sum deg v and W_H = sum deg(v)^2 over the
        # surviving intermediates (H = 0: all).  Our kernels avoid most of these
        # bytes, so this is an effective figure, reported beside the roofline.
        degs = (off[1:] - off[:-1]).double()
        surv = degs[(degs > 0) & ((degs <= hub) if hub > 0 else (degs > 0))]
        b_call = 8 * (span + 1) + 8 * ginfo["nnz"] + 8 * float(surv.sum()) + 4 * float((surv * surv).sum()) + 12 * cnt
        call_eff = b_call / (ms_per_step * 1e-3) / 1e9
        line = {
            "metric": "predicted edges/sec + F1, LHub Jaccard, 0.1|E| removed",
            "value": value,
            "unit": "predicted edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32/f32",
            "data": "synthetic (Chung-Lu stand-in of %s, generated on device)" % args.config,
            "config": {"workload": "%s x%d: predictLinks%sOmp<%d>, k=|del|/2" % (args.config, world, metric, hub),
                       "n": spec[0], "m": spec[1], "alpha": alpha, "M": ginfo["nnz"], "k": k,
                       "deletion_fraction": d, "parallelism": "source-range shards x%d" % world},
            "predicted": cnt,
            # the reference's README quotes "edges/s" without a definition,
            # so the graph's adjacency entries per second of prediction are reported too
            "graph_entries_per_s": ginfo["nnz"] / (ms_per_step * 1e-3),
            "f1": f1, "precision": p, "recall": r,
            "score_ms": score_ms, "select_ms": select_ms,
            "host_overhead_ms": ms_per_step - score_ms - select_ms,
            "wedges": wedges, "candidates": cands, "path": last.get("path"),
            "graph_gen_s": gen_s, "graph_create_s": create_s,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                         "traffic": traffic["bytes_per_launch"] if traffic else None,
                         "kernel": HOT_KERNELS.get(int(last.get("hot_kernel", 0)), "?"),
                         "algorithmic_bytes": hot_bytes, "kernel_ms": hot_ms,
                         "traffic_source": traffic["source"] if traffic else None},
            "graph_replay": replays == args.steps,
            "pipelined": pipelined, "sync_call_ms": sync_call_ms,
            "call_effective": {"algorithmic_bytes": b_call, "achieved": call_eff, "unit": "GB/s",
                               "frac": call_eff / HBM_PEAK_GBS, "definition": "SURVEY.md 8(d) B_alg(H) per call"},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                h_off, h_keys = off.cpu().numpy(), keys.cpu().numpy().view(np.uint32)
                line["cpu_baseline"] = cpu_baseline(h_off, h_keys, metric, hub, k, cands)
                # the 1-thread time beside the all-cores one
                line["cpu_baseline_1thread"] = cpu_baseline(h_off, h_keys, metric, hub, k, cands, threads=1)
            except Exception as e:  # report, never hide
                line["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(line), flush=True)
    G.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
