"""bench.py -- predicted edges/s of the link-prediction hot path on MI355X.

BASELINE.json metric: "predicted edges/sec + F1, LHub Jaccard, 0.1|E| removed,
1/2/4/8 MI355X", quoted by the reference on sk-2005 (README.md:9,17).
Workload: configs[3], the sk-2005-shaped Chung-Lu stand-in (n = 50,636,154,
m = 1,949,412,601, alpha 0.7, seed 14), symmetrized, 0.1|E|
undirected edges deleted (M = 3.53e9 adjacency entries, k = |deletions| / 2 =
1.8e8), then predictLinksJaccardCoefficient<4> with maxEdges = k exactly as
main.cxx:50 calls it.  It fits one MI355X, so N = 1 runs the whole config.

A step = one full synchronous prediction through the drop-in API
(nlp_predict_device: score + top-k select + canonical order, the call
returns with the result in HBM), graph resident in HBM.  For N > 1 a step
also includes the exchange: histogram-first quota selection over RCCL and one
all_gather of the ranks' shares, then the device merge (dist.py).  Scaling is
STRONG: every rank holds the same C4 graph and owns a wedge-balanced 1/N of
the source vertices, so N = 1 of the scaling curve is this line.

Built once per graph in nlp_graph_create and NOT timed (like the reference's
untimed graph load and table allocation, predict.hxx:420-424): the degrees,
the degree-class index, the transposed CSR (when asymmetric), the edge-
membership table and the AA/RA tables (graph_create_s in the line).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C] [--sweep H,H,...]
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
               9: "k_sp_grouprun", 10: "k_sp_exbucket"}
METRIC_NAMES = {"CN": "CommonNeighbors", "JAC": "JaccardCoefficient", "SOR": "SorensenIndex",
                "SAL": "SaltonCosineSimilarity", "HPI": "HubPromoted", "HDI": "HubDepressed",
                "LHN": "LeichtHolmeNermanScore", "AA": "AdamicAdarCoefficient", "RA": "ResourceAllocationScore"}


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


def host_cores():
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    return max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)), 16))


def ref_time(path, metric, hub, me, threads, timeout):
    """oracle/_ref/ref_driver time: the reference's own predictLinks<Metric>Omp
    (compiled from /root/reference/inc by oracle/Makefile) on the CSR file."""
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    metric_id = ["CN", "JAC", "SOR", "SAL", "HPI", "HDI", "LHN", "AA", "RA"].index(metric)
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    t0 = time.perf_counter()
    r = subprocess.run([drv, "time", path, str(metric_id), str(hub), str(me), str(threads), "1"],
                       capture_output=True, text=True, env=env, timeout=timeout)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError("ref_driver failed: %s" % r.stderr[-400:])
    t_ms, ts_ms, n = r.stdout.split()
    return float(t_ms), float(ts_ms), int(n), wall


def cpu_baseline(off, keys, metric, hub, k, ncand, budget_s=240.0):
    """The reference's own OpenMP path on this host's cores, same graph, same
    call (repeat 1), then the same on ONE thread when the all-cores time says
    it fits the budget.  maxEdges is capped at the candidate count: above it
    the reference's OpenMP merge reads past its per-thread lists (SURVEY
    Appendix A.2).  The CSR goes through /dev/shm (the driver reads a file).
    Returns (all-cores dict, 1-thread dict)."""
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    if not os.path.exists(drv):
        return {"error": "oracle/_ref/ref_driver not built"}, None
    cores = host_cores()
    me = min(k, ncand) if ncand else k
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else None
    with tempfile.TemporaryDirectory(dir=shm) as tmp:
        path = os.path.join(tmp, "g.csr")
        with open(path, "wb") as f:
            np.array([len(off) - 1, len(keys)], np.uint64).tofile(f)
            off.astype(np.uint64).tofile(f)
            keys.tofile(f)
        t0 = time.perf_counter()
        t_ms, ts_ms, n, wall = ref_time(path, metric, hub, me, cores, timeout=budget_s)
        sample = "full workload: predictLinks%sOmp<%d>(G, {repeat 1, maxEdges %d}), DiGraphCsr of the same CSR" % (
            METRIC_NAMES[metric], hub, me)
        full = dict(value=n / (t_ms / 1e3) if t_ms > 0 else None, unit="predicted edges/s", cores=cores,
                    kind="reference", time_ms=t_ms, scoring_ms=ts_ms, predicted=n, sample=sample,
                    driver_wall_s=wall)
        one = None
        left = budget_s - (time.perf_counter() - t0)
        est = t_ms / 1e3 * cores * 1.3 + (wall - t_ms / 1e3)  # linear in the cores, plus the CSR load
        if est < left:
            t1, ts1, n1, wall1 = ref_time(path, metric, hub, me, 1, timeout=left)
            one = dict(value=n1 / (t1 / 1e3) if t1 > 0 else None, unit="predicted edges/s", cores=1,
                       kind="reference", time_ms=t1, scoring_ms=ts1, predicted=n1, sample=sample)
        else:
            one = {"skipped": "estimated %.0f s on one thread > the %.0f s left of the baseline budget" % (est, left)}
    return full, one


def pmc_traffic(config, world, metric, hub, kernel):
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
    if kernel not in d.get("kernels", {}):
        return None
    return {"bytes_per_launch": d["kernels"][kernel]["traffic_bytes"], "source": d.get("source"), "kernel": kernel}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C4-sk-2005")
    ap.add_argument("--metric", default=None)
    ap.add_argument("--hub", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sweep", default="2,8,16,32",
                    help="N = 1: hub thresholds (main.cxx:67-80) timed once each after the timed region; '' = none")
    ap.add_argument("--pipelined", action="store_true",
                    help="N = 1: also time the same calls enqueued back to back (nlp_predict_device_async)")
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
    spec = (n, m, alpha, seed, d, metric, hub)  # strong scaling: the same graph on every rank
    t0 = time.time()
    off, keys, du, dw, info = gg.make_workload(spec, "cuda")
    torch.cuda.synchronize()
    torch.cuda.empty_cache()  # hand the generator's cached blocks back: libnlp allocates with hipMalloc
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
    xstate = dmod.Exchange()
    # shard bounds balanced by the per-source wedge estimate, once per graph
    weights = dmod.source_weights(off, keys, hub) if world > 1 else None

    def step():
        if world == 1:
            cnt, t = G.predict_device(mid, hub, k, out, stream=stream)
            last.clear()
            last.update(t)
            return cnt
        res, cnt, inf = dmod.predict_sharded(dmod.hip_local_predict(G, mid, hub, k, out_local, stream),
                                             dmod.hip_merge(G, out, stream), span, k, state=xstate,
                                             weights=weights)
        last.clear()
        last.update(inf)
        return cnt

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    score_ms = select_ms = hot_ms = 0.0
    hot_bytes = replays = 0
    t0 = time.perf_counter()
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
    timing = dict(last)

    pipelined_ms = None
    if world == 1 and args.pipelined:  # serving loop: the same calls without a host wait (outside the line's value)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            G.predict_device_async(mid, hub, k, out, stream=stream)
        try:
            G.sync()
            pipelined_ms = (time.perf_counter() - t1) / args.steps * 1e3
        except nlp.NlpError as e:
            log("bench: asynchronous batch needs a redo (%s)" % e)
        step()  # leave the synchronous result in `out`

    sweep = []
    if world == 1 and args.sweep not in ("", "none", "="):
        # the reference's MINDEGREE1 sweep (main.cxx:67-80) for the bench metric; one warm call each,
        # then the bench call again so `out` holds the line's result for F1
        out_s = torch.empty((max(k, 1), 3), dtype=torch.int32, device="cuda")
        for h in (int(x) for x in args.sweep.split(",") if x):
            G.predict_device(mid, h, k, out_s, stream=stream)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            c, t = G.predict_device(mid, h, k, out_s, stream=stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t1) * 1e3
            sweep.append(dict(H=h, ms=ms, predicted=c, predicted_per_s=c / (ms * 1e-3), wedges=t["wedges"],
                              candidates=t["candidates"], path=t["path"], chunks=t["chunks"]))
        del out_s
        cnt = step()
    if rank == 0:
        p, r, f1 = f1_on_device(G, out, cnt, du, dw)
        score_ms /= args.steps
        select_ms /= args.steps
        # Roofline of the dominant kernel of the step: its
        # algorithmic bytes per launch (from the call's own counters) over its
        # device time (the kernel's own s_memrealtime stamps on the stream it
        # runs on; rocprofv3 kernel trace of the same command in profiles/r03/),
        # averaged over the timed steps.
        hot_ms /= args.steps
        hot_bytes //= args.steps
        achieved = hot_bytes / (hot_ms * 1e-3) / 1e9 if hot_ms > 0 else None
        kname = HOT_KERNELS.get(int(timing.get("hot_kernel", 0)), "?")
        traffic = pmc_traffic(args.config, world, metric, hub, kname)
        line = {
            "metric": "predicted edges/sec + F1, LHub Jaccard, 0.1|E| removed",
            "value": value,
            "unit": "predicted edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32/f32",
            "data": "synthetic (Chung-Lu stand-in of %s, generated on device; SURVEY §8(d))" % args.config,
            "config": {"workload": "%s x%d: predictLinks%sOmp<%d>(G, {1, k = |del|/2}), synchronous drop-in call"
                                   % (args.config, world, METRIC_NAMES[metric], hub),
                       "n": spec[0], "m": spec[1], "alpha": alpha, "M": ginfo["nnz"], "k": k,
                       "deletion_fraction": d,
                       "parallelism": "source-range shards x%d, histogram-quota exchange" % world
                       if world > 1 else "one GPU"},
            "predicted": cnt,
            # the reference's README quotes "edges/s" without a definition,
            # so the graph's adjacency entries per second of prediction are reported too
            "graph_entries_per_s": ginfo["nnz"] / (ms_per_step * 1e-3),
            "f1": f1, "precision": p, "recall": r,
            "score_ms": score_ms, "select_ms": select_ms,
            "host_overhead_ms": ms_per_step - score_ms - select_ms if world == 1 else None,
            "wedges": int(timing.get("wedges", 0)), "candidates": int(timing.get("candidates", 0)),
            "path": timing.get("path"),
            "graph_gen_s": gen_s,
            "graph_create_s": create_s,
            "untimed_per_graph": "degrees, degree-class index, transposed CSR (if asymmetric), edge-membership "
                                 "table, AA/RA tables: built once in nlp_graph_create (graph_create_s)",
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                         "traffic": traffic["bytes_per_launch"] if traffic else None,
                         "kernel": kname, "algorithmic_bytes": hot_bytes, "kernel_ms": hot_ms,
                         "traffic_source": traffic["source"] if traffic else None} if world == 1 else None,
            "graph_replay": replays == args.steps if world == 1 else None,
            "pipelined_ms_per_step": pipelined_ms,
            "hub_sweep": sweep,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                h_off, h_keys = off.cpu().numpy(), keys.cpu().numpy().view(np.uint32)
                full, one = cpu_baseline(h_off, h_keys, metric, hub, k, int(timing.get("candidates", 0)))
                line["cpu_baseline"] = full
                line["cpu_baseline_1thread"] = one  # the 1-thread time beside the all-cores one
                del h_off, h_keys
            except Exception as e:  # report, never hide
                line["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(line), flush=True)
    G.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
