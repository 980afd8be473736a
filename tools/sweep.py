"""Hub-threshold sweep (main.cxx:67-80 PREDICT_LINKS_ALL) on one GPU.

For the C2 stand-in (BASELINE.json configs[1]) and each metric / hub threshold
H, times predictLinks<Metric>Hip<H> on the GPU (graph resident, device output,
the last of `--reps` calls) and, for a bounded set of H, the reference's own
OpenMP code (oracle/_ref/ref_driver, all host cores; OMP_NUM_THREADS caps them) on the same CSR.
One JSON line per (metric, H) on stdout.

    python tools/sweep.py [--metrics JAC,CN,AA] [--hubs 0,2,4,...] [--cpu-hubs 2,4,8,16,32,64]
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nlp_loader  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2-soc-LiveJournal1")
    ap.add_argument("--metrics", default="JAC,CN,AA")
    ap.add_argument("--hubs", default="0,2,4,8,16,32,64,128,256,512,1024")
    ap.add_argument("--cpu-hubs", default="2,4,8,16,32,64")
    ap.add_argument("--cpu-metrics", default="JAC")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--envs", default="",
                    help="';'-separated environment settings (A=1,B=2), one graph handle each (the library reads "
                         "its switches when a handle is created); '' = the current environment")
    args = ap.parse_args()
    nlp = nlp_loader.load()
    gg = nlp_loader.load_sub("graphgen")
    off, keys, du, dw, info = gg.make_workload(gg.CONFIGS[args.config], "cuda")
    torch.cuda.synchronize()
    torch.cuda.empty_cache()  # hand the generator's cached blocks back: libnlp allocates with hipMalloc
    torch.cuda.synchronize()
    k = info["k"]
    out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    cpu_hubs = {int(h) for h in args.cpu_hubs.split(",") if h}
    csr = None
    if cpu_hubs:  # the reference driver reads the CSR from a file
        tmp = tempfile.mkdtemp()
        csr = os.path.join(tmp, "g.csr")
        with open(csr, "wb") as f:
            o = off.cpu().numpy().astype(np.uint64)
            np.array([len(o) - 1, keys.numel()], np.uint64).tofile(f)
            o.tofile(f)
            keys.cpu().numpy().view(np.uint32).tofile(f)
    # algorithmic bytes of the reference's wedge scan per call,
    # B_alg(H) = 8(S+1) + 4M + 4M + 8 P_H + 4 W_H + 12 k_out
    degs = (off[1:] - off[:-1]).double()
    span, nnz = off.numel() - 1, keys.numel()

    def b_alg(H, kout):
        sv = degs[(degs > 0) & ((degs <= H) if H > 0 else (degs > 0))]
        return 8 * (span + 1) + 8 * nnz + 8 * float(sv.sum()) + 4 * float((sv * sv).sum()) + 12 * kout
    cpu_metrics = set(args.cpu_metrics.split(","))
    for envspec in args.envs.split(";"):
        env = dict(kv.split("=", 1) for kv in envspec.split(",") if "=" in kv)
        saved = {kk: os.environ.get(kk) for kk in env}
        os.environ.update(env)
        G = nlp.Graph.from_device(off, keys)
        for kk, vv in saved.items():  # the handle has read its switches
            if vv is None:
                os.environ.pop(kk, None)
            else:
                os.environ[kk] = vv
        run_sweep(args, nlp, G, out, k, span, nnz, b_alg, csr, cpu_hubs, cpu_metrics, drv, cores, envspec)
        G.close()


def _checksum(out, cnt):
    """Position-weighted sum of the links (u, w, score bits): equal outputs give equal sums."""
    x = out[:cnt].to(torch.int64)
    pos = torch.arange(1, cnt + 1, device=out.device, dtype=torch.int64)
    return int(((x[:, 0] * 1000003 + x[:, 1]) * 1000033 + x[:, 2]).mul(pos).sum().item())


def run_sweep(args, nlp, G, out, k, span, nnz, b_alg, csr, cpu_hubs, cpu_metrics, drv, cores, envspec):
    for metric in args.metrics.split(","):
        mid = nlp.METRICS.index(metric)
        for H in (int(h) for h in args.hubs.split(",")):
            for _ in range(args.reps):
                t0 = time.perf_counter()
                cnt, t = G.predict_device(mid, H, k, out)
                torch.cuda.synchronize()
                wall = (time.perf_counter() - t0) * 1e3
            line = {"config": args.config, "env": envspec, "metric": metric, "H": H, "k": k, "predicted": cnt,
                    "gpu_ms": wall, "score_ms": t["score_ms"], "select_ms": t["select_ms"], "path": t["path"],
                    "chunks": t["chunks"], "wedges": t["wedges"], "candidates": t["candidates"],
                    "hot_kernel": t.get("hot_kernel"), "hot_ms": t.get("hot_ms"), "hot_bytes": t.get("hot_bytes"),
                    "gpu_predicted_per_s": cnt / (wall / 1e3), "gpu_wedges_per_s": t["wedges"] / (wall / 1e3),
                    "n": span - 1, "M": nnz, "order_route": t.get("order_route"),
                    "checksum": _checksum(out, cnt)}
            ba = b_alg(H, cnt)
            line.update(call_alg_bytes=ba, call_effective_gbs=ba / (wall / 1e3) / 1e9)
            if csr and H in cpu_hubs and metric in cpu_metrics and os.path.exists(drv):
                me = min(k, t["candidates"])
                env = dict(os.environ, OMP_NUM_THREADS=str(cores))
                r = subprocess.run([drv, "time", csr, str(mid), str(H), str(me), str(cores), "1"], capture_output=True,
                                   text=True, env=env, timeout=900)
                if r.returncode == 0:
                    t_ms, ts_ms, n = r.stdout.split()
                    line.update(cpu_ms=float(t_ms), cpu_cores=cores, cpu_kind="reference",
                                speedup=float(t_ms) / wall)
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
