"""One PREDICT_LINKS_ALL batch timed end to end: the
reference's unit of work is a batch graph and its 9 metrics x hub thresholds
(main.cxx:67-80, 157-179, 208-221), so the per-graph build (nlp_graph_create)
and the drop-in's fingerprint show up here, not in a single resident call.

  python tools/batch_all.py [--config C2-soc-LiveJournal1] [--hubs 2,4,8,16,32,64]
                            [--ref-budget 300] [--dropin-timeout 900] --out FILE

1. The config's Chung-Lu pairs (graphgen, the bench's generator) are written
   as a MatrixMarket file in /dev/shm (tools/mtxwrite.c).
2. nlp_main reads it (device ingest), deletes 0.1|E| on the device with
   std::default_random_engine(seed + 1000) -- the bench's batch graph -- builds
   the graph once and runs the 9 metrics x the hubs, one line per call
   (main.cxx's format): wall time of the process, of the build, of the calls.
3. oracle/_ref/main_dropin -- the reference's own main.cxx compiled against
   include/nlp/predict.hxx -- on the same file: its compiled-in sweep (H = 0 and
   2..1024, main.cxx:67-80), the lines that finish within the timeout.
4. The reference's own predictLinks<Metric>Omp<H> (oracle/_ref/ref_driver) on
   the same batch graph's CSR for the (metric, H) calls, in the nlp_main order,
   while the budget lasts.
One JSON object is written to --out."""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nlp_loader  # noqa: E402

METRICS = ["CN", "JAC", "SOR", "SAL", "HPI", "HDI", "LHN", "AA", "RA"]
LINE = re.compile(r"\{-[^/]+/\+(\S+) batchf, (\d+) threads\} -> \{\s*([\d.]+)ms,\s*([\d.]+)ms scoring, "
                  r"(\S+) precision, (\S+) recall\} (\w+?)(\d+)$")


def parse_lines(text):
    out = []
    for ln in text.splitlines():
        m = LINE.search(ln.strip())
        if m:
            out.append(dict(fn=m.group(7), H=int(m.group(8)), ms=float(m.group(3)), scoring_ms=float(m.group(4)),
                            precision=float(m.group(5)), recall=float(m.group(6))))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2-soc-LiveJournal1")
    ap.add_argument("--hubs", default="2,4,8,16,32,64")
    ap.add_argument("--ref-budget", type=float, default=300.0)
    ap.add_argument("--dropin-timeout", type=float, default=900.0)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    import torch
    gg = nlp_loader.load_sub("graphgen")
    n, m, alpha, seed, d, metric, hub = gg.CONFIGS[args.config]
    res = dict(config=args.config, n=n, m=m, deletion_fraction=d, hubs=args.hubs, metrics=METRICS)
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else None
    tmp = tempfile.TemporaryDirectory(dir=shm)
    try:
        # 1. the MatrixMarket file
        t0 = time.time()
        src, dst = gg.chung_lu_edges(n, m, alpha, seed, "cuda")
        pb = os.path.join(tmp.name, "pairs.bin")
        with open(pb, "wb") as f:
            src.to(torch.int32).cpu().numpy().tofile(f)
            dst.to(torch.int32).cpu().numpy().tofile(f)
        del src, dst
        torch.cuda.empty_cache()
        bindir = tempfile.mkdtemp()  # /dev/shm may be mounted noexec
        mw = os.path.join(bindir, "mtxwrite")
        subprocess.run(["gcc", "-O2", "-o", mw, os.path.join(ROOT, "tools", "mtxwrite.c")], check=True)
        mtx = os.path.join(tmp.name, "g.mtx")
        subprocess.run([mw, pb, str(n), mtx], check=True)
        os.unlink(pb)
        res["mtx_write_s"] = time.time() - t0
        res["mtx_bytes"] = os.path.getsize(mtx)
        env = dict(os.environ, BATCH_DELETIONS_BEGIN=str(d), BATCH_DELETIONS_END=str(d), REPEAT_BATCH="1",
                   BATCH_LENGTH="1", REPEAT_METHOD="1", NLP_SEED=str(seed + 1000), NLP_HUBS=args.hubs,
                   MAX_THREADS=os.environ.get("OMP_NUM_THREADS", "16"))
        # 2. nlp_main
        exe = os.path.join(ROOT, "neighborhood-link-prediction-openmp_amd", "nlp_main")
        t0 = time.time()
        r = subprocess.run([exe, mtx], capture_output=True, text=True, env=env, timeout=1200)
        wall = time.time() - t0
        if r.returncode != 0:
            raise RuntimeError("nlp_main: " + r.stderr[-1000:])
        calls = parse_lines(r.stdout)
        bl = [ln for ln in r.stdout.splitlines() if ln.startswith("graph build:")]
        build_ms = float(bl[0].split()[2]) if bl else None
        res["nlp_main"] = dict(wall_s=wall, calls=len(calls), build_ms=build_ms, build_line=bl[0] if bl else None,
                               calls_ms=sum(c["ms"] for c in calls),
                               per_call=calls, log_head=r.stdout.splitlines()[:8])
        # 3. the reference's main.cxx on the drop-in header
        dexe = os.path.join(ROOT, "oracle", "_ref", "main_dropin")
        if os.path.exists(dexe):
            t0 = time.time()
            try:
                r = subprocess.run([dexe, mtx], capture_output=True, text=True, env=env, timeout=args.dropin_timeout)
                out, rc = r.stdout, r.returncode
            except subprocess.TimeoutExpired as e:
                out, rc = (e.stdout.decode() if isinstance(e.stdout, bytes) else (e.stdout or "")), "timeout"
            dc = parse_lines(out)
            res["main_dropin"] = dict(wall_s=time.time() - t0, rc=rc, calls=len(dc), calls_ms=sum(c["ms"] for c in dc),
                                      per_call=dc)
        # 4. the reference's own OpenMP calls on the same batch graph
        drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
        if os.path.exists(drv):
            off, keys, du, dw, info = gg.make_workload((n, m, alpha, seed, d, metric, hub), "cuda")
            k = info["k"]
            csr = os.path.join(tmp.name, "g.csr")
            with open(csr, "wb") as f:
                o = off.cpu().numpy().astype(np.uint64)
                np.array([len(o) - 1, keys.numel()], np.uint64).tofile(f)
                o.tofile(f)
                keys.cpu().numpy().view(np.uint32).tofile(f)
            # maxEdges capped at the candidate count (from our own call): above it the
            # reference's OpenMP merge reads past its per-thread lists
            nlp = nlp_loader.load()
            G = nlp.Graph.from_device(off, keys)
            outb = torch.empty((max(k, 1), 3), dtype=torch.int32, device="cuda")
            ncand = {}
            for mi in range(len(METRICS)):
                for h in (int(x) for x in args.hubs.split(",")):
                    _, t = G.predict_device(mi, h, k, outb)
                    ncand[(mi, h)] = int(t["candidates"])
            G.close()
            del off, keys, du, dw, outb
            torch.cuda.empty_cache()
            threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
            ref = []
            t_start = time.time()
            for mi, mname in enumerate(METRICS):
                for h in (int(x) for x in args.hubs.split(",")):
                    left = args.ref_budget - (time.time() - t_start)
                    if left <= 5:
                        break
                    try:
                        me = max(1, min(k, ncand[(mi, h)]))
                        rr = subprocess.run([drv, "time", csr, str(mi), str(h), str(me), str(threads), "1"],
                                            capture_output=True, text=True, timeout=left,
                                            env=dict(os.environ, OMP_NUM_THREADS=str(threads)))
                    except subprocess.TimeoutExpired:
                        ref.append(dict(metric=mname, H=h, timeout=True))
                        break
                    if rr.returncode != 0:
                        ref.append(dict(metric=mname, H=h, error=rr.stderr[-200:]))
                        continue
                    t_ms, ts_ms, cnt = rr.stdout.split()
                    ref.append(dict(metric=mname, H=h, ms=float(t_ms), scoring_ms=float(ts_ms), predicted=int(cnt)))
            res["reference"] = dict(threads=threads, k=k, calls=ref, budget_s=args.ref_budget)
            # the same calls of nlp_main, matched
            ours = {(c["fn"], c["H"]): c["ms"] for c in calls}
            pairs = []
            for c in ref:
                if "ms" not in c:
                    continue
                fn = "predictLinks%sHip" % {"CN": "CommonNeighbors", "JAC": "JaccardCoefficient",
                                             "SOR": "SorensenIndex", "SAL": "SaltonCosineSimilarity",
                                             "HPI": "HubPromoted", "HDI": "HubDepressed",
                                             "LHN": "LeichtHolmeNermanScore", "AA": "AdamicAdarCoefficient",
                                             "RA": "ResourceAllocationScore"}[c["metric"]]
                if (fn, c["H"]) in ours:
                    pairs.append(dict(metric=c["metric"], H=c["H"], ref_ms=c["ms"], gpu_ms=ours[(fn, c["H"])]))
            res["matched"] = dict(calls=len(pairs), ref_ms=sum(p["ref_ms"] for p in pairs),
                                  gpu_ms=sum(p["gpu_ms"] for p in pairs), per_call=pairs)
    finally:
        tmp.cleanup()
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("reference",)}, default=str)[:3000])


if __name__ == "__main__":
    main()
