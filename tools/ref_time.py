"""Time the reference's own predictLinks<Metric>Omp<H> (oracle/_ref/ref_driver)
on a full-size stand-in (diagnostic: sizes full-size reference checks before
they enter the GPU suite).

    python tools/ref_time.py [--config C4-sk-2005] --calls JAC:32,AA:32 [--threads 16]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import nlp_loader  # noqa: E402

METRICS = ["CN", "JAC", "SOR", "SAL", "HPI", "HDI", "LHN", "AA", "RA"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4-sk-2005")
    ap.add_argument("--calls", default="JAC:32")
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--timeout", type=float, default=600)
    args = ap.parse_args()
    import numpy as np
    import torch
    import refcheck
    gg = nlp_loader.load_sub("graphgen")
    off, keys, du, dw, info = gg.make_workload(args.config, "cuda")
    k = info["k"]
    path, tmp = refcheck.write_csr(off.cpu().numpy().astype(np.uint64), keys.cpu().numpy().view(np.uint32))
    del off, keys
    torch.cuda.empty_cache()
    try:
        for c in args.calls.split(","):
            m, h = c.split(":")
            t0 = time.time()
            try:
                u, w, s, inf = refcheck.ref_predict(path, METRICS.index(m), int(h), k, threads=args.threads,
                                                    timeout=args.timeout)
            except Exception as e:  # the reference over the budget: report and go on
                print(json.dumps(dict(config=args.config, metric=m, H=int(h), error=repr(e)[:200],
                                      wall_s=time.time() - t0)), flush=True)
                continue
            print(json.dumps(dict(config=args.config, metric=m, H=int(h), k=k, n=inf["n"], ref_ms=inf["time_ms"],
                                  wall_s=time.time() - t0, threads=args.threads)), flush=True)
    finally:
        tmp.cleanup()


if __name__ == "__main__":
    main()
