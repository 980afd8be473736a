"""Diagnostics: run the C2 workload at several hub thresholds / grouping
variants in one process and print per-call timing (GPU box)."""
import os, sys, time, json
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nlp_loader
nlp = nlp_loader.load()
gg = nlp_loader.load_sub("graphgen")

def main():
    cfg = os.environ.get("TRY_CONFIG", "C2-soc-LiveJournal1")
    runs = [r.split(":") for r in sys.argv[1:]]  # metric:H:ENV=V,ENV=V
    off, keys, du, dw, info = gg.make_workload(gg.CONFIGS[cfg], "cuda")
    torch.cuda.synchronize()
    k = info["k"]
    out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
    ref = {}
    for r in runs:
        metric, H = r[0], int(r[1])
        env = dict(kv.split("=") for kv in r[2].split(",")) if len(r) > 2 and r[2] else {}
        saved = {e: os.environ.get(e) for e in env}
        os.environ.update(env)
        G = nlp.Graph.from_device(off, keys)
        for e, v in saved.items():
            if v is None: os.environ.pop(e, None)
            else: os.environ[e] = v
        print("run", metric, H, env, flush=True)
        try:
            for rep in range(int(os.environ.get("TRY_REPS", "2"))):
                t0 = time.perf_counter()
                cnt, t = G.predict_device(nlp.METRICS.index(metric), H, k, out)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                print("  wall %.3f ms cnt %d path %s chunks %s wedges %s cands %s score %.3f sel %.3f" % (
                    dt * 1e3, cnt, t["path"], t["chunks"], t["wedges"], t["candidates"], t["score_ms"], t["select_ms"]), flush=True)
            h = out[:cnt].cpu()
            key = (metric, H)
            if key in ref:
                print("  equal to first variant:", bool(torch.equal(ref[key], h)), flush=True)
            else:
                ref[key] = h
        except Exception as e:
            print("  ERROR", repr(e), flush=True)
        G.close()

main()
