"""Wall time per predict_device call vs device span (host overhead probe)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import nlp_loader
nlp = nlp_loader.load()
gg = nlp_loader.load_sub("graphgen")
off, keys, du, dw, info = gg.make_workload("C2-soc-LiveJournal1", "cuda")
G = nlp.Graph.from_device(off, keys)
k = info["k"]
out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
for _ in range(20):
    G.predict_device(1, 4, k, out, stream=st)
torch.cuda.synchronize()
n = 300
t0 = time.perf_counter()
tot = 0.0
for _ in range(n):
    c, t = G.predict_device(1, 4, k, out, stream=st)
    tot += t["total_ms"]
el = (time.perf_counter() - t0) / n * 1e6
print("wall %.1f us/call, device span %.1f us, python+lib overhead %.1f us" % (el, tot / n * 1e3, el - tot / n * 1e3))
t0 = time.perf_counter()
for _ in range(n):
    G.lib_predict_raw = None
el2 = (time.perf_counter() - t0) / n * 1e6
