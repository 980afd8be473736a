"""Probe: host time of enqueuing K asynchronous calls vs the batch's total
(does hipGraphLaunch of a running graph exec block?)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import nlp_loader  # noqa: E402

nlp = nlp_loader.load()
gg = nlp_loader.load_sub("graphgen")
n, m, alpha, seed, d, metric, hub = gg.CONFIGS["C2-soc-LiveJournal1"]
off, keys, du, dw, info = gg.make_workload((n, m, alpha, seed, d, metric, hub), "cuda")
torch.cuda.empty_cache()
G = nlp.Graph.from_device(off, keys)
k = info["k"]
out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
mid = nlp.METRICS.index(metric)
for _ in range(5):
    G.predict_device(mid, hub, k, out, stream=st)
torch.cuda.synchronize()
K = 100
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(K):
        G.predict_device_async(mid, hub, k, out, stream=st)
    t1 = time.perf_counter()
    G.sync()
    t2 = time.perf_counter()
    print("async: enqueue %.1f us/call, total %.1f us/call" % ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6), flush=True)
    t0 = time.perf_counter()
    for _ in range(K):
        G.predict_device(mid, hub, k, out, stream=st)
    t1 = time.perf_counter()
    print("sync: %.1f us/call" % ((t1 - t0) / K * 1e6), flush=True)
G.close()
