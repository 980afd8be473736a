"""Diagnostic: the N=2 bench graph, rank 0's range on the GPU vs the oracle and
vs the full-range GPU result restricted to that range."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import nlp_loader, pyoracle
nlp = nlp_loader.load(); gg = nlp_loader.load_sub("graphgen")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n, m, alpha, seed, d, metric, hub = gg.CONFIGS["C2-soc-LiveJournal1"]
off, keys, du, dw, info = gg.make_workload((n * N, m * N, alpha, seed, d, metric, hub), "cuda")
k = info["k"]; mid = nlp.METRICS.index(metric)
offn = off.cpu().numpy().astype(np.uint64); keysn = keys.cpu().numpy().view(np.uint32)
span = len(offn) - 1
ub, ue = 0, span // N
def rows(t, c):
    a = t[:c].cpu().numpy(); return a
with nlp.Graph.from_device(off, keys) as G:
    for order in ("range_first", "full_first"):
        full = torch.empty((k, 3), dtype=torch.int32, device="cuda"); part = torch.empty((k, 3), dtype=torch.int32, device="cuda")
        if order == "range_first":
            c, t1 = G.predict_device(mid, hub, k, part, ub, ue); nf, t2 = G.predict_device(mid, hub, k, full)
        else:
            nf, t2 = G.predict_device(mid, hub, k, full); c, t1 = G.predict_device(mid, hub, k, part, ub, ue)
        fa = rows(full, nf); pa = rows(part, c)
        eu, ew, es, _ = pyoracle.predict(offn, keysn, mid, hub, max_edges=k, u_begin=ub, u_end=ue)
        ora = np.stack([eu.view(np.int32), ew.view(np.int32), es.view(np.int32)], 1)
        fu = fa[:, 0].view(np.uint32); fr = fa[(fu >= ub) & (fu < ue)]
        def canon(a):
            sc = a[:, 2].view(np.float32).astype(np.float64)
            o = np.lexsort((a[:, 1].view(np.uint32), a[:, 0].view(np.uint32), -sc))
            return a[o]
        same_set = pa.shape == ora.shape and np.array_equal(canon(pa), canon(ora))
        ndiff = int((pa != ora).any(axis=1).sum()) if pa.shape == ora.shape else -1
        bad_u = sorted(set(pa[(pa != ora).any(axis=1)][:, 0].view(np.uint32).tolist()))[:10] if ndiff > 0 else []
        print(order, "same multiset", same_set, "rows differing", ndiff, "u", bad_u, "ub", ue)
        print(order, "range vs oracle:", pa.shape == ora.shape and np.array_equal(pa, ora),
              "full|range vs oracle:", fr.shape == ora.shape and np.array_equal(fr, ora),
              "paths", t1["path"], t2["path"], "wedges", t1["wedges"], t2["wedges"], flush=True)
