"""Run the random-multigraph parity cases one by one and report failures
(NLP_DEBUG=1 prints the failing runtime step).  Diagnostics only."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import nlp_loader  # noqa: E402
from oracle import pyoracle  # noqa: E402
from test_gpu_parity import random_csr  # noqa: E402

gpu = nlp_loader.load()
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
off, keys = random_csr(4000 if seed == 1 else 20000, 12, seed)
bad = 0
with gpu.Graph(off, keys) as G:
    for m in range(9):
        for H in ((0, 1, 3, 4, 16) if seed == 1 else (2, 4, 8)):
            for k in (50, 5000):
                try:
                    u, w, s, t = G.predict(m, H, k)
                except Exception as e:  # noqa: BLE001
                    print("FAIL m=%d H=%d k=%d: %s" % (m, H, k, e), flush=True)
                    bad += 1
                    continue
                eu, ew, es, info = pyoracle.predict(off, keys, m, H, max_edges=k)
                ok = sorted(zip(eu.tolist(), ew.tolist())) == sorted(zip(u.tolist(), w.tolist()))
                if not ok:
                    print("MISMATCH m=%d H=%d k=%d path=%s" % (m, H, k, t.get("path")), flush=True)
                    bad += 1
print("bad", bad)
