"""Debug: all-candidates calls on the golden g300 graph, counted passes on/off."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import nlp_loader  # noqa: E402

nlp = nlp_loader.load()
g = dict(np.load(os.path.join(ROOT, "tests", "golden", "g300.npz"), allow_pickle=False))
with nlp.Graph(g["offsets"], g["keys"], device=0) as G:
    for m, H in [(0, 0), (0, 4), (1, 0), (1, 4)]:
        ref = len(g["cand_%d_%d_u" % (m, H)]) if "cand_%d_%d_u" % (m, H) in g else -1
        for k in (None, 100000):
            u, w, s, t = G.predict(m, H, k)
            print("m", m, "H", H, "k", k, "got", len(u), "ref", ref, {x: t[x] for x in ("candidates", "wedges", "path")},
                  flush=True)
