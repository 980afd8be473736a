"""Diagnostics: path-4 results vs the oracle under several switches (GPU box)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import nlp_loader, pyoracle
nlp = nlp_loader.load()
g = dict(np.load(os.path.join(ROOT, "tests/golden/g3k.npz")))
off, keys = g["offsets"], g["keys"]
for env in (dict(NLP_HASH="1"), dict(NLP_HASH="1", NLP_HASH_MINBIN="1"), dict(NLP_HASH="1", NLP_HASH_MINBIN="2")):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    G = nlp.Graph(off, keys)
    for k_, v in old.items():
        if v is None: os.environ.pop(k_)
        else: os.environ[k_] = v
    for m, H, k in ((0, 0, None), (0, 16, None)):
        u, w, s, t = G.predict(m, H, k)
        eu, ew, es, info = pyoracle.predict(off, keys, m, H, max_edges=k if k else 10**9)
        pairs = set(zip(u.tolist(), w.tolist()))
        ok = np.array_equal(u, eu) and np.array_equal(w, ew)
        print(env, m, H, k, "ok" if ok else "DIFF", "n", len(u), len(eu), "uniq", len(pairs),
              "cands", t["candidates"], info["candidates"], "wedges", t["wedges"], info["wedges_gt"], "chunks", t["chunks"], flush=True)
        if not ok:
            from collections import Counter
            c = Counter(zip(u.tolist(), w.tolist()))
            print("   dups:", [p for p, n in c.items() if n > 1][:10], flush=True)
    G.close()
