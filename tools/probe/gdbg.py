import sys, time
sys.path.insert(0, "/root/repo")
import nlp_loader, numpy as np, torch
nlp = nlp_loader.load()
g = dict(np.load("/root/repo/tests/golden/g3k.npz"))
G = nlp.Graph(g["offsets"], g["keys"])
for i in range(3):
    u, w, s, t = G.predict(1, 4, 100)
    print(i, t["graph_replay"], t["hot_ms"], t["path"], len(u))
