"""Shared helpers of the full-size config tests (tests/test_gpu_c*.py): the
SURVEY §8(d) stand-in generated on the device, resident in one nlp_graph, with
host copies of the CSR for the parallel oracle (oracle/nlp_oracle.c
nlpo_predict_par).  One config per test module, so a module-scoped fixture
frees its HBM before the next module's graph is generated."""
import os
import time

import numpy as np

ORACLE_THREADS = int(os.environ.get("NLP_ORACLE_THREADS", "16"))


class Config:
    def __init__(self, nlp, name, spec_override=None):
        import torch
        import nlp_loader
        gg = nlp_loader.load_sub("graphgen")
        t0 = time.time()
        spec = gg.CONFIGS[name] if spec_override is None else spec_override
        off_t, keys_t, du, dw, info = gg.make_workload(spec, "cuda")
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        self.gen_s = time.time() - t0
        t0 = time.time()
        self.G = nlp.Graph.from_device(off_t, keys_t)
        torch.cuda.synchronize()
        self.create_s = time.time() - t0
        self.info = info
        self.k = info["k"]
        self.off = off_t.cpu().numpy().astype(np.uint64)
        self.keys = keys_t.cpu().numpy().view(np.uint32)
        self.off_t, self.keys_t = off_t, keys_t
        self.del_u, self.del_w = du, dw
        self.nlp = nlp
        self.name = name

    def out(self, n=None):
        import torch
        return torch.empty((max(self.k if n is None else n, 1), 3), dtype=torch.int32, device="cuda")

    def close(self):
        import torch
        self.G.close()
        self.off_t = self.keys_t = self.del_u = self.del_w = None
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
