import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")


class _MemoOracle:
    """pyoracle with predict() memoised on the graph's CONTENT (xxh3 of the
    offsets and keys bytes) and the call's arguments, for graphs up to
    MEMO_BYTES: the variant tests run the same oracle calls under every
    environment variant of the library, and the oracle's answer does not depend
    on it.  Results are returned as copies; larger graphs are not memoised."""
    MEMO_BYTES = 64 << 20

    def __init__(self, mod):
        self._mod = mod
        self._memo = {}

    def __getattr__(self, name):
        return getattr(self._mod, name)

    def predict(self, offsets, keys, *args, **kw):
        import xxhash
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ks = np.ascontiguousarray(keys, dtype=np.uint32)
        if off.nbytes + ks.nbytes > self.MEMO_BYTES:
            return self._mod.predict(off, ks, *args, **kw)
        key = (xxhash.xxh3_64_hexdigest(off.tobytes()), xxhash.xxh3_64_hexdigest(ks.tobytes()), len(off), len(ks),
               args, tuple(sorted(kw.items())))
        if key not in self._memo:
            self._memo[key] = self._mod.predict(off, ks, *args, **kw)
        u, w, s, info = self._memo[key]
        return u.copy(), w.copy(), s.copy(), dict(info)


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return _MemoOracle(pyoracle)


@pytest.fixture(scope="session")
def nlp():
    import nlp_loader
    return nlp_loader.load()


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def golden():
    return {n: load_golden(n) for n in ("g300", "g3k", "edge")}
