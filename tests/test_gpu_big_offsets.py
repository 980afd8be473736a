"""A graph with more than 2^32 adjacency entries (every adjacency offset and
position beyond u32), checked exactly against the oracle.

No config reaches 2^32 entries (C4 has 3.53e9), so this graph is built for it:
a small power-law multigraph (duplicates, asymmetric entries) whose vertex ids
are split around 64 "giant" vertices inserted in the middle of the id range,
each with ~69 M entries pointing at 2^20 "sink" vertices of degree 0 (sorted,
with duplicates).  Giants only reach sinks and sinks have no edges, so no
wedge, candidate or degree of a small-graph vertex changes: the expected
result is the oracle's on the small graph with the same id remap (monotone, so
the canonical order is kept).  The small graph's upper half sits at offsets
beyond 2^32, and the giants make every per-graph pass (degrees, key check,
transpose, tile rows of path 4, the edge filter) run over > 2^32 entries."""
import numpy as np
import pytest

from parity import assert_canonical_equal, assert_canonical_order
from test_gpu_parity import random_csr

pytestmark = pytest.mark.gpu

GIANTS = 64
SINKS = 1 << 20
TOTAL = (1 << 32) + (1 << 28)  # entries of the giant rows


@pytest.fixture(scope="module")
def big(nlp):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    off_s, keys_s = random_csr(20000, 12, 7)
    n_s = len(off_s) - 2
    mid = n_s // 2

    def remap(x):
        x = np.asarray(x, np.int64)
        return np.where(x < mid, x, x + GIANTS)

    deg_s = np.diff(off_s).astype(np.int64)
    span_r = n_s + GIANTS + 1
    # the expected graph: the small one with remapped ids (giant rows empty)
    deg_r = np.zeros(span_r, np.int64)
    deg_r[remap(np.arange(n_s + 1))] = deg_s
    off_r = np.zeros(span_r + 1, np.uint64)
    off_r[1:] = np.cumsum(deg_r)
    keys_r = remap(keys_s).astype(np.uint32)  # rows stay in id order: remap is monotone
    # the big graph: + giants (ids mid .. mid + GIANTS - 1) and sinks (ids after everything)
    L = TOTAL // GIANTS + 1
    sink0 = span_r
    span = span_r + SINKS
    deg = torch.zeros(span, dtype=torch.int64, device="cuda")
    deg[:span_r] = torch.from_numpy(deg_r).cuda()
    deg[mid:mid + GIANTS] = L
    off = torch.zeros(span + 1, dtype=torch.int64, device="cuda")
    off[1:] = torch.cumsum(deg, 0)
    M = int(off[-1])
    assert M > (1 << 32)
    keys = torch.empty(M, dtype=torch.int32, device="cuda")
    # small rows: their entries at the new offsets
    rows_r = np.repeat(np.arange(span_r), deg_r)
    pos = off[torch.from_numpy(rows_r).cuda()] + torch.from_numpy(
        np.arange(len(keys_r)) - off_r[rows_r].astype(np.int64)).cuda()
    keys[pos] = torch.from_numpy(keys_r.view(np.int32)).cuda()
    # giant rows: sorted sink ids with duplicates
    for gi in range(GIANTS):
        base = int(off[mid + gi])
        for c in range(0, L, 1 << 28):
            e = min(L, c + (1 << 28))
            j = torch.arange(c, e, dtype=torch.int64, device="cuda")
            keys[base + c:base + e] = (sink0 + j * SINKS // L).to(torch.int32)
    torch.cuda.synchronize()
    G = nlp.Graph.from_device(off, keys)
    del keys, pos
    torch.cuda.empty_cache()
    yield dict(G=G, off_r=off_r, keys_r=keys_r, span=span, M=M, mid=mid)
    G.close()
    torch.cuda.empty_cache()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("metric,H", [(1, 4), (0, 0), (7, 4), (1, 16), (8, 2)])
def test_gpu_offsets_beyond_2e32(big, nlp, oracle, metric, H):
    import torch
    G = big["G"]
    info = G.info()
    assert info["nnz"] == big["M"] > (1 << 32) and info["span"] == big["span"]
    k = 4000
    out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
    n, t = G.predict_device(metric, H, k, out)
    u, w, s = nlp.edges_from_tensor(out, n)
    eu, ew, es, oi = oracle.predict(big["off_r"], big["keys_r"], metric, H, max_edges=k)
    assert_canonical_equal(eu, ew, es, u, w, s)
    assert_canonical_order(u, w, s)
    assert t["candidates"] == oi["candidates"] and t["wedges"] == oi["wedges_gt"]
    # the sources whose rows lie beyond the 2^32 offset, as a range of their own
    ua = big["mid"] + 64
    n, t = G.predict_device(metric, H, k, out, ua, big["span"])
    u, w, s = nlp.edges_from_tensor(out, n)
    eu, ew, es, oi = oracle.predict(big["off_r"], big["keys_r"], metric, H, max_edges=k, u_begin=ua)
    assert n > 0 and np.all(u >= ua)
    assert_canonical_equal(eu, ew, es, u, w, s)
    assert t["candidates"] == oi["candidates"] and t["wedges"] == oi["wedges_gt"]
