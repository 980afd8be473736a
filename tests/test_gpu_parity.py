"""GPU parity: libnlp (HIP, gfx950) through the C-ABI against the reference's
golden outputs and the pinned C oracle.  Bit-exact for every metric (scores
compared as bit patterns, NaN by NaN-ness); ties per the canonical rule.

All tests run in one process on cuda:0."""
import os

import numpy as np
import pytest

from bigconf import ORACLE_THREADS
from parity import (assert_canonical_equal, assert_canonical_order, assert_same_candidates,
                    assert_topk_matches_reference, f1_score)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(nlp):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return nlp


def golden_cases(g):
    out = []
    for key in g:
        if key.startswith("topk_") and key.endswith("_u"):
            _, m, H, _ = key.split("_")
            out.append((int(m), int(H)))
    return sorted(out)


@pytest.mark.parametrize("name", ["g300", "g3k", "edge"])
def test_gpu_all_candidates_match_reference(gpu, golden, name):
    g = golden[name]
    with gpu.Graph(g["offsets"], g["keys"]) as G:
        n = 0
        for m, H in golden_cases(g):
            if "cand_%d_%d_u" % (m, H) not in g:
                continue
            u, w, s, t = G.predict(m, H, None)
            assert_same_candidates(g["cand_%d_%d_u" % (m, H)], g["cand_%d_%d_w" % (m, H)],
                                   g["cand_%d_%d_s" % (m, H)], u, w, s)
            assert_canonical_order(u, w, s)
            n += 1
        assert n >= 9


@pytest.mark.parametrize("name", ["g300", "g3k", "edge"])
def test_gpu_topk_matches_reference_and_oracle(gpu, golden, oracle, name):
    g = golden[name]
    k = int(g["k"][0])
    with gpu.Graph(g["offsets"], g["keys"]) as G:
        for m, H in golden_cases(g):
            u, w, s, t = G.predict(m, H, k)
            eu, ew, es, info = oracle.predict(g["offsets"], g["keys"], m, H, max_edges=k)
            assert_canonical_equal(eu, ew, es, u, w, s)
            assert t["candidates"] == info["candidates"]
            assert t["nan_candidates"] == info["nan"]
            cand = None
            if "cand_%d_%d_u" % (m, H) in g:
                cand = (g["cand_%d_%d_u" % (m, H)], g["cand_%d_%d_w" % (m, H)], g["cand_%d_%d_s" % (m, H)])
                if np.isnan(cand[2]).any():
                    continue  # reference order undefined with NaN
            assert_topk_matches_reference(g["topk_%d_%d_u" % (m, H)], g["topk_%d_%d_w" % (m, H)],
                                          g["topk_%d_%d_s" % (m, H)], u, w, s, cand)


def random_csr(n, avg, seed, dup_frac=0.02, asym_frac=0.02, alpha=0.7):
    """Power-law multigraph with duplicate entries and some asymmetric edges."""
    rng = np.random.default_rng(seed)
    m = n * avg // 2
    p = np.arange(1, n + 1, dtype=np.float64) ** (-alpha)
    p /= p.sum()
    a = rng.choice(np.arange(1, n + 1), size=m, p=p)
    b = rng.choice(np.arange(1, n + 1), size=m, p=p)
    ok = a != b
    a, b = a[ok], b[ok]
    src = np.concatenate([a, b])
    dst = np.concatenate([b, a])
    # drop some reverse directions (asymmetry) and duplicate some entries
    keep = rng.random(len(src)) >= asym_frac
    src, dst = src[keep], dst[keep]
    d = rng.random(len(src)) < dup_frac
    src = np.concatenate([src, src[d]])
    dst = np.concatenate([dst, dst[d]])
    order = np.lexsort((dst, src))
    src, dst = src[order], dst[order]
    span = n + 1
    off = np.zeros(span + 1, np.uint64)
    np.add.at(off, src + 1, 1)
    off = np.cumsum(off).astype(np.uint64)
    return off, dst.astype(np.uint32)


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_random_multigraphs_vs_oracle(gpu, oracle, seed):
    off, keys = random_csr(4000 if seed == 1 else 20000, 12, seed)
    with gpu.Graph(off, keys) as G:
        assert not G.info()["symmetric"]
        for m in range(9):
            for H in (0, 1, 3, 4, 16) if seed == 1 else (2, 4, 8):
                for k in (50, 5000):
                    u, w, s, t = G.predict(m, H, k)
                    eu, ew, es, info = oracle.predict(off, keys, m, H, max_edges=k)
                    assert_canonical_equal(eu, ew, es, u, w, s)
                    assert t["wedges"] == info["wedges_gt"]


def _csr_from_pairs(src, dst, span):
    order = np.lexsort((dst, src))
    src, dst = src[order], dst[order]
    off = np.zeros(span + 1, np.uint64)
    np.add.at(off, src + 1, 1)
    return np.cumsum(off).astype(np.uint64), dst.astype(np.uint32)


def _is_symmetric(off, keys):
    src = np.repeat(np.arange(len(off) - 1), np.diff(off).astype(np.int64))
    a = np.lexsort((keys, src))
    b = np.lexsort((src, keys))
    return bool(np.array_equal(src[a], keys[b]) and np.array_equal(keys[a], src[b]))


def test_gpu_symmetry_flag_and_transpose(gpu, oracle):
    """The graph's symmetric flag (the transposed sort compared with the CSR,
    nlp.hip finish_graph) against a numpy transpose, and predictions on each
    graph against the oracle: simple symmetric graphs with and without self
    loops, one missing mirror on each side of the diagonal (equal counts above
    and below it), a one-sided extra edge, a symmetric multigraph, a duplicate
    in one direction only, and extra copies around a triangle (in-degrees equal
    out-degrees, supports mirror images, multiplicities not).  (A table-based
    test that skipped the sort for symmetric inputs was tried in round 6: the
    bench's batch graph is asymmetric -- the reference's deletions leave 154
    one-sided pairs on C4 -- so it cost 114 ms there and saved nothing.)"""
    rng = np.random.default_rng(5)
    n = 3000
    a = rng.integers(0, n, 20000)
    b = rng.integers(0, n, 20000)
    ok = a != b
    pairs = np.unique(np.stack([np.minimum(a[ok], b[ok]), np.maximum(a[ok], b[ok])], 1), axis=0)
    lo, hi = pairs[:, 0], pairs[:, 1]
    cases = {}
    cases["simple"] = (np.concatenate([lo, hi]), np.concatenate([hi, lo]))
    loops = np.arange(0, n, 7)
    cases["loops"] = (np.concatenate([lo, hi, loops]), np.concatenate([hi, lo, loops]))
    # drop (lo0 -> hi0) above the diagonal and (hi1 -> lo1) below it
    s, d = cases["simple"]
    drop = np.zeros(len(s), bool)
    drop[0] = True
    drop[len(lo) + 1] = True
    cases["two_missing_mirrors"] = (s[~drop], d[~drop])
    cases["one_sided"] = (np.concatenate([s, [5]]), np.concatenate([d, [n - 1]]))
    dup = rng.random(len(lo)) < 0.05
    cases["symmetric_multigraph"] = (np.concatenate([lo, hi, lo[dup], hi[dup]]),
                                     np.concatenate([hi, lo, hi[dup], lo[dup]]))
    # a duplicate in one direction only
    cases["unequal_multiplicity"] = (np.concatenate([s, [lo[3]]]), np.concatenate([d, [hi[3]]]))
    # one extra copy around a triangle: every in-degree still equals its out-degree
    t3 = np.array([n - 3, n - 2, n - 1])
    ts, td = np.concatenate([t3, np.roll(t3, 1)]), np.concatenate([np.roll(t3, 1), t3])
    cases["triangle_extra_copies"] = (np.concatenate([s, ts, t3]), np.concatenate([d, td, np.roll(t3, -1)]))
    for name, (src, dst) in cases.items():
        off, keys = _csr_from_pairs(src.astype(np.int64), dst.astype(np.int64), n)
        want = _is_symmetric(off, keys)
        assert want == (name in ("simple", "loops", "symmetric_multigraph")), name
        if name == "triangle_extra_copies":
            deg = np.diff(off).astype(np.int64)
            assert np.array_equal(deg, np.bincount(keys, minlength=len(deg)))
        with gpu.Graph(off, keys) as G:
            assert G.info()["symmetric"] == want, name
            for m, H in ((0, 0), (1, 4), (4, 0)):
                u, w, sc, t = G.predict(m, H, 500)
                eu, ew, es, info = oracle.predict(off, keys, m, H, max_edges=500)
                assert_canonical_equal(eu, ew, es, u, w, sc)


def test_gpu_path2_chunking_equals_path1(gpu, oracle):
    """Force tiny wedge budgets: path 1 falls back to path 2, which then runs
    in many source-range chunks with candidate pruning in between."""
    off, keys = random_csr(5000, 10, 3)
    try:
        os.environ["NLP_WEDGE_BUDGET"] = "2000"
        with gpu.Graph(off, keys) as G:
            for m, H, k in ((1, 4, 300), (7, 4, 300), (0, 0, 1000), (8, 0, 100), (3, 8, 10 ** 6)):
                u, w, s, t = G.predict(m, H, k)
                assert t["path"] == 2 and t["chunks"] > 1
                eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
                assert_canonical_equal(eu, ew, es, u, w, s)
    finally:
        del os.environ["NLP_WEDGE_BUDGET"]


def test_gpu_shard_ranges_and_merge(gpu, oracle):
    """Per-range device predictions + the device merge == the single-range result
    (the multi-GPU exchange step, run on one GPU)."""
    import torch
    off, keys = random_csr(8000, 14, 4)
    span = len(off) - 1
    k = 3000
    with gpu.Graph(off, keys) as G:
        for m, H in ((1, 4), (7, 8), (0, 0)):
            parts = []
            for r in range(4):
                out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
                n, _ = G.predict_device(m, H, k, out, span * r // 4, span * (r + 1) // 4)
                parts.append(out[:n])
            allv = torch.cat(parts)
            res = torch.empty((k, 3), dtype=torch.int32, device="cuda")
            kk = G.select_edges_device(allv, allv.shape[0], k, res)
            u, w, s = gpu.edges_from_tensor(res, kk)
            eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
            assert_canonical_equal(eu, ew, es, u, w, s)
            # the all_gather layout: fixed-stride blocks with count headers (nlp_merge_blocks_device),
            # at k and at smaller k (truncation inside the tie runs)
            stride = max(p.shape[0] for p in parts) + 7
            blocks = _blocks(parts, stride)
            for kk_ in (k, 777, 1):
                res = torch.empty((k, 3), dtype=torch.int32, device="cuda")
                kk = G.merge_blocks_device(blocks, kk_, res)
                u, w, s = gpu.edges_from_tensor(res, kk)
                eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=kk_)
                assert_canonical_equal(eu, ew, es, u, w, s)
            # a block beyond its stride: NLP_ERR_CAPACITY with the largest count
            small = _blocks(parts, stride)[:, : stride // 2].contiguous()
            with pytest.raises(gpu.NlpError) as ei:
                G.merge_blocks_device(small, k, res)
            assert ei.value.status == 5 and ei.value.count == max(p.shape[0] for p in parts)


def _blocks(parts, stride):
    """[len(parts), stride, 3] int32 device blocks, entry 0 = {count lo, count hi, NLP_BLOCK_MAGIC}."""
    import torch
    b = torch.zeros((len(parts), stride, 3), dtype=torch.int32, device="cuda")
    for r, p in enumerate(parts):
        n = p.shape[0]
        b[r, 0] = torch.from_numpy(np.array([n & 0xFFFFFFFF, n >> 32, 0x4E4C5042], np.uint32).view(np.int32))
        b[r, 1:1 + n] = p
    return b


def test_gpu_edge_cases(gpu, oracle):
    # empty graph (only vertex 0), a graph without edges, max_edges = 0
    with gpu.Graph(np.zeros(2, np.uint64), np.zeros(0, np.uint32)) as G:
        u, w, s, t = G.predict(0, 0, 10)
        assert len(u) == 0
    off = np.zeros(11, np.uint64)
    with gpu.Graph(off, np.zeros(0, np.uint32)) as G:
        assert len(G.predict(1, 4, 10)[0]) == 0
    off, keys = random_csr(500, 6, 5)
    with gpu.Graph(off, keys) as G:
        assert len(G.predict(1, 4, 0)[0]) == 0
        # min_score filter (PredictLinkOptions::minScore, predict.hxx:311)
        u, w, s, _ = G.predict(1, 0, 1000, min_score=0.25)
        eu, ew, es, _ = oracle.predict(off, keys, 1, 0, max_edges=1000, min_score=0.25)
        assert_canonical_equal(eu, ew, es, u, w, s)
        assert (s > 0.25).all()


def test_gpu_invalid_inputs(gpu):
    with pytest.raises(gpu.NlpError) as e:
        gpu.Graph(np.array([0, 1, 2], np.uint64), np.array([1, 5], np.uint32))  # key >= span
    assert e.value.status == 1
    with pytest.raises(gpu.NlpError):
        gpu.Graph(np.array([0, 2, 3], np.uint64), np.array([1, 0, 0], np.uint32))  # unsorted row
    with pytest.raises(gpu.NlpError):
        gpu.Graph(np.array([0, 2, 1], np.uint64), np.array([1, 0], np.uint32))  # offsets decrease
    # descents at row starts are legal, one inside a row is not (the build counts both kinds)
    with gpu.Graph(np.array([0, 2, 4, 5], np.uint64), np.array([1, 2, 0, 2, 1], np.uint32)) as G:
        assert G.info()["nnz"] == 5
    with pytest.raises(gpu.NlpError):
        gpu.Graph(np.array([0, 2, 4, 5], np.uint64), np.array([1, 2, 2, 0, 1], np.uint32))


def test_gpu_reference_api_names(gpu, golden):
    g = golden["g3k"]
    k = int(g["k"][0])
    with gpu.Graph(g["offsets"], g["keys"]) as G:
        r = gpu.predictLinksJaccardCoefficientHip(G, gpu.PredictLinkOptions(1, k), mindegree1=4)
        assert len(r.edges) == len(g["topk_1_4_u"])
        assert r.time >= r.scoringTime >= 0
        p, rr, f = f1_score([e[0] for e in r.edges], [e[1] for e in r.edges], g["del_u"], g["del_w"])
        assert 0 <= f <= 1


def test_gpu_full_size_c2_vs_oracle(gpu, oracle, nlp):
    """BASELINE configs[1] stand-in (soc-LiveJournal1 shape, 125M entries):
    exact canonical equality with the oracle for the bench metric (LHub-4
    Jaccard) and Adamic-Adar, plus size-independent properties."""
    import torch
    import nlp_loader
    gg = nlp_loader.load_sub("graphgen")
    off_t, keys_t, du, dw, info = gg.make_workload("C2-soc-LiveJournal1", "cuda")
    with gpu.Graph.from_device(off_t, keys_t) as G:
        off = off_t.cpu().numpy().astype(np.uint64)
        keys = keys_t.cpu().numpy().view(np.uint32)
        k = info["k"]
        out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
        for m in (1, 7):
            n, t = G.predict_device(m, 4, k, out)
            u, w, s = gpu.edges_from_tensor(out, n)
            eu, ew, es, oi = oracle.predict(off, keys, m, 4, max_edges=k)
            assert_canonical_equal(eu, ew, es, u, w, s)
            assert t["wedges"] == oi["wedges_gt"] and t["candidates"] == oi["candidates"]
            assert_canonical_order(u, w, s)
            # idempotence: a second call gives the identical result
            n2, _ = G.predict_device(m, 4, k, out)
            assert n2 == n
            u2, w2, s2 = gpu.edges_from_tensor(out, n2)
            assert np.array_equal(u, u2) and np.array_equal(w, w2)


def star_csr(leaves=12000):
    """Hub 1 joined to `leaves` vertices of degree 2 (each also joined to its own
    private vertex): vertex 1's bucket holds > 8192 wedges (LDS bucket cap)."""
    n = 1 + 2 * leaves
    rows = {1: list(range(2, 2 + leaves))}
    for i in range(leaves):
        a, b = 2 + i, 2 + leaves + i
        rows.setdefault(a, []).extend([1, b])
        rows.setdefault(b, []).append(a)
    off = [0]
    keys = []
    for u in range(n + 1):
        keys += sorted(rows.get(u, []))
        off.append(len(keys))
    return np.array(off, np.uint64), np.array(keys, np.uint32)


@pytest.mark.parametrize("grouping", ["sort", "lsd", "bucket"])
def test_gpu_oversized_bucket_falls_back(gpu, oracle, grouping):
    """A source with a huge wedge bucket: the sort grouping has no size limit
    (path 1); the bucket grouping exceeds its LDS cap and falls back (path 3)."""
    off, keys = star_csr()
    try:
        os.environ["NLP_GROUPING"] = grouping
        with gpu.Graph(off, keys) as G:
            for m, H, k in ((0, 2, 500), (7, 4, 20000), (1, 2, 10 ** 6)):
                u, w, s, t = G.predict(m, H, k)
                eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
                assert_canonical_equal(eu, ew, es, u, w, s)
                assert t["path"] == (3 if grouping == "bucket" else 1)
    finally:
        del os.environ["NLP_GROUPING"]


_GROUPING_DEFAULT = {}


@pytest.mark.parametrize("other", ["bucket", "lsd", "fused"])
def test_gpu_sort_grouping_equals_bucket_grouping(gpu, oracle, other):
    """The sync-free groupings (wedge records: MSD buckets / full LSD sort;
    per-source buckets) give identical results and counters, IHub included
    (sort groupings only)."""
    off, keys = random_csr(8000, 14, 7)
    k = 3000
    if "res" not in _GROUPING_DEFAULT:  # the default grouping's results, shared by the parametrisations
        with gpu.Graph(off, keys) as Gs:
            _GROUPING_DEFAULT["res"] = {(m, H): Gs.predict(m, H, k) for m in (0, 1, 3, 7, 8) for H in (0, 1, 4, 16)}
    res = _GROUPING_DEFAULT["res"]
    env = ("NLP_BUCKET_FUSED", "1") if other == "fused" else ("NLP_GROUPING", other)
    try:
        os.environ[env[0]] = env[1]
        with gpu.Graph(off, keys) as Gb:
            for (m, H), (u, w, s, t) in res.items():
                assert t["path"] == 1
                ub, wb, sb, tb = Gb.predict(m, H, k)
                assert_canonical_equal(ub, wb, sb, u, w, s)
                assert t["wedges"] == tb["wedges"] and t["candidates"] == tb["candidates"]
                assert t["nan_candidates"] == tb["nan_candidates"]
    finally:
        del os.environ[env[0]]


def test_gpu_radix_path_equals_bucket_path(gpu, oracle):
    off, keys = random_csr(6000, 16, 6)
    k = 4000
    with gpu.Graph(off, keys) as G1:
        res1 = {(m, H): G1.predict(m, H, k) for m in range(9) for H in (1, 4, 32)}
    try:
        os.environ["NLP_FORCE_RADIX"] = "1"
        with gpu.Graph(off, keys) as G3:
            for (m, H), (u, w, s, t) in res1.items():
                u3, w3, s3, t3 = G3.predict(m, H, k)
                assert t["path"] in (1, 3) and t3["path"] == 3  # 3 also when a bucket exceeds the LDS cap
                assert_canonical_equal(u3, w3, s3, u, w, s)
                assert t["wedges"] == t3["wedges"] and t["candidates"] == t3["candidates"]
    finally:
        del os.environ["NLP_FORCE_RADIX"]


def test_gpu_cpp_dropin_header(gpu, golden, oracle, tmp_path):
    """main.cxx-style C++ caller of include/nlp/predict.hxx (tests/cpp/predict_main.cxx):
    the reference's template names on a graph-concept type and on a resident
    nlp::HipGraph agree, and equal the oracle for all nine metrics."""
    import subprocess
    from nlp_amd import build as b
    exe = b.build_cpp_test(verbose=False)
    g = golden["g3k"]
    k = int(g["k"][0])
    csr = str(tmp_path / "g.csr")
    oracle.write_csr(csr, g["offsets"], g["keys"])
    for H in (0, 4, 8):
        pre = str(tmp_path / ("out%d" % H))
        subprocess.run([exe, csr, str(H), str(k), pre], check=True, timeout=300)
        for m in range(9):
            u, w, s = oracle.read_edges(pre + "." + str(m))
            eu, ew, es, _ = oracle.predict(g["offsets"], g["keys"], m, H, max_edges=k)
            assert_canonical_equal(eu, ew, es, u, w, s)


def test_gpu_graph_replay_equals_direct_launch(gpu, oracle):
    """The sync-free path is captured once per (metric, H, k, range, buffers)
    and replayed as hipGraphs; replays must equal the directly launched run and
    the oracle, across interleaved cache entries and a capacity regrow.
    (Synchronous stamp-timed calls launch kernel by kernel by default;
    NLP_DIRECT_LAUNCH=0 selects the single replayed graph.)"""
    off, keys = random_csr(6000, 14, 5)
    runs = [(1, 4, 400), (7, 4, 400), (1, 4, 400), (0, 8, 50), (7, 4, 400), (1, 4, 400)]
    with gpu.Graph(off, keys) as G:  # default: direct launches
        for m, H, k in runs[:3]:
            u, w, s, t = G.predict(m, H, k)
            eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
            assert_canonical_equal(eu, ew, es, u, w, s)
    with _env(NLP_DIRECT_LAUNCH="0"), gpu.Graph(off, keys) as G:
        seen = {}
        for m, H, k in runs:
            u, w, s, t = G.predict(m, H, k)
            eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
            assert_canonical_equal(eu, ew, es, u, w, s)
            if t["path"] == 1 and (m, H, k) in seen:
                assert t["graph_replay"] == 1
            seen[(m, H, k)] = True
            assert t["hot_ms"] > 0 and t["hot_bytes"] > 0
    with _env(NLP_DIRECT_LAUNCH="1"), gpu.Graph(off, keys) as G:  # no graphs at all
        for m, H, k in runs[:3]:
            u, w, s, t = G.predict(m, H, k)
            assert t["graph_replay"] == 0
            eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
            assert_canonical_equal(eu, ew, es, u, w, s)


def test_gpu_degree_index_equals_survivor_scan(gpu, oracle):
    """Count metrics take their survivors from the degree-class index (any
    order within a degree); the result must equal the ordered survivor scan and
    the oracle, including thresholds at and above the index cap."""
    off, keys = random_csr(7000, 12, 11)
    cases = [(m, H) for m in (0, 1, 2, 3, 4, 5, 6) for H in (1, 2, 4, 9, 1024, 2000)]
    with gpu.Graph(off, keys) as G:
        res = {c: G.predict(c[0], c[1], 2500) for c in cases}
    try:
        os.environ["NLP_NO_DINDEX"] = "1"
        with gpu.Graph(off, keys) as G2:
            for (m, H), (u, w, s, t) in res.items():
                u2, w2, s2, t2 = G2.predict(m, H, 2500)
                assert_canonical_equal(u2, w2, s2, u, w, s)
                assert t["wedges"] == t2["wedges"] and t["candidates"] == t2["candidates"]
    finally:
        del os.environ["NLP_NO_DINDEX"]
    for (m, H), (u, w, s, t) in list(res.items())[::5]:
        eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=2500)
        assert_canonical_equal(eu, ew, es, u, w, s)


class _env:
    """Set environment variables for the graphs created inside the block (the
    library reads its switches at graph creation)."""

    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


# Path-4 variants against the oracle (round 5: cut to the defaults plus the
# fallbacks that trigger on real inputs): 0 the defaults (on `edge`: the
# round-4 emission-window hang case), 1-3 rows forced into bins 1 / 2 / 3 (bin
# 3 with a tiny k_hp_part scratch and no hub pass), 4 no row batches (graphs
# with ids beyond 2^26), 5 bins 2-3 by k_hp_part (a chunk beyond the hub
# scratch), 6 hub pass with 128-entry item tables and no direct counters
# (heavy buckets split by their segment histograms), 7 bin-1 rows by the hub
# pass, 8 AA / RA hub items by the ordered re-walk, 9 / 10 sort-mode items of
# at most 16 / 40 wedges (heavy buckets split, single bins beyond flagged
# HH_BIG), 11-14 the per-graph tables a full HBM leaves out (degree classes,
# entry degrees, rank bytes, exclusion starts), 15 one w-bucket rows with
# 64-wide direct counters (HH_WIDE sub-ranges), 16 bin-1 rows by k_hp_block,
# 17 every bin-1 row in the 8192-entry tier, 18 every row's exclusion by the
# membership table, 19 every row's by marks (no table), 20 the count metrics'
# survivor lists compacted per call (k_dc_*, the AA / RA route), 21 short lists
# of the classes up to 3 only, 22 / 23 the final order over rank-compressed
# 8-byte keys on every call (by default from ES8_MIN links on), 24 its
# two-level form on every call with runs beyond 2 keys by k_es_long and beyond
# 8 by the very-long sort
HASH_VARIANTS = [dict(), dict(NLP_HASH_MINBIN="1"), dict(NLP_HASH_MINBIN="2"),
                 dict(NLP_HASH_MINBIN="3", NLP_HASH_SCAP="300", NLP_HASH_HUB="0"),
                 dict(NLP_HASH_BATCH="0"), dict(NLP_HASH_MINBIN="2", NLP_HASH_HUB="0"),
                 dict(NLP_HASH_MINBIN="2", NLP_HASH_HUB_BW="1000000", NLP_HASH_HUB_TL="7", NLP_HH_DIRECT="0"),
                 dict(NLP_HASH_MINBIN="1", NLP_HASH_HUB_MIN="1"),
                 dict(NLP_HASH_MINBIN="2", NLP_HASH_HUB_SORT="0"),
                 dict(NLP_HASH_MINBIN="2", NLP_HASH_HUB_SCAP="16", NLP_HASH_HUB_TL="7"),
                 dict(NLP_HASH_MINBIN="2", NLP_HASH_HUB_SCAP="40", NLP_HASH_HUB_BW="1000000"),
                 dict(NLP_HASH_DCLS="0"), dict(NLP_HASH_KDEG="0"), dict(NLP_HASH_DRANK="0"), dict(NLP_HASH_XS="0"),
                 dict(NLP_HASH_MINBIN="2", NLP_HASH_HUB_BW="1000000", NLP_HASH_HUB_TL="7", NLP_HH_DIRECT="64"),
                 dict(NLP_HASH_MINBIN="1", NLP_HASH_ROWB="0"), dict(NLP_HASH_MINBIN="1", NLP_HASH_ROWB="2"),
                 dict(NLP_HASH_UX="0", NLP_HASH_MINBIN="1"), dict(NLP_HASH_UX="off"),
                 dict(NLP_HASH_SLIST="0"), dict(NLP_HASH_SLIST="3"),
                 dict(NLP_ES8="2"), dict(NLP_ES8="2", NLP_HASH_MINBIN="2"),
                 dict(NLP_ES8="2", NLP_ES_RUNS="2", NLP_ES_RS="2", NLP_ES_LCAP="8")]


@pytest.mark.parametrize("variant", range(len(HASH_VARIANTS)))
def test_gpu_hash_path_vs_oracle(gpu, oracle, golden, variant):
    """Path 4 against the oracle: every metric, IHub and LHub, top-k smaller and
    larger than the candidate count, tiny emission buffers (many chunks, pruning
    and the running threshold), multigraphs with duplicates and asymmetry."""
    graphs = [(golden["g3k"]["offsets"], golden["g3k"]["keys"]), (golden["edge"]["offsets"], golden["edge"]["keys"]),
              random_csr(3000, 12, 11)]
    with _env(NLP_HASH="1", NLP_HASH_EMIT="1", **HASH_VARIANTS[variant]):
        for off, keys in graphs:
            with gpu.Graph(off, keys) as G:
                for m in range(9):
                    for H in (0, 2, 4, 16):
                        for k in (40, 4000):
                            u, w, s, t = G.predict(m, H, k)
                            eu, ew, es, info = oracle.predict(off, keys, m, H, max_edges=k)
                            assert t["path"] == 4
                            assert_canonical_equal(eu, ew, es, u, w, s)
                            assert t["wedges"] == info["wedges_gt"]
                            assert t["candidates"] == info["candidates"] and t["nan_candidates"] == info["nan"]


def test_gpu_short_list_prefixes_up_to_class_254(gpu, oracle):
    """The count metrics' S(u) as prefixes of the class-ordered short lists:
    rows of hundreds of short entries of mixed classes (the sort's histogram
    path), H at the classes' ends (1, 254) and just beyond them (255: per-call
    lists), every chunk of a tiny emission buffer, a source range."""
    off, keys = random_csr(3000, 60, 21)
    with _env(NLP_HASH="1", NLP_HASH_EMIT="1"):
        with gpu.Graph(off, keys) as G:
            for m in (0, 1, 4, 8):
                for H in (1, 7, 64, 254, 255):
                    u, w, s, t = G.predict(m, H, 3000)
                    eu, ew, es, info = oracle.predict(off, keys, m, H, max_edges=3000)
                    assert t["path"] == 4
                    assert_canonical_equal(eu, ew, es, u, w, s)
                    assert t["wedges"] == info["wedges_gt"] and t["candidates"] == info["candidates"]


def test_gpu_hash_path_all_candidates_and_min_score(gpu, golden, oracle):
    """maxEdges = all (no pruning) and minScore < 0 (excluded first-order pairs
    with score 0 become candidates, predict.hxx:306-311)."""
    with _env(NLP_HASH="1"):
        for name in ("g300", "edge"):  # every reference candidate list of these fixtures
            g = golden[name]
            with gpu.Graph(g["offsets"], g["keys"]) as G:
                for key in g:
                    if key.startswith("cand_") and key.endswith("_u"):
                        _, m, H, _ = key.split("_")
                        u, w, s, t = G.predict(int(m), int(H), None)
                        assert t["path"] == 4 or len(u) == 0  # no candidates: the fetch call has maxEdges 0
                        assert_same_candidates(g[key], g["cand_%s_%s_w" % (m, H)], g["cand_%s_%s_s" % (m, H)], u, w, s)
        g = golden["g3k"]
        with gpu.Graph(g["offsets"], g["keys"]) as G:
            for m in (0, 1, 7, 8):
                for H in (0, 4):
                    u, w, s, t = G.predict(m, H, 5000, min_score=-1.0)
                    eu, ew, es, _ = oracle.predict(g["offsets"], g["keys"], m, H, max_edges=5000, min_score=-1.0)
                    assert_canonical_equal(eu, ew, es, u, w, s)


def test_gpu_hash_path_star_hub(gpu, oracle):
    """A hub source whose row holds > 10^4 distinct second hops (bins 2 and 3)."""
    off, keys = star_csr(20000)
    for v in (dict(), dict(NLP_HASH_SCAP="5000"), dict(NLP_HASH_HUB="0"), dict(NLP_HASH_HUB="0", NLP_HASH_SCAP="5000")):
        with _env(NLP_HASH="1", **v):
            with gpu.Graph(off, keys) as G:
                for m, H, k in ((0, 0, 500), (7, 0, 30000), (1, 2, 10 ** 6), (8, 4, 100)):
                    u, w, s, t = G.predict(m, H, k)
                    eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
                    assert t["path"] == 4
                    assert_canonical_equal(eu, ew, es, u, w, s)


def test_gpu_short_lists_of_hub_rows(gpu, oracle):
    """Hub rows whose class-ordered short lists are long (>= 4096 entries: a
    workgroup per row, k_sl_sort_long) with mixed classes, beside short rows:
    the count metrics' prefixes S(u) for several H against the oracle."""
    L = 9000
    leaves = np.arange(L)
    src, dst = [], []
    for hub in (0, 1):
        src.append(np.full(L, hub)); dst.append(2 + leaves)
    for j in range(1, 30):
        sel = leaves[(leaves % 30) >= j]
        src.append(2 + sel); dst.append(2 + (sel + j) % L)
    a = np.concatenate(src).astype(np.int64)
    b = np.concatenate(dst).astype(np.int64)
    pairs = np.unique(np.stack([np.minimum(a, b), np.maximum(a, b)], 1), axis=0)
    pairs = pairs[pairs[:, 0] != pairs[:, 1]]
    off, keys = _csr_from_pairs(np.concatenate([pairs[:, 0], pairs[:, 1]]),
                                np.concatenate([pairs[:, 1], pairs[:, 0]]), L + 2)
    deg = np.diff(off).astype(np.int64)
    assert deg[0] == L and deg[1] == L and len(np.unique(np.minimum(deg[keys[off[0]:off[1]]], 255))) > 10
    with _env(NLP_HASH="1"):
        with gpu.Graph(off, keys) as G:
            for m in (0, 1, 4, 6):
                for H in (4, 16, 64):
                    u, w, sc, t = G.predict(m, H, 20000)
                    eu, ew, es, info = oracle.predict(off, keys, m, H, max_edges=20000)
                    assert t["path"] == 4
                    assert_canonical_equal(eu, ew, es, u, w, sc)
                    assert t["wedges"] == info["wedges_gt"]


def test_gpu_aa_ra_tables_beyond_the_dense_degrees(gpu, oracle):
    """Adamic-Adar / Resource-Allocation through an intermediate of degree
    70,001 (> 65,536: its contribution computed for the degrees present only,
    nlp.hip finish_graph): IHub over a source range of leaves, every wedge via
    the hub, against the oracle on the same range."""
    import torch
    L = 70000
    leaves = np.arange(2, 2 + L, dtype=np.int64)
    a = np.concatenate([np.ones(L, np.int64), leaves[:-1]])
    b = np.concatenate([leaves, leaves[1:]])
    off, keys = _csr_from_pairs(np.concatenate([a, b]), np.concatenate([b, a]), L + 2)
    assert np.diff(off)[1] == L
    k = 3000
    out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
    with gpu.Graph(off, keys) as G:
        for m in (7, 8):
            for H in (0, 100000):
                n, t = G.predict_device(m, H, k, out, 2, 12)
                u, w, sc = gpu.edges_from_tensor(out, n)
                eu, ew, es, info = oracle.predict(off, keys, m, H, max_edges=k, u_begin=2, u_end=12)
                assert n > 0
                assert_canonical_equal(eu, ew, es, u, w, sc)
                assert t["wedges"] == info["wedges_gt"]


def test_gpu_final_prune_folded_into_order(gpu, oracle):
    """The call's last prune folded into the 8-byte order (hp_prune fuse: the
    keys >= the k-th sorted straight from the unpruned buffer, the first k
    written -- the canonical tie rule is the sort order): Jaccard with few
    ties takes it (nlp_timing.order_route = NLP_ORDER_FOLD8), Adamic-Adar is
    never offered the fold (nearly every score distinct: pruned, then
    ordered), Common Neighbours (a tie set far beyond k) falls back to the
    split; every result exact against the oracle, one and several chunks."""
    off, keys = random_csr(20000, 16, 41)
    routes = {}
    for env in (dict(), dict(NLP_HASH_EMIT="300000")):
        with _env(NLP_HASH="1", **env):
            with gpu.Graph(off, keys) as G:
                for m in (1, 7, 0, 3):
                    for H in (0, 16):
                        for k in (70000, 250000):
                            u, w, s, t = G.predict(m, H, k)
                            assert t["path"] == 4
                            routes.setdefault(m, set()).add(t["order_route"] & 15)  # 16: the two-level form
                            eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
                            assert_canonical_equal(eu, ew, es, u, w, s)
    assert 1 in routes[1], routes                 # Jaccard: the fold
    assert not routes[7] & {1, 2}, routes         # Adamic-Adar: never folded
    assert all(r in (1, 2, 3, 4) for rs in routes.values() for r in rs), routes


def test_gpu_two_level_order(gpu, oracle):
    """The 8-byte order's two-level form (edgesort.hpp k_es_runs): LSD passes
    over (rank, u) only, then every run of equal (rank, u) put in w order in
    place -- runs ranked in their tile (up to NLP_ES_RS keys, across tile
    boundaries), sorted by a workgroup (k_es_long, up to NLP_ES_LCAP) and by
    the very-long gather + sort; Common Neighbours has long runs (few distinct
    counts), Jaccard short ones; several tiles of keys, the fold's first k of
    an unpruned buffer; exact against the oracle, route flagged."""
    off, keys = random_csr(20000, 16, 41)
    ran = 0
    for env in (dict(), dict(NLP_ES_RS="1", NLP_ES_LCAP="2"), dict(NLP_ES_RS="3", NLP_ES_LCAP="16"),
                dict(NLP_ES_LCAP="64", NLP_HASH_EMIT="300000"), dict(NLP_ES8_NT="256")):
        with _env(NLP_HASH="1", NLP_ES_RUNS="2", **env):
            with gpu.Graph(off, keys) as G:
                for m in (1, 0, 7, 2):
                    for H in (0, 16):
                        for k in (70000, 250000):
                            u, w, s, t = G.predict(m, H, k)
                            assert t["path"] == 4
                            if t["order_route"] & 15 in (1, 3):  # the 8-byte order ran
                                assert t["order_route"] & 16, t["order_route"]
                                ran += 1
                            eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
                            assert_canonical_equal(eu, ew, es, u, w, s)
    assert ran >= 16, ran


def test_gpu_hash_routing_and_shards(gpu, oracle):
    """Automatic routing by the wedge estimate, and per-shard path-4 results
    merged on the device equal the single-range result."""
    import torch
    off, keys = random_csr(8000, 16, 12)
    span = len(off) - 1
    k = 3000
    with _env(NLP_HASH_MIN_WEDGES="1000"):
        with gpu.Graph(off, keys) as G:
            for m, H in ((1, 16), (7, 0), (0, 32), (2, 0)):
                u, w, s, t = G.predict(m, H, k)
                assert t["path"] == 4  # AA / RA too (ordered accumulation, hub sort mode)
                eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
                assert_canonical_equal(eu, ew, es, u, w, s)
                parts = []
                for r in range(3):
                    out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
                    n, _ = G.predict_device(m, H, k, out, span * r // 3, span * (r + 1) // 3)
                    parts.append(out[:n])
                allv = torch.cat(parts)
                res = torch.empty((k, 3), dtype=torch.int32, device="cuda")
                kk = G.select_edges_device(allv, allv.shape[0], k, res)
                u2, w2, s2 = gpu.edges_from_tensor(res, kk)
                assert_canonical_equal(eu, ew, es, u2, w2, s2)
                kk = G.merge_blocks_device(_blocks(parts, k + 1), k, res)
                u2, w2, s2 = gpu.edges_from_tensor(res, kk)
                assert_canonical_equal(eu, ew, es, u2, w2, s2)


def test_gpu_full_size_c2_large_hub_threshold(gpu, oracle, nlp):
    """C2 stand-in at H = 16 (1.6e8 wedges) against the oracle: Jaccard and
    Adamic-Adar on path 4 (automatic routing), and Adamic-Adar on the sort path
    (NLP_HASH_AA=0: persistent scans over many tiles)."""
    import torch
    import nlp_loader
    gg = nlp_loader.load_sub("graphgen")
    off_t, keys_t, du, dw, info = gg.make_workload("C2-soc-LiveJournal1", "cuda")
    off = off_t.cpu().numpy().astype(np.uint64)
    keys = keys_t.cpu().numpy().view(np.uint32)
    k = info["k"]
    out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
    ref = {m: oracle.predict_par(off, keys, m, 16, max_edges=k, threads=ORACLE_THREADS) for m in (1, 7)}
    for env, cases in ((dict(), ((1, 4), (7, 4))), (dict(NLP_HASH_AA="0"), ((7, 1),))):
        with _env(**env):
            with gpu.Graph.from_device(off_t, keys_t) as G:
                for m, path in cases:
                    n, t = G.predict_device(m, 16, k, out)
                    assert t["path"] == path
                    u, w, s = gpu.edges_from_tensor(out, n)
                    eu, ew, es, oi = ref[m]
                    assert_canonical_equal(eu, ew, es, u, w, s)
                    assert t["wedges"] == oi["wedges_gt"] and t["candidates"] == oi["candidates"]


def test_gpu_device_evaluation_matches_host(gpu, golden):
    """N3: |insertions1 ∩ deletions0| on the device (nlp_last_common,
    nlp_count_common_device) equals main.cxx's host evaluation."""
    import torch
    g = golden["g3k"]
    k = int(g["k"][0])
    with gpu.Graph(g["offsets"], g["keys"]) as G:
        G.set_truth(g["del_u"], g["del_w"])
        for m, H in ((1, 4), (0, 0), (7, 8)):
            u, w, s, t = G.predict(m, H, k)
            ins = set(zip(u.tolist(), w.tolist())) | set(zip(w.tolist(), u.tolist()))
            dels = set(zip(g["del_u"].tolist(), g["del_w"].tolist()))
            assert G.last_common() == len(ins & dels)
            out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
            n, _ = G.predict_device(m, H, k, out)
            assert G.count_common_device(out, n) == len(ins & dels)
            assert G.last_common() == len(ins & dels)


def test_gpu_experiment_driver(gpu, golden, oracle, tmp_path):
    """N4: nlp_main (main.cxx flow: ingest, deletion batch, PREDICT_LINKS sweep,
    process.js log lines) on g300's MatrixMarket input with seed 42, d = 0.1 --
    the same graph and deletions as the fixture, so precision / recall must equal
    the oracle's top-k evaluated as main.cxx does."""
    import re
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_golden import chung_lu_mtx
    from parity import f1_score
    from nlp_amd import build as B
    binary = B.build_main(verbose=False)
    mtx = str(tmp_path / "g300.mtx")
    chung_lu_mtx(mtx, 300, 1200, 0.6, 1)
    env = dict(os.environ, NLP_SEED="42", BATCH_DELETIONS_BEGIN="0.1", BATCH_DELETIONS_END="0.1",
               NLP_METRICS="CN,JAC,AA,RA", NLP_HUBS="0,4,64")
    r = subprocess.run([binary, mtx, "0", "0"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    g = golden["g300"]
    k = int(g["k"][0])
    rx = re.compile(r"^\{\-(.+?)\/\+(.+?) batchf, (.+?) threads\} -> \{(.+?)ms, (.+?) scoring, (.+?) precision, "
                    r"(.+?) recall\} predictLinks(\w+)Hip(\d+)$")
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{-")]
    assert len(lines) == 4 * 3
    assert re.search(r"^order: \d+ size: \d+ \[directed\] \{\} \(removeSelfLoops\)$", r.stdout, re.M)
    names = {"CommonNeighbors": 0, "JaccardCoefficient": 1, "AdamicAdarCoefficient": 7, "ResourceAllocationScore": 8}
    for ln in lines:
        m = rx.match(ln)
        assert m, ln
        metric, H = names[m.group(8)], int(m.group(9))
        u, w, s, _ = oracle.predict(g["offsets"], g["keys"], metric, H, max_edges=k)
        p, rc, _ = f1_score(u, w, g["del_u"], g["del_w"])
        assert float(m.group(6)) == pytest.approx(p, rel=1e-3, abs=1e-12)
        assert float(m.group(7)) == pytest.approx(rc, rel=1e-3, abs=1e-12)


@pytest.mark.parametrize("passes", [1, 2])
def test_gpu_msd_passes_on_source_ranges(gpu, oracle, passes):
    """Sort path with 1 and 2 MSD passes forced, on sub-ranges whose record key
    is narrower than the full-range key (odd and even MSD shifts), vs the oracle."""
    import torch
    off, keys = random_csr(20000, 12, 21)
    span = len(off) - 1
    k = 50000
    with _env(NLP_MSD_PASSES=str(passes)):
        with gpu.Graph(off, keys) as G:
            bad = []
            for m, H in ((1, 4), (7, 4), (0, 8)):
                for ub, ue in ((0, span), (0, span // 2), (span // 3, span), (5, span // 2 + 7)):
                    out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
                    n, t = G.predict_device(m, H, k, out, ub, ue)
                    u, w, s = gpu.edges_from_tensor(out, n)
                    eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k, u_begin=ub, u_end=ue)
                    assert t["path"] == 1
                    try:
                        assert_canonical_equal(eu, ew, es, u, w, s)
                    except AssertionError as e:
                        bad.append((m, H, ub, ue, len(eu), int((eu != u).sum()) if len(eu) == len(u) else -1,
                                    str(e)[:40]))
            assert not bad, bad


def _maxf2_cases(f):
    out = []
    for key in f:
        if "_topk_" in key and key.endswith("_u"):
            name, _, F, m, H, _ = key.split("_")
            out.append((name, int(F), int(m), int(H)))
    return sorted(out)


def test_gpu_maxfactor2_matches_reference(gpu, golden, oracle):
    """MAXFACTOR2 (predict.hxx:221,295) through nlp_predict_ex: all candidates
    against the compiled reference (tests/golden/maxf2.npz), top-k against the
    reference (contract) and the oracle (exact)."""
    from conftest import load_golden
    f = load_golden("maxf2")
    graphs = {}
    try:
        for name, F, m, H in _maxf2_cases(f):
            g = golden[name]
            if name not in graphs:
                graphs[name] = gpu.Graph(g["offsets"], g["keys"])
            G = graphs[name]
            k = int(g["k"][0])
            tag = "%s_%%s_%d_%d_%d" % (name, F, m, H)
            cu, cw, cs = f[tag % "cand" + "_u"], f[tag % "cand" + "_w"], f[tag % "cand" + "_s"]
            u, w, s, t = G.predict(m, H, None, maxfactor2=F)
            assert_same_candidates(cu, cw, cs, u, w, s)
            u, w, s, t = G.predict(m, H, k, maxfactor2=F)
            eu, ew, es, _ = oracle.predict(g["offsets"], g["keys"], m, H, max_edges=k, maxfactor2=F)
            assert_canonical_equal(eu, ew, es, u, w, s)
            if not np.isnan(cs).any():
                assert_topk_matches_reference(f[tag % "topk" + "_u"], f[tag % "topk" + "_w"],
                                              f[tag % "topk" + "_s"], u, w, s, (cu, cw, cs))
    finally:
        for G in graphs.values():
            G.close()


@pytest.mark.parametrize("env", [dict(), dict(NLP_HASH="1"), dict(NLP_WEDGE_BUDGET="3000"),
                                 dict(NLP_BUCKET_FUSED="1"), dict(NLP_GROUPING="lsd")])
def test_gpu_maxfactor2_every_path_vs_oracle(gpu, oracle, env):
    """The MAXFACTOR2 filter on every path (sort path, hash path, chunked
    path 2, fused bucket, LSD grouping) against the oracle on a multigraph."""
    off, keys = random_csr(6000, 12, 11)
    with _env(**env):
        with gpu.Graph(off, keys) as G:
            for m in (0, 1, 3, 7):
                for H in (0, 4, 16):
                    for F in (1, 3):
                        u, w, s, t = G.predict(m, H, 2000, maxfactor2=F)
                        eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=2000, maxfactor2=F)
                        assert_canonical_equal(eu, ew, es, u, w, s)


def test_gpu_count_query_and_copy_last(gpu, golden, oracle):
    """nlp.h count query: out = NULL predicts and keeps the result on the
    device (*out_count = its size), nlp_copy_last fetches it; max_edges = 0
    predicts nothing (the reference's o.maxEdges > 0 guard)."""
    import ctypes
    g = golden["g3k"]
    L = gpu.lib()
    with gpu.Graph(g["offsets"], g["keys"]) as G:
        for m, H in ((1, 4), (7, 8), (0, 0)):
            eu, ew, es, info = oracle.predict(g["offsets"], g["keys"], m, H)
            cnt, t = ctypes.c_uint64(), gpu.Timing()
            assert L.nlp_predict(G._h, m, H, 0.0, gpu.UINT64_MAX, 1, None, ctypes.byref(cnt), ctypes.byref(t)) == 0
            assert cnt.value == len(eu) == t.candidates
            out = np.zeros(cnt.value + 5, dtype=gpu.EDGE_DTYPE)
            got = ctypes.c_uint64()
            assert L.nlp_copy_last(G._h, out.ctypes.data, cnt.value + 5, ctypes.byref(got)) == 0
            assert got.value == cnt.value
            assert_canonical_equal(eu, ew, es, out["u"][:got.value], out["v"][:got.value], out["score"][:got.value])
            # a shorter copy takes the first n links
            assert L.nlp_copy_last(G._h, out.ctypes.data, 7, ctypes.byref(got)) == 0 and got.value == min(7, len(eu))
            t0 = gpu.Timing()
            assert L.nlp_predict(G._h, m, H, 0.0, 0, 1, None, ctypes.byref(cnt), ctypes.byref(t0)) == 0
            assert cnt.value == 0 and t0.candidates == 0
            assert L.nlp_copy_last(G._h, out.ctypes.data, 10, ctypes.byref(got)) == 0 and got.value == 0


def test_gpu_exclusion_without_edge_table(gpu, oracle):
    """First-order exclusion by the edge filter + list search (NLP_ETAB=0, the
    path taken when the membership table does not fit) equals the table path
    and the oracle."""
    off, keys = random_csr(8000, 14, 5)
    k = 3000
    with gpu.Graph(off, keys) as Gt:
        res = {(m, H): Gt.predict(m, H, k) for m in (0, 1, 7, 8) for H in (0, 2, 16)}
    with _env(NLP_ETAB="0"):
        with gpu.Graph(off, keys) as G:
            for (m, H), (u, w, s, t) in res.items():
                u2, w2, s2, t2 = G.predict(m, H, k)
                assert_canonical_equal(u, w, s, u2, w2, s2)
                eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
                assert_canonical_equal(eu, ew, es, u2, w2, s2)


@pytest.mark.parametrize("env", [dict(NLP_DIRECT="0"), dict(NLP_MSD_PASSES="2"), dict(NLP_DX_BITS="1"),
                                 dict(NLP_DX_BITS="3"), dict(NLP_DX_BITS="12"), dict(NLP_COUNTED="0"),
                                 dict(NLP_EDGE_FILTER="2"), dict(NLP_SV_PACK="0")])
def test_gpu_sort_path_variants_equal(gpu, oracle, env):
    """Sort-path variants (two MSD passes + group sort, separate grouping and
    scoring, direct buckets so wide that k_sp_grouprun sorts 2 or 4 keys per
    thread or falls back on too-big ranges, look-back ordering passes instead
    of the counted k_sp_cpass, the edge filter in front of the membership
    table, unpacked survivor rows) give the default's results."""
    off, keys = random_csr(9000, 14, 21)
    k = 2500
    with gpu.Graph(off, keys) as G:
        res = {(m, H): G.predict(m, H, k) for m in (0, 1, 7) for H in (1, 2, 4, 8)}
    with _env(**env):
        with gpu.Graph(off, keys) as G:
            for (m, H), (u, w, s, t) in res.items():
                u2, w2, s2, t2 = G.predict(m, H, k)
                assert_canonical_equal(u, w, s, u2, w2, s2)
                assert t["candidates"] == t2["candidates"]
    eu, ew, es, _ = oracle.predict(off, keys, 1, 4, max_edges=k)
    assert_canonical_equal(eu, ew, es, *res[(1, 4)][:3])


@pytest.mark.parametrize("n,avg,H,env", [(100000, 8, 6, {}), (150000, 6, 6, dict(NLP_COUNTED="2"))])
def test_gpu_counted_passes_tiles_and_redo(gpu, oracle, n, avg, H, env):
    """Counted ordering passes (k_sp_cpass: per-tile digit counts from the pass
    before instead of a look-back) over ~97 candidate tiles, and -- forced
    beyond CP_MAXT = 128 tiles (~148) by NLP_COUNTED=2 -- the F_CPASS redo
    with look-back passes; both equal the oracle and the look-back build."""
    off, keys = random_csr(n, avg, 5, alpha=0.5)
    eu, ew, es, _ = oracle.predict(off, keys, 1, H, max_edges=10**9)
    k = len(eu)
    with _env(**env):
        with gpu.Graph(off, keys) as G:
            for _ in range(2):  # capture, then replay
                u, w, s, t = G.predict(1, H, k)
                assert_canonical_equal(eu, ew, es, u, w, s)
                assert t["candidates"] == k
    with _env(NLP_COUNTED="0"):
        with gpu.Graph(off, keys) as G:
            u, w, s, _ = G.predict(1, H, k)
            assert_canonical_equal(eu, ew, es, u, w, s)


@pytest.mark.parametrize("env", [{}])
def test_gpu_async_batch_equals_sync(gpu, oracle, env):
    """nlp_predict_device_async / nlp_sync: a call with no synchronous
    predecessor runs synchronously; after a synchronous call with the same
    arguments the calls are only enqueued (kernel by kernel); a batch mixing
    both ends with the last
    call's count and output; nlp_sync with nothing pending is refused."""
    import torch
    off, keys = random_csr(20000, 12, 31)
    k = 4000
    st = torch.cuda.current_stream()
    with _env(**env), gpu.Graph(off, keys) as G:
        with pytest.raises(gpu.NlpError) as e:
            G.sync()
        assert e.value.status == 1
        ref = {}
        for m, H in ((1, 4), (0, 8), (7, 4)):
            eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
            ref[(m, H)] = (eu, ew, es)
        outs = {mh: torch.zeros((k, 3), dtype=torch.int32, device="cuda") for mh in ref}
        for rnd in range(3):  # 0: nothing replayable yet; later rounds replay
            for (m, H), out in outs.items():
                out.zero_()
                for _ in range(4):
                    G.predict_device_async(m, H, k, out, stream=st)
                with pytest.raises(gpu.NlpError) as e:  # a batch is pending: synchronous calls are refused
                    G.predict_device(m, H, k, out, stream=st)
                assert e.value.status == 1
                cnt, t = G.sync()
                eu, ew, es = ref[(m, H)]
                assert cnt == len(eu) and t["candidates"] >= cnt
                a = out[:cnt].cpu().numpy()
                assert_canonical_equal(eu, ew, es, a[:, 0].view(np.uint32), a[:, 1].view(np.uint32),
                                       a[:, 2].view(np.float32))
                G.predict_device(m, H, k, out, stream=st)  # makes the next round's calls replayable
        # a batch that ends with a different (synchronous) call reports that call
        (m1, H1), (m2, H2) = list(outs)[:2]
        G.predict_device(m1, H1, k, outs[(m1, H1)], stream=st)
        for _ in range(3):
            G.predict_device_async(m1, H1, k, outs[(m1, H1)], stream=st)
        G.predict_device_async(m2, H2, k, outs[(m2, H2)], u_begin=0, u_end=gpu.UINT64_MAX - 1, stream=st)
        cnt, _ = G.sync()
        assert cnt == len(ref[(m2, H2)][0])


def test_gpu_survivor_scan_after_other_survivor_set(gpu, oracle):
    """the fused/counted paths must reset k_sp_survivors'
    look-back descriptors when that scan runs (no degree-class index: H = 0,
    H > 1024).  A graph of > 32768 vertices (several survivor tiles), an
    Adamic-Adar call (ordered survivor scan, other survivor set) first, then
    count-metric calls without the index on the same handle, each exact."""
    off, keys = random_csr(40000, 6, 11)
    k = 8000
    with gpu.Graph(off, keys) as G:
        for m, H in ((7, 4), (1, 0), (7, 8), (1, 2048), (0, 0), (8, 3), (1, 0)):
            u, w, s, t = G.predict(m, H, k)
            eu, ew, es, info = oracle.predict_par(off, keys, m, H, max_edges=k, threads=ORACLE_THREADS)
            assert_canonical_equal(eu, ew, es, u, w, s)
            assert t["wedges"] == info["wedges_gt"]


@pytest.mark.parametrize("n,avg,H", [(30000, 6, 2), (30000, 6, 3), (100000, 8, 4), (150000, 6, 6)])
def test_gpu_small_order_equals_counted_passes(gpu, oracle, n, avg, H):
    """k_sp_order_rank (one launch ranks all candidates of a small fused call)
    against the counted passes (NLP_SMALL_ORDER=0) and the oracle, below
    and above its SO_MAX = 16384 candidates; NLP_SMALL_ORDER=2 forces it
    whatever the estimate, so calls beyond SO_MAX take the F_SMALL redo."""
    off, keys = random_csr(n, avg, 21 + H)
    k_list = (50, 7000, 10 ** 6)
    res = {}
    for env in ("1", "0", "2"):
        os.environ["NLP_SMALL_ORDER"] = env
        try:
            with gpu.Graph(off, keys) as G:
                for m in (1, 0, 6):
                    for k in k_list:
                        u, w, s, t = G.predict(m, H, k)
                        res[(env, m, k)] = (u, w, s, t["candidates"])
                        if k == 10 ** 6:
                            u2, w2, s2, t2 = G.predict(m, H, k)  # the memo after a redo
                            assert np.array_equal(u, u2) and np.array_equal(w, w2)
        finally:
            del os.environ["NLP_SMALL_ORDER"]
    for m in (1, 0, 6):
        for k in k_list:
            eu, ew, es, info = oracle.predict(off, keys, m, H, max_edges=k)
            for env in ("1", "0", "2"):
                u, w, s, c = res[(env, m, k)]
                assert_canonical_equal(eu, ew, es, u, w, s)
                assert c == info["candidates"]


def test_gpu_generic_score_lambdas(gpu, golden, oracle, tmp_path):
    """The generic predictLinksWithIntersectionBasicOmp / ...Omp<CUSTOMVALUE =
    false> with user score lambdas (tests/cpp/generic_main.cxx): the
    reference's own Jaccard lambda (predict.hxx:557-559) through the generic
    entry equals the built-in metric bit for bit, and a count-based lambda
    equals its host recomputation from the oracle's intersection counts, in
    the canonical order."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "generic_main")
    lib = os.path.join(root, "neighborhood-link-prediction-openmp_amd")
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "cpp", "generic_main.cxx"), "-L", lib, "-lnlp", "-Wl,-rpath," + lib,
                    "-o", exe], check=True)
    g = golden["g3k"]
    k = int(g["k"][0])
    csr = str(tmp_path / "g.csr")
    oracle.write_csr(csr, g["offsets"], g["keys"])
    for H in (0, 4, 8):
        pre = str(tmp_path / ("o%d" % H))
        subprocess.run([exe, csr, str(H), str(k), pre], check=True, timeout=300)
        a = oracle.read_edges(pre + ".jac_generic")
        b = oracle.read_edges(pre + ".jac_builtin")
        assert all(np.array_equal(x.view(np.uint32), y.view(np.uint32)) for x, y in zip(a, b))
        eu, ew, es, _ = oracle.predict(g["offsets"], g["keys"], 1, H, max_edges=k)
        assert_canonical_equal(eu, ew, es, *a)
        # the custom lambda from the oracle's counts (CN with minScore -1: every touched w, count 0 included)
        cu_, cw_, cn_, _ = oracle.predict(g["offsets"], g["keys"], 0, H, max_edges=None, min_score=-1.0)
        sc = cn_.astype(np.float32) * np.float32(0.5) + np.float32(1.0) / (cu_ % 7 + 1).astype(np.float32)
        keep = sc > 0
        from parity import keys_of
        kk = keys_of(sc[keep]).astype(np.int64)
        order = np.lexsort((cw_[keep], cu_[keep], -kk))[:k]
        u, w, s = oracle.read_edges(pre + ".custom")
        assert np.array_equal(u, cu_[keep][order]) and np.array_equal(w, cw_[keep][order])
        assert np.array_equal(s.view(np.uint32), sc[keep][order].view(np.uint32))
