"""Parity checks shared by the oracle tests and the GPU tests (SURVEY.md
Appendix A.1 contract).

Against the reference (whose tie order depends on the OpenMP schedule):
  1. same number of links;
  2. identical score multiset (bitwise; NaN compared by NaN-ness);
  3. identical set of links strictly above the k-th score;
  4. every link at the k-th score is one of the reference's candidates with
     that score (the tie set).
Against the canonical oracle: identical arrays, in order.
"""
import numpy as np


def keys_of(scores):
    s = np.asarray(scores, dtype=np.float32).copy()
    s[s == 0] = 0.0
    b = s.view(np.uint32)
    k = np.where(b & 0x80000000, ~b, b | 0x80000000).astype(np.uint32)
    k[np.isnan(s)] = 0
    return k


def pair_keys(u, w):
    return (np.asarray(u, np.uint64) << np.uint64(32)) | np.asarray(w, np.uint64)


def assert_same_candidates(ru, rw, rs, ou, ow, os_):
    """Multiset equality of (u, w, score bits) -- all-candidates mode."""
    assert len(ru) == len(ou), (len(ru), len(ou))
    a = np.lexsort((rw, ru))
    b = np.lexsort((ow, ou))
    assert np.array_equal(np.asarray(ru)[a], np.asarray(ou)[b])
    assert np.array_equal(np.asarray(rw)[a], np.asarray(ow)[b])
    ka, kb = keys_of(np.asarray(rs)[a]), keys_of(np.asarray(os_)[b])
    assert np.array_equal(ka, kb), "scores differ at %d entries" % int((ka != kb).sum())


def assert_topk_matches_reference(ru, rw, rs, ou, ow, os_, ref_cand=None):
    """Contract 1-4 above.  ref_cand = (u, w, s) of all reference candidates
    (for the tie-set check); without it ties are only checked by score."""
    assert len(ru) == len(ou), (len(ru), len(ou))
    if len(ru) == 0:
        return
    rk, ok = keys_of(rs), keys_of(os_)
    assert np.array_equal(np.sort(rk), np.sort(ok)), "score multisets differ"
    kth = rk.min()
    ra = set(pair_keys(np.asarray(ru)[rk > kth], np.asarray(rw)[rk > kth]).tolist())
    oa = set(pair_keys(np.asarray(ou)[ok > kth], np.asarray(ow)[ok > kth]).tolist())
    assert ra == oa, "above-boundary sets differ (%d vs %d)" % (len(ra), len(oa))
    ot = pair_keys(np.asarray(ou)[ok == kth], np.asarray(ow)[ok == kth])
    if ref_cand is not None:
        cu, cw, cs = ref_cand
        ck = keys_of(cs)
        tie_set = set(pair_keys(np.asarray(cu)[ck == kth], np.asarray(cw)[ck == kth]).tolist())
        assert set(ot.tolist()) <= tie_set, "tie links outside the reference's tie set"
    assert len(set(pair_keys(ou, ow).tolist())) == len(ou), "duplicate links in output"


def assert_canonical_equal(eu, ew, es, ou, ow, os_):
    """Exact equality with the canonical oracle (order included)."""
    assert len(eu) == len(ou), (len(eu), len(ou))
    assert np.array_equal(np.asarray(eu), np.asarray(ou)), "u differs"
    assert np.array_equal(np.asarray(ew), np.asarray(ow)), "w differs"
    assert np.array_equal(keys_of(es), keys_of(os_)), "scores differ"


def assert_canonical_order(u, w, s):
    """Sorted by (score key desc, u asc, w asc), u < w, no duplicates."""
    k = keys_of(s).astype(np.int64)
    u = np.asarray(u, np.int64)
    w = np.asarray(w, np.int64)
    assert np.all(u < w)
    if len(k) > 1:
        dk = k[1:] - k[:-1]
        du = u[1:] - u[:-1]
        dw = w[1:] - w[:-1]
        ok = (dk < 0) | ((dk == 0) & ((du > 0) | ((du == 0) & (dw > 0))))
        assert np.all(ok), "not in canonical order at %s" % np.nonzero(~ok)[0][:5]


def f1_score(pu, pw, del_u, del_w):
    """main.cxx:48-57, 199-206: predictions as both directions, set
    intersection with the directed deletions; P, R, F1."""
    ins = set(pair_keys(pu, pw).tolist()) | set(pair_keys(pw, pu).tolist())
    dels = set(pair_keys(del_u, del_w).tolist())
    common = len(ins & dels)
    p = common / max(len(ins), 1)
    r = common / max(len(dels), 1)
    f = 0.0 if p + r == 0 else 2 * p * r / (p + r)
    return p, r, f
