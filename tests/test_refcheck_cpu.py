"""The full-size reference checker (tests/refcheck.py) on the CPU, with the
reference's own small fixtures: the canonical oracle's top-k stands in for the
GPU result, the reference's OpenMP top-k is ref_k, and the reference's
sequential all-candidate list cut at the k-th score is the tie-set call.  Also
checks that a wrong tie, a changed score and an F1 outside the bounds fail."""
import numpy as np
import pytest

from conftest import load_golden
import refcheck

torch = pytest.importorskip("torch")


def _case(oracle, name, m, H):
    g = load_golden(name)
    k = int(g["k"][0])
    tag = "%d_%d" % (m, H)
    ru, rw, rs = g["topk_%s_u" % tag], g["topk_%s_w" % tag], g["topk_%s_s" % tag]
    cu, cw, cs = g["cand_%s_u" % tag], g["cand_%s_w" % tag], g["cand_%s_s" % tag]
    u, w, s, _ = oracle.predict(g["offsets"], g["keys"], m, H, max_edges=k)
    kth = refcheck.keys_t(torch.as_tensor(rs)).min()
    ge = refcheck.keys_t(torch.as_tensor(cs)) >= kth
    ge = ge.numpy()
    gpu = (torch.as_tensor(u.astype(np.int64)), torch.as_tensor(w.astype(np.int64)), torch.as_tensor(s))
    return g, k, gpu, (ru, rw, rs), (cu[ge], cw[ge], cs[ge])


@pytest.mark.parametrize("m,H", [(1, 8), (7, 8), (0, 8)])
def test_refcheck_accepts_the_oracle(oracle, m, H):
    g, k, gpu, ref_k, ref_ge = _case(oracle, "g3k", m, H)
    r = refcheck.check_contract(gpu, ref_k, ref_ge, k, g["del_u"], g["del_w"], dev="cpu")
    assert r["n"] == len(ref_k[0]) and r["f1_lo"] <= r["f1_gpu"] <= r["f1_hi"]
    assert r["ties_total"] >= r["ties_taken"]


@pytest.mark.parametrize("m,H", [(1, 8), (7, 8)])
def test_refcheck_tie_set_call_with_one_more(oracle, m, H):
    """The full-size form: the tie-set call asks for |at or above| + 1 links and
    gets one below the k-th score -- accepted; asked for exactly |at or above|
    (as if our output had lost a candidate, so our count is one short), every
    link it returns is at or above the k-th score -- rejected."""
    g, k, gpu, ref_k, ref_ge = _case(oracle, "g3k", m, H)
    tag = "%d_%d" % (m, H)
    cu, cw, cs = g["cand_%s_u" % tag], g["cand_%s_w" % tag], g["cand_%s_s" % tag]
    kth = refcheck.keys_t(torch.as_tensor(ref_k[2])).min()
    below = (refcheck.keys_t(torch.as_tensor(cs)) < kth).numpy()
    j = int(np.nonzero(below)[0][0])
    plus = tuple(np.concatenate([a, b[j:j + 1]]) for a, b in zip(ref_ge, (cu, cw, cs)))
    r = refcheck.check_contract(gpu, ref_k, plus, k, g["del_u"], g["del_w"], dev="cpu", asked=len(plus[0]))
    assert r["ties_total"] >= r["ties_taken"]
    short = tuple(a[:-1] for a in ref_ge)  # one tie fewer: our count would have been one short
    with pytest.raises(AssertionError):
        refcheck.check_contract(gpu, ref_k, short, k, g["del_u"], g["del_w"], dev="cpu", asked=len(short[0]))


def test_refcheck_single_reference_call(oracle):
    """The one-call form (the tie-set call alone stands for the reference's
    top-k): accepted for the oracle's result, a changed score rejected."""
    g, k, gpu, ref_k, ref_ge = _case(oracle, "g3k", 1, 8)
    cu, cw, cs = g["cand_1_8_u"], g["cand_1_8_w"], g["cand_1_8_s"]
    kth = refcheck.keys_t(torch.as_tensor(ref_k[2])).min()
    j = int(np.nonzero((refcheck.keys_t(torch.as_tensor(cs)) < kth).numpy())[0][0])
    plus = tuple(np.concatenate([a, b[j:j + 1]]) for a, b in zip(ref_ge, (cu, cw, cs)))
    r = refcheck.check_contract(gpu, None, plus, k, g["del_u"], g["del_w"], dev="cpu", asked=len(plus[0]))
    assert r["common_ref"] is None and r["f1_lo"] <= r["f1_gpu"] <= r["f1_hi"]
    u, w, s = gpu
    s2 = s.clone()
    s2[0] = torch.nextafter(s2[0], torch.tensor(0.0))
    with pytest.raises(AssertionError):
        refcheck.check_contract((u, w, s2), None, plus, k, g["del_u"], g["del_w"], dev="cpu", asked=len(plus[0]))


def test_refcheck_rejects_wrong_results(oracle):
    g, k, gpu, ref_k, ref_ge = _case(oracle, "g3k", 1, 8)
    u, w, s = gpu
    # a changed score
    s2 = s.clone()
    s2[0] = torch.nextafter(s2[0], torch.tensor(0.0))
    with pytest.raises(AssertionError):
        refcheck.check_contract((u, w, s2), ref_k, ref_ge, k, g["del_u"], g["del_w"], dev="cpu")
    # a boundary link that is not a candidate at that score
    kk = refcheck.keys_t(s)
    i = int(torch.nonzero(kk == kk.min())[-1])
    w2 = w.clone()
    w2[i] = int(g["offsets"].shape[0])  # no such vertex
    with pytest.raises(AssertionError):
        refcheck.check_contract((u, w2, s), ref_k, ref_ge, k, g["del_u"], g["del_w"], dev="cpu")
