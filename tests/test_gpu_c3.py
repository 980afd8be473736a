"""BASELINE configs[2] / SURVEY §8(d) C3: the uk-2005-shaped stand-in
(n = 39.5 M, M = 1.7e9) -- the "HBM-roofline run".  LHub Adamic-Adar (the
config's metric) and Jaccard at H = 4 (path 1), exact against the parallel
oracle, order included; Adamic-Adar at H = 16 (path 4: ordered accumulation in
the row kernels, sort-mode items in the hub pass -- k = 8.7e7 of 9.6e8
candidates) against the reference itself, which with refcheck's canonical
checks pins the same bits.  (Jaccard at H = 16 on path 4 is the C4 tests'
call.)"""
import numpy as np
import pytest

from bigconf import ORACLE_THREADS, Config
from parity import assert_canonical_equal, assert_canonical_order

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c3(nlp):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = Config(nlp, "C3-uk-2005")
    yield c
    c.close()


def _check(c, oracle, metric, H, path=None):
    out = c.out()
    n, t = c.G.predict_device(metric, H, c.k, out)
    if path is not None:
        assert t["path"] == path, t
    u, w, s = c.nlp.edges_from_tensor(out, n)
    del out
    eu, ew, es, oi = oracle.predict_par(c.off, c.keys, metric, H, max_edges=c.k, threads=ORACLE_THREADS)
    assert_canonical_equal(eu, ew, es, u, w, s)
    assert t["wedges"] == oi["wedges_gt"] and t["candidates"] == oi["candidates"]
    assert t["nan_candidates"] == oi["nan"]
    assert_canonical_order(u, w, s)
    return n, t


@pytest.mark.timeout(300)
def test_gpu_c3_adamic_adar_h4(c3, oracle):
    _check(c3, oracle, 7, 4, path=1)


@pytest.mark.timeout(300)
def test_gpu_c3_jaccard_h4(c3, oracle):
    _check(c3, oracle, 1, 4, path=1)


@pytest.fixture(scope="module")
def c3_csr(c3):
    import refcheck
    if not refcheck.have_ref():
        pytest.skip("oracle/_ref/ref_driver not built (needs the reference headers in the build container)")
    path, tmp = refcheck.write_csr(c3.off, c3.keys)
    yield path
    tmp.cleanup()


@pytest.mark.timeout(600)
def test_gpu_c3_adamic_adar_h16_vs_reference(c3, c3_csr, oracle):
    """BASELINE's "HBM-roofline run" (uk-2005, LHub Adamic-Adar) at H = 16 on path 4
    (ordered accumulation in the row kernels, sort-mode items in the hub pass, 3
    chunks) against the reference ITSELF (predictLinksAdamicAdarCoefficientOmp<16>):
    the A.1 contract, F1 within the tie bounds, our canonical contract (the
    oracle's output bit for bit, see refcheck) and the wedge counter."""
    import refcheck
    r = refcheck.run_reference_check(c3, c3_csr, 7, 16, "C3-uk-2005")
    assert r["n"] == c3.k and r["path"] == 4
    assert r["f1_lo"] <= r["f1_gpu"] <= r["f1_hi"]
    assert r["wedges"] == oracle.wedges_gt(c3.off, c3.keys, 16, 0, len(c3.off) - 1, threads=ORACLE_THREADS)
