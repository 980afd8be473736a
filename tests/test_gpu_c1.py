"""BASELINE configs[0] / SURVEY §8(d) C1: the web-Google-shaped stand-in
(n = 0.92 M, 0.01|E| removed) -- the reference's CPU-runnable case -- through
the HIP path for the whole MINDEGREE1 sweep of the bench metric and the
config's other metrics (main.cxx:67-80, 212-220), exact against the oracle."""
import numpy as np
import pytest

from bigconf import ORACLE_THREADS, Config
from parity import assert_canonical_equal, f1_score

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c1(nlp):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = Config(nlp, "C1-web-Google")
    yield c
    c.close()


@pytest.mark.timeout(300)
def test_gpu_c1_jaccard_hub_sweep(c1, oracle):
    for H in (0, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024):
        out = c1.out()
        n, t = c1.G.predict_device(1, H, c1.k, out)
        u, w, s = c1.nlp.edges_from_tensor(out, n)
        eu, ew, es, oi = oracle.predict_par(c1.off, c1.keys, 1, H, max_edges=c1.k, threads=ORACLE_THREADS)
        assert_canonical_equal(eu, ew, es, u, w, s)
        assert t["candidates"] == oi["candidates"], H


@pytest.mark.timeout(300)
def test_gpu_c1_all_metrics_h4_and_f1(c1, oracle):
    for m in range(9):
        out = c1.out()
        n, t = c1.G.predict_device(m, 4, c1.k, out)
        u, w, s = c1.nlp.edges_from_tensor(out, n)
        eu, ew, es, oi = oracle.predict_par(c1.off, c1.keys, m, 4, max_edges=c1.k, threads=ORACLE_THREADS)
        assert_canonical_equal(eu, ew, es, u, w, s)
        if m == 1:  # main.cxx:199-206 on the device equals the host evaluation
            c1.G.set_truth(c1.del_u.cpu().numpy(), c1.del_w.cpu().numpy())
            common = c1.G.count_common_device(out, n)
            p, r, f = f1_score(u, w, c1.del_u.cpu().numpy(), c1.del_w.cpu().numpy())
            assert abs(common / max(2 * n, 1) - p) < 1e-12
