"""The multi-device graph handle behind the C-ABI (nlp_graph_create_multi,
SURVEY §8(b) devices[], ndev): P logical partitions of the source range, here
all on the box's one GPU (devices = [0] * P), each predicting its canonical
top-k, then the in-library histogram-first selection and the merge.  Results
must equal the oracle (and so the single-device handle) bit for bit and in
order, for every metric, hub threshold, k (ties split across partitions) and
the all-candidates query; the C++ header reaches the same path through
NLP_DEVICES."""
import os
import subprocess

import numpy as np
import pytest

from parity import assert_canonical_equal
from test_gpu_parity import random_csr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu(nlp):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return nlp


@pytest.mark.parametrize("P", [2, 4, 8])
def test_gpu_logical_partitions_equal_oracle(gpu, oracle, golden, P):
    for off, keys, k in ((golden["g3k"]["offsets"], golden["g3k"]["keys"], int(golden["g3k"]["k"][0])),
                         random_csr(20000, 10, 9) + (3000,)):
        with gpu.Graph(off, keys, devices=[0] * P) as G:
            n_parts, _ = G.parts()
            assert n_parts == P
            for m, H in ((1, 4), (7, 8), (0, 0), (3, 2), (8, 16), (1, 2048)):
                for me in (k, 37, None):
                    u, w, s, t = G.predict(m, H, me)
                    eu, ew, es, info = oracle.predict(off, keys, m, H, max_edges=me)
                    assert_canonical_equal(eu, ew, es, u, w, s)
                    assert t["candidates"] == info["candidates"] and t["wedges"] == info["wedges_gt"]
                    _, b = G.parts()
                    assert b[0] == 0 and b[-1] == len(off) - 1 and np.all(np.diff(b.astype(np.int64)) >= 0)


def test_gpu_partitions_device_output_and_ranges(gpu, oracle):
    import torch
    off, keys = random_csr(20000, 10, 10)
    span = len(off) - 1
    k = 2500
    with gpu.Graph(off, keys, devices=[0, 0, 0]) as G:
        out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
        for m, H, ua, ub in ((1, 4, 0, span), (0, 8, span // 5, span - span // 7), (7, 4, 100, 101)):
            n, t = G.predict_device(m, H, k, out, ua, ub)
            u, w, s = gpu.edges_from_tensor(out, n)
            eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k, u_begin=ua, u_end=ub)
            assert_canonical_equal(eu, ew, es, u, w, s)
        # the last result stays on the handle (count query + copy, evaluation)
        n, _ = G.predict_device(1, 4, k, out)
        assert G.last_common() >= 0


def test_gpu_cpp_header_on_partitions(gpu, golden, oracle, tmp_path):
    """include/nlp/predict.hxx with NLP_DEVICES=0,0,0,0: the reference's
    template names on four partitions equal the oracle."""
    from nlp_amd import build as b
    exe = b.build_cpp_test(verbose=False)
    g = golden["g3k"]
    k = int(g["k"][0])
    csr = str(tmp_path / "g.csr")
    oracle.write_csr(csr, g["offsets"], g["keys"])
    env = dict(os.environ, NLP_DEVICES="0,0,0,0")
    pre = str(tmp_path / "out4")
    subprocess.run([exe, csr, "4", str(k), pre], check=True, timeout=300, env=env)
    for m in range(9):
        u, w, s = oracle.read_edges(pre + "." + str(m))
        eu, ew, es, _ = oracle.predict(g["offsets"], g["keys"], m, 4, max_edges=k)
        assert_canonical_equal(eu, ew, es, u, w, s)


def test_gpu_partitions_replicas_copied_device_to_device(gpu, oracle, golden, monkeypatch):
    """NLP_MULTI_EACH=1: one member graph per partition even on a repeated
    device, so members 1.. are built from member 0's CSR by the device-to-device
    (peer) copy that an 8-GPU handle uses instead of one PCIe upload per GPU."""
    monkeypatch.setenv("NLP_MULTI_EACH", "1")
    g = golden["g3k"]
    off, keys, k = g["offsets"], g["keys"], int(g["k"][0])
    with gpu.Graph(off, keys, devices=[0, 0, 0]) as G:
        for m, H in ((1, 4), (0, 0), (8, 16)):
            u, w, s, _ = G.predict(m, H, k)
            eu, ew, es, _ = oracle.predict(off, keys, m, H, max_edges=k)
            assert_canonical_equal(eu, ew, es, u, w, s)
