"""SURVEY §8(f) N1 + N2 on the device (nlp_ingest_device,
nlp_delete_edges_device) bit-exact against the reference's own ingest:
tests/golden/ingest_*.npz (and the prediction fixtures g300 / g3k) were made by
oracle/_ref/ref_driver -- readMtxOmpW -> symmetrizeOmp -> removeSelfLoopsOmpU ->
generateEdgeDeletions(default_random_engine(seed)) -> tidyBatchUpdateU ->
applyBatchUpdateOmpU (main.cxx:164-169, 241-245) -- so the CSR after the
deletions (duplicate entries of the symmetrize quirk included) and the
directed deletion list must match byte for byte."""
import os
import sys

import numpy as np
import pytest

from mtx import parse_mtx

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gpu(nlp):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return nlp


def ingest(nlp, text, seed, d):
    import torch
    u, v, n, _ = parse_mtx(text)
    src = torch.from_numpy(u.view(np.int32)).cuda()
    dst = torch.from_numpy(v.view(np.int32)).cuda()
    off, keys = nlp.ingest_device(src, dst, n)  # ref_driver ingest symmetrizes every input
    batch = int(d * keys.numel() / 2)  # size_t(d * x.size()/2), main.cxx:166
    off2, keys2, du, dv, state = nlp.delete_edges_device(off, keys, batch, seed)
    return (off2.cpu().numpy().astype(np.uint64), keys2.cpu().numpy().view(np.uint32),
            du.cpu().numpy().view(np.uint32), dv.cpu().numpy().view(np.uint32), state)


@pytest.mark.parametrize("name", ["general", "sym", "d0"])
def test_gpu_ingest_matches_reference_fixtures(gpu, name):
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "ingest_%s.npz" % name), allow_pickle=False))
    off, keys, du, dv, _ = ingest(gpu, g["mtx"].tobytes(), int(g["seed"][0]), float(g["d"][0]))
    assert np.array_equal(off, g["offsets"]), "offsets differ"
    assert np.array_equal(keys, g["keys"]), "adjacency differs"
    assert np.array_equal(du, g["del_u"]) and np.array_equal(dv, g["del_w"]), "deletions differ"


@pytest.mark.parametrize("name,params", [("g300", (300, 1200, 0.6, 1)), ("g3k", (3000, 20000, 0.6, 7))])
def test_gpu_ingest_reproduces_prediction_fixtures(gpu, tmp_path, name, params):
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import chung_lu_mtx
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False))
    mtx = str(tmp_path / "in.mtx")
    chung_lu_mtx(mtx, *params)
    off, keys, du, dv, _ = ingest(gpu, open(mtx, "rb").read(), 42, 0.1)
    assert np.array_equal(off, g["offsets"]) and np.array_equal(keys, g["keys"])
    assert np.array_equal(du, g["del_u"]) and np.array_equal(dv, g["del_w"])
    if name == "g3k":  # the symmetrize duplicates are there
        assert int(np.sum(np.diff(keys.astype(np.int64)) == 0)) > 0


def test_gpu_rng_state_continues_one_engine(gpu):
    """Two batches from one engine (main.cxx keeps one default_random_engine):
    the second call, started from the state the first returned, draws what a
    single engine draws next -- the same as deleting twice on the host."""
    import torch
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "ingest_general.npz"), allow_pickle=False))
    u, v, n, _ = parse_mtx(g["mtx"].tobytes())
    off, keys = gpu.ingest_device(torch.from_numpy(u.view(np.int32)).cuda(), torch.from_numpy(v.view(np.int32)).cuda(), n)
    a = gpu.delete_edges_device(off, keys, 200, 7)
    b = gpu.delete_edges_device(off, keys, 200, a[4])
    c = gpu.delete_edges_device(off, keys, 400, 7)  # the same 400 draws in one call
    pairs = lambda r: set(zip(r[2].cpu().tolist(), r[3].cpu().tolist()))
    assert pairs(a) | pairs(b) == pairs(c)
    assert b[4] == c[4]


def test_gpu_workload_uses_the_reference_ingest(gpu, tmp_path):
    """graphgen's GPU workload (the bench / config graphs) = the host
    restatement of the reference's ingest (include/nlp/ingest.hxx, itself
    bit-exact against the reference) run on the same pairs written as a
    MatrixMarket file, with the same seed and deletion fraction."""
    import subprocess
    import torch
    import nlp_loader
    gg = nlp_loader.load_sub("graphgen")
    spec = gg.CONFIGS["C2-soc-LiveJournal1"]
    off, keys, du, dw, info = gg.make_workload(spec, "cuda", scale=0.002)
    assert info["ingest"] == "reference"
    n, m, alpha, seed, d = info["n"], info["m"], spec[2], spec[3], spec[4]
    src, dst = gg.chung_lu_edges(n, m, alpha, seed, "cpu")  # counter-based: the same pairs as on the device
    mtx = str(tmp_path / "w.mtx")
    with open(mtx, "w") as f:
        f.write("%%%%MatrixMarket matrix coordinate pattern general\n%d %d %d\n" % (n, n, src.numel()))
        f.write("\n".join("%d %d" % (a, b) for a, b in zip(src.tolist(), dst.tolist())) + "\n")
    exe = str(tmp_path / "ingest_main")
    subprocess.run(["g++", "-std=c++17", "-O2", "-fopenmp", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "ingest_main.cxx"), "-o", exe], check=True)
    subprocess.run([exe, mtx, str(seed + 1000), repr(d), str(tmp_path / "h")], check=True, capture_output=True)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    hoff, hkeys = pyoracle.read_csr(str(tmp_path / "h.csr"))
    hu, hw = pyoracle.read_deletions(str(tmp_path / "h.del"))
    assert np.array_equal(off.cpu().numpy().astype(np.uint64), hoff)
    assert np.array_equal(keys.cpu().numpy().view(np.uint32), hkeys)
    assert np.array_equal(du.cpu().numpy().view(np.uint32), hu) and np.array_equal(dw.cpu().numpy().view(np.uint32), hw)


def test_ingest_rejects_id_above_n(gpu):
    """One id above n in the pairs: NLP_ERR_INVALID, nothing indexed by it
    (the rows are addressed by id on the device)."""
    import torch
    src = torch.tensor([1, 2, 3, 9], dtype=torch.int32, device="cuda")
    dst = torch.tensor([2, 3, 1, 1], dtype=torch.int32, device="cuda")
    with pytest.raises(gpu.NlpError) as e:
        gpu.ingest_device(src, dst, 5)
    assert e.value.status == 1
    off, keys = gpu.ingest_device(src, dst, 9)  # the same pairs with n large enough
    assert int(off[-1]) == keys.numel() == 8


def _dev_route(tmp_path, mtx_bytes, seed, d):
    """nlp_main's ingest route (tests/cpp/ingest_dev_main.cxx: readMtxPairs on all
    threads, nlp_dcsr_ingest, nlp_dcsr_delete_batch) on a MatrixMarket text."""
    import json
    import subprocess
    from nlp_amd import build as B
    exe = B.build_ingest_dev(verbose=False)
    mtx = str(tmp_path / "in.mtx")
    open(mtx, "wb").write(mtx_bytes)
    r = subprocess.run([exe, mtx, str(seed), repr(d), str(tmp_path / "dev")], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-1000:]
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    off, keys = pyoracle.read_csr(str(tmp_path / "dev.csr"))
    du, dw = pyoracle.read_deletions(str(tmp_path / "dev.del"))
    return off, keys, du, dw, json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("name", ["general", "sym", "d0"])
def test_gpu_device_route_matches_reference_fixtures(gpu, tmp_path, name):
    """N1 at the drivers' level: nlp_main's route -- parallel
    MatrixMarket parse + nlp_dcsr_* -- byte for byte against the reference's ingest."""
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "ingest_%s.npz" % name), allow_pickle=False))
    off, keys, du, dw, info = _dev_route(tmp_path, g["mtx"].tobytes(), int(g["seed"][0]), float(g["d"][0]))
    assert np.array_equal(off, g["offsets"]) and np.array_equal(keys, g["keys"])
    assert np.array_equal(du, g["del_u"]) and np.array_equal(dw, g["del_w"])


@pytest.mark.parametrize("name,params", [("g300", (300, 1200, 0.6, 1)), ("g3k", (3000, 20000, 0.6, 7))])
def test_gpu_device_route_reproduces_prediction_fixtures(gpu, tmp_path, name, params):
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import chung_lu_mtx
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False))
    mtx = str(tmp_path / "gen.mtx")
    chung_lu_mtx(mtx, *params)
    off, keys, du, dw, info = _dev_route(tmp_path, open(mtx, "rb").read(), 42, 0.1)
    assert np.array_equal(off, g["offsets"]) and np.array_equal(keys, g["keys"])
    assert np.array_equal(du, g["del_u"]) and np.array_equal(dw, g["del_w"])


@pytest.mark.timeout(300)
def test_gpu_device_route_c2_size_file(gpu, tmp_path):
    """A generated C2-sized MatrixMarket file (soc-LiveJournal1 shape: 4.85 M
    vertices, 69 M lines, ~1 GB of text) through nlp_main's route: parsed on
    all threads and ingested on the device in seconds (times reported)."""
    import json
    import subprocess
    from nlp_amd import build as B
    exe = B.build_ingest_dev(verbose=False)
    mtx = str(tmp_path / "c2.mtx")
    subprocess.run([exe, "gen", mtx, "4847571", "68993773", "0.6", "12"], check=True, timeout=240)
    r = subprocess.run([exe, mtx, "42", "0.1", str(tmp_path / "c2")], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-1000:]
    info = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(info))
    d = os.environ.get("NLP_TEST_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "c2_mtx_ingest.json"), "w") as f:
            json.dump(info, f)
    assert info["lines"] == 68993773
    assert info["size"] > 68993773  # symmetrized (duplicate pairs and self loops removed)
    assert info["parse_ms"] + info["ingest_ms"] < 60000
