"""Host ingest (include/nlp/ingest.hxx, SURVEY §8(f) N1 + N2) against the
reference's own ingest: MatrixMarket read, symmetrize with the duplicate quirk,
self-loop removal, the seeded deletion sampler, tidy and apply.  Bit-exact
CSR and deletion lists.  CPU only."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, GOLDEN)


@pytest.fixture(scope="module")
def ingest_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("ingest") / "ingest_main")
    subprocess.run(["g++", "-std=c++17", "-O2", "-fopenmp", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "ingest_main.cxx"), "-o", out], check=True)
    return out


def run_ingest(binary, mtx, seed, d, prefix):
    subprocess.run([binary, mtx, str(seed), str(d), prefix], check=True, capture_output=True)
    import pyoracle as O
    off, keys = O.read_csr(prefix + ".csr")
    du, dw = O.read_deletions(prefix + ".del")
    return off, keys, du, dw


def assert_same(got, g):
    off, keys, du, dw = got
    assert np.array_equal(off, g["offsets"]), "offsets differ"
    assert np.array_equal(keys, g["keys"]), "adjacency differs"
    assert np.array_equal(du, g["del_u"]) and np.array_equal(dw, g["del_w"]), "deletions differ"


@pytest.mark.parametrize("name", ["general", "sym", "d0"])
def test_ingest_matches_reference_fixtures(ingest_bin, tmp_path, name):
    g = dict(np.load(os.path.join(GOLDEN, "ingest_%s.npz" % name), allow_pickle=False))
    mtx = str(tmp_path / "in.mtx")
    open(mtx, "wb").write(g["mtx"].tobytes())
    got = run_ingest(ingest_bin, mtx, int(g["seed"][0]), float(g["d"][0]), str(tmp_path / "out"))
    assert_same(got, g)


@pytest.mark.parametrize("name,params", [("g300", (300, 1200, 0.6, 1)), ("g3k", (3000, 20000, 0.6, 7))])
def test_ingest_reproduces_prediction_fixtures(ingest_bin, tmp_path, name, params):
    """The prediction fixtures' graphs and deletions were made by the reference's
    ingest (make_golden.py): regenerate their MatrixMarket input and ingest it."""
    from make_golden import chung_lu_mtx
    g = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    mtx = str(tmp_path / "in.mtx")
    chung_lu_mtx(mtx, *params)
    got = run_ingest(ingest_bin, mtx, 42, 0.1, str(tmp_path / "out"))
    assert_same(got, g)
    # the duplicate quirk of the reference's symmetrize is present and reproduced
    off, keys = got[0], got[1]
    dup = sum(int(np.sum(np.diff(keys[off[u]:off[u + 1]].astype(np.int64)) == 0)) for u in range(len(off) - 1))
    if name == "g3k":
        assert dup > 0


def test_ingest_matches_live_reference(ingest_bin, tmp_path):
    """Against oracle/_ref/ref_driver itself (build container only)."""
    import pyoracle as O
    if not os.path.exists(O.REF_DRIVER) or not os.path.isdir("/root/reference"):
        pytest.skip("reference driver not built here")
    from make_golden import chung_lu_mtx
    for n, m, alpha, gseed, seed, d in ((1500, 9000, 0.9, 21, 5, 0.2), (800, 4000, 0.5, 22, 6, 0.02)):
        mtx = str(tmp_path / "in.mtx")
        chung_lu_mtx(mtx, n, m, alpha, gseed)
        pre = str(tmp_path / "ref")
        subprocess.run([O.REF_DRIVER, "ingest", mtx, str(seed), str(d), pre], check=True, capture_output=True)
        off, keys = O.read_csr(pre + ".csr")
        du, dw = O.read_deletions(pre + ".del")
        got = run_ingest(ingest_bin, mtx, seed, d, str(tmp_path / "out"))
        assert_same(got, dict(offsets=off, keys=keys, del_u=du, del_w=dw))


def test_minstd0_canonical_matches_libstdcxx(tmp_path):
    """include/nlp/random.hxx (the engine the device ingest draws from, its
    state exposed) equals std::default_random_engine +
    uniform_real_distribution<double>(0, 1) draw for draw."""
    src = tmp_path / "rt.cxx"
    src.write_text(r'''
#include "nlp/random.hxx"
#include <random>
#include <cstdio>
int main() {
  for (unsigned seed : {0u, 1u, 42u, 123456789u, 2147483647u, 4294967295u}) {
    std::default_random_engine a(seed);
    nlp::Minstd0 b(seed);
    std::uniform_real_distribution<> d(0.0, 1.0);
    for (int i = 0; i < 3000000; ++i)
      if (d(a) != nlp::canonical01(b)) { printf("differ: seed %u draw %d\n", seed, i); return 1; }
    if (a() != b()) return 2;
  }
  return 0;
}''')
    exe = str(tmp_path / "rt")
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), str(src), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout


def test_ingest_reads_a_pipe(ingest_bin, tmp_path):
    """a stream that cannot seek (a FIFO, as `<(zcat g.mtx.gz)` gives)
    is read to its end like the reference's ifstream (mtx.hxx:138), not taken
    for an empty graph."""
    g = dict(np.load(os.path.join(GOLDEN, "ingest_general.npz"), allow_pickle=False))
    fifo = str(tmp_path / "in.fifo")
    os.mkfifo(fifo)
    import threading

    def feed():
        with open(fifo, "wb") as f:
            f.write(g["mtx"].tobytes())

    th = threading.Thread(target=feed)
    th.start()
    got = run_ingest(ingest_bin, fifo, int(g["seed"][0]), float(g["d"][0]), str(tmp_path / "out"))
    th.join()
    assert_same(got, g)
