"""Generate the golden fixtures in tests/golden/ from the REAL reference.

Runs only in the build container (needs /root/reference and oracle/_ref/ref_driver,
built by `make -C oracle`).  The fixtures are data: inputs (CSR after the
reference's own ingest + deletions, or hand-made CSRs) and the reference's
outputs.  Nothing from the reference's sources is stored.

    python tests/golden/make_golden.py

Per graph file <name>.npz:
    offsets, keys           the adjacency the reference predicted on (multiset rows)
    del_u, del_w            directed sorted unique deletions (main.cxx `deletions0`)
    k                       maxEdges = len(deletions0) // 2       (main.cxx:50)
    cand_<m>_<H>_{u,w,s}    every candidate, predictLinks<M><H>(y, {1, SIZE_MAX})
                            (sequential reference, predict.hxx:358-374)
    topk_<m>_<H>_{u,w,s}    predictLinks<M>Omp<H>(y, {1, k}) with 4 threads when the
                            candidates >= k (OpenMP path, predict.hxx:409-467);
                            otherwise the sequential reference with {1, k}
                            (the OpenMP merge is UB there)
    topk_<m>_<H>_omp        1 if topk came from the OpenMP path (0 also when the OpenMP
                            run crashed on NaN scores, A.2/A.4)

maxf2.npz (python tests/golden/make_golden.py maxf2): the MAXFACTOR2 template
parameter (predict.hxx:221,295) on the g300 and edge graphs of the files above:
    <graph>_cand_<F>_<m>_<H>_{u,w,s}   predictLinks<M><H, F>(y, {1, SIZE_MAX})
    <graph>_topk_<F>_<m>_<H>_{u,w,s}   predictLinks<M>Omp<H, F>(y, {1, k}) (sequential
                                       when the candidates < k, as above)
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as O  # noqa: E402


def chung_lu_mtx(path, n, m, alpha, seed):
    """Small Chung-Lu power-law graph as a 1-based 'general' MatrixMarket file."""
    rng = np.random.default_rng(seed)
    w = np.arange(1, n + 1, dtype=np.float64) ** (-alpha)
    p = np.cumsum(w)
    p /= p[-1]
    perm = rng.permutation(n) + 1
    keys = set()
    while len(keys) < m:
        u = perm[np.searchsorted(p, rng.random(m))]
        v = perm[np.searchsorted(p, rng.random(m))]
        for a, b in zip(u.tolist(), v.tolist()):
            if a != b and len(keys) < m:
                keys.add((a, b))
    E = sorted(keys)
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate pattern general\n")
        f.write("%d %d %d\n" % (n, n, len(E)))
        for a, b in E:
            f.write("%d %d\n" % (a, b))


def edge_case_csr():
    """Hand-made CSR exercising the reference's corner cases (not produced by
    its ingest): duplicate entries, asymmetric edges to degree-0 vertices
    (Salton/LHN/HubPromoted +inf, NaN after first-order exclusion), the
    Jaccard size_t wrap (du + dw - c < 0), degree-1 intermediates (Adamic-Adar
    1/log(1) = +inf), an empty row 0 and isolated vertices."""
    rows = {
        1: [2, 3, 3, 9],
        2: [1, 4, 5],
        3: [1, 1, 4, 6],
        4: [2, 3, 7, 7, 7, 11],
        5: [2, 8],
        6: [3],
        7: [4, 11],
        8: [5, 10, 10, 10],
        9: [12],
        10: [],
        11: [],
        12: [9],
        13: [14],
        14: [13, 15],
        15: [14],
        16: [],
    }
    span = 17
    off = [0]
    keys = []
    for u in range(span):
        keys += sorted(rows.get(u, []))
        off.append(len(keys))
    return np.array(off, np.uint64), np.array(keys, np.uint32)


CASES_H = {
    "g300": [0, 1, 2, 3, 4, 8, 64],
    "g3k": [2, 4, 8],
    "edge": [0, 1, 2, 3, 4, 8],
}
TOPK_ONLY_H = {"g3k": [0, 64]}


def run_graph(name, csr_path, off, keys, dels, tmp):
    k = len(dels[0]) // 2
    out = dict(offsets=off, keys=keys, del_u=dels[0], del_w=dels[1], k=np.array([k], np.int64))
    hs = CASES_H[name] + TOPK_ONLY_H.get(name, [])
    for m in range(9):
        for H in hs:
            ncand = None
            if H in CASES_H[name]:
                u, w, s, _ = O.ref_predict(csr_path, m, H, -1, "seq", 1, 1, os.path.join(tmp, "p.bin"))
                out["cand_%d_%d_u" % (m, H)], out["cand_%d_%d_w" % (m, H)], out["cand_%d_%d_s" % (m, H)] = u, w, s
                ncand = len(u)
            if ncand is None:
                # candidate count from the restatement is only used to pick the path
                ncand = O.predict(off, keys, m, H)[3]["candidates"]
            omp = ncand >= k and k > 0
            try:
                u, w, s, _ = O.ref_predict(csr_path, m, H, k, "omp" if omp else "seq", 4, 1,
                                           os.path.join(tmp, "t.bin"))
            except subprocess.CalledProcessError:
                # NaN scores break the OpenMP heaps and the merge then
                # reads past an empty per-thread list (A.2): the reference crashes.
                # Record the sequential reference instead.
                omp = False
                u, w, s, _ = O.ref_predict(csr_path, m, H, k, "seq", 1, 1, os.path.join(tmp, "t.bin"))
            out["topk_%d_%d_u" % (m, H)], out["topk_%d_%d_w" % (m, H)], out["topk_%d_%d_s" % (m, H)] = u, w, s
            out["topk_%d_%d_omp" % (m, H)] = np.array([int(omp)], np.int8)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, "span", len(off) - 1, "nnz", len(keys), "k", k, flush=True)


MAXF2_CASES = {"g300": ([1, 2, 4], [0, 4]), "edge": ([1, 2], [0, 4])}


def make_maxf2():
    """MAXFACTOR2 fixtures on the committed g300 / edge graphs (their CSR and k)."""
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, (fs, hs) in MAXF2_CASES.items():
            g = dict(np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False))
            csr = os.path.join(tmp, name + ".csr")
            O.write_csr(csr, g["offsets"], g["keys"])
            k = int(g["k"][0])
            for F in fs:
                for m in range(9):
                    for H in hs:
                        tag = "%s_%%s_%d_%d_%d" % (name, F, m, H)
                        u, w, s_, _ = O.ref_predict(csr, m, H, -1, "seq", 1, 1, os.path.join(tmp, "p.bin"), F)
                        out[tag % "cand" + "_u"], out[tag % "cand" + "_w"], out[tag % "cand" + "_s"] = u, w, s_
                        omp = len(u) >= k and k > 0
                        try:
                            u, w, s_, _ = O.ref_predict(csr, m, H, k, "omp" if omp else "seq", 4, 1,
                                                        os.path.join(tmp, "t.bin"), F)
                        except subprocess.CalledProcessError:
                            u, w, s_, _ = O.ref_predict(csr, m, H, k, "seq", 1, 1, os.path.join(tmp, "t.bin"), F)
                        out[tag % "topk" + "_u"], out[tag % "topk" + "_w"], out[tag % "topk" + "_s"] = u, w, s_
    np.savez_compressed(os.path.join(HERE, "maxf2.npz"), **out)
    print("maxf2", len(out) // 6, "cases", flush=True)


def main():
    if not os.path.exists(O.REF_DRIVER):
        sys.exit("build the reference driver first: make -C oracle")
    if len(sys.argv) > 1 and sys.argv[1] == "maxf2":
        make_maxf2()
        return
    with tempfile.TemporaryDirectory() as tmp:
        for name, (n, m, alpha, seed, d, dseed) in {"g300": (300, 1200, 0.6, 1, 0.1, 42),
                                                   "g3k": (3000, 20000, 0.6, 7, 0.1, 42)}.items():
            mtx = os.path.join(tmp, name + ".mtx")
            chung_lu_mtx(mtx, n, m, alpha, seed)
            pre = os.path.join(tmp, name)
            subprocess.run([O.REF_DRIVER, "ingest", mtx, str(dseed), str(d), pre], check=True,
                           capture_output=True)
            off, keys = O.read_csr(pre + ".csr")
            dels = O.read_deletions(pre + ".del")
            run_graph(name, pre + ".csr", off, keys, dels, tmp)
        off, keys = edge_case_csr()
        p = os.path.join(tmp, "edge.csr")
        O.write_csr(p, off, keys)
        dels = (np.array([1, 2, 3, 4], np.uint32), np.array([2, 1, 4, 3], np.uint32))
        run_graph("edge", p, off, keys, dels, tmp)


if __name__ == "__main__":
    main()
