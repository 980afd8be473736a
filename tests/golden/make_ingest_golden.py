"""Golden fixtures for the host ingest (include/nlp/ingest.hxx) from the REAL
reference's ingest (oracle/_ref/ref_driver ingest: readMtxOmpW -> symmetrizeOmp
-> removeSelfLoopsOmpU -> generateEdgeDeletions(default_random_engine(seed)) ->
tidyBatchUpdateU -> applyBatchUpdateOmpU, main.cxx:164-169, 241-245).

Runs only in the build container.  Each ingest_<name>.npz holds data only: the
MatrixMarket input text (uint8), the seed and deletion fraction, and the
reference's outputs (CSR after the deletions, directed sorted deletions).

    python tests/golden/make_ingest_golden.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)
import pyoracle as O  # noqa: E402
from make_golden import chung_lu_mtx  # noqa: E402


def sym_mtx(path, n, m, seed):
    """Symmetric-header pattern file with self-loops and repeated lines."""
    rng = np.random.default_rng(seed)
    a = rng.integers(1, n + 1, m)
    b = rng.integers(1, n + 1, m)
    lines = ["%d %d" % (max(x, y), min(x, y)) for x, y in zip(a.tolist(), b.tolist())]
    lines += lines[: m // 20]  # repeated lines
    lines += ["%d %d" % (i, i) for i in range(1, n + 1, 7)]  # self-loops
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate pattern symmetric\n% a comment line\n")
        f.write("%d %d %d\n" % (n, n, len(lines)))
        f.write("\n".join(lines) + "\n")


CASES = {
    # name: (maker, seed, d)
    "general": (lambda p: chung_lu_mtx(p, 2000, 12000, 0.8, 3), 7, 0.05),
    "sym": (lambda p: sym_mtx(p, 500, 3000, 5), 11, 0.1),
    "d0": (lambda p: chung_lu_mtx(p, 300, 1200, 0.6, 1), 42, 0.0),
}


def main():
    if not os.path.exists(O.REF_DRIVER):
        sys.exit("build the reference driver first: make -C oracle")
    with tempfile.TemporaryDirectory() as tmp:
        for name, (maker, seed, d) in CASES.items():
            mtx = os.path.join(tmp, name + ".mtx")
            maker(mtx)
            pre = os.path.join(tmp, name)
            subprocess.run([O.REF_DRIVER, "ingest", mtx, str(seed), str(d), pre], check=True, capture_output=True)
            off, keys = O.read_csr(pre + ".csr")
            du, dw = O.read_deletions(pre + ".del")
            text = np.frombuffer(open(mtx, "rb").read(), np.uint8)
            np.savez_compressed(os.path.join(HERE, "ingest_%s.npz" % name), mtx=text, seed=np.array([seed]),
                                d=np.array([d]), offsets=off, keys=keys, del_u=du, del_w=dw)
            print(name, "span", len(off) - 1, "nnz", len(keys), "deletions", len(du))


if __name__ == "__main__":
    main()
