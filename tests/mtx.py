"""MatrixMarket coordinate text -> the directed pairs readMtxOmpW feeds the
graph (mtx.hxx:39-54, 119-135): comment lines skipped, the banner's
symmetric / skew-symmetric adding the reverse of every line, the size line
giving n = max(rows, cols).  Test helper (the host restatement of the whole
read is include/nlp/ingest.hxx readMtx)."""
import numpy as np


def parse_mtx(text):
    if isinstance(text, (bytes, bytearray)):
        text = text.decode()
    lines = text.splitlines()
    symmetric = False
    i = 0
    while i < len(lines) and lines[i].startswith("%"):
        h = lines[i].split()
        if lines[i].startswith("%%") and len(h) >= 5:
            symmetric = h[4] in ("symmetric", "skew-symmetric")
        i += 1
    rows, cols, _ = (int(x) for x in lines[i].split()[:3])
    n = max(rows, cols)
    body = [ln.split() for ln in lines[i + 1:] if ln.strip()]
    u = np.array([int(b[0]) for b in body], np.uint32)
    v = np.array([int(b[1]) for b in body], np.uint32)
    if symmetric:
        u, v = np.concatenate([u, v]), np.concatenate([v, u])
    return u, v, n, symmetric
