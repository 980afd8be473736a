"""ctypes wrapper of oracle/libnlp_oracle.so plus file readers for the oracle's
binary formats.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libnlp_oracle.so")
REF_DRIVER = os.path.join(HERE, "_ref", "ref_driver")

METRICS = ["CN", "JAC", "SOR", "SAL", "HPI", "HDI", "LHN", "AA", "RA"]

_lib = None


def build():
    """Compile the C restatement (and, where /root/reference exists, the reference driver)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.nlpo_predict_range.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32,
            ctypes.c_float, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, u64p, u64p, u64p, u64p, u64p]
        L.nlpo_predict_range.restype = ctypes.c_int
        L.nlpo_predict_range2.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
            ctypes.c_float, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, u64p, u64p, u64p, u64p, u64p]
        L.nlpo_predict_range2.restype = ctypes.c_int
        L.nlpo_predict_par.argtypes = [
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
            ctypes.c_float, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.nlpo_predict_par.restype = ctypes.c_int
        L.nlpo_edge_hash.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float]
        L.nlpo_edge_hash.restype = ctypes.c_uint64
        L.nlpo_score_key.argtypes = [ctypes.c_float]
        L.nlpo_score_key.restype = ctypes.c_uint32
        L.nlpo_wedges_gt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]
        L.nlpo_wedges_gt.restype = ctypes.c_uint64
        _lib = L
    return _lib


def predict(offsets, keys, metric, hub, max_edges=None, min_score=0.0, u_begin=0, u_end=None, maxfactor2=0):
    """Canonical top-k from the C restatement (maxfactor2: the reference's
    MAXFACTOR2 template parameter, predict.hxx:221,295).

    Returns (u, w, score, info) with info = dict(candidates, nan, wedges, wedges_gt):
    wedges = all (u, v, w) the reference scans, wedges_gt = those with w > u."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    span = len(offsets) - 1
    if u_end is None:
        u_end = span
    if isinstance(metric, str):
        metric = METRICS.index(metric)
    L = lib()
    ncand, nnan, nw, nwg, cnt = (ctypes.c_uint64() for _ in range(5))
    if max_edges is None:
        # first pass: count, so the output buffer can be sized exactly
        rc = L.nlpo_predict_range2(offsets.ctypes.data, keys.ctypes.data, span, metric, hub, maxfactor2,
                                   min_score, 0, u_begin, u_end, None, None, None,
                                  ctypes.byref(cnt), ctypes.byref(ncand), ctypes.byref(nnan),
                                  ctypes.byref(nw), ctypes.byref(nwg))
        if rc:
            raise MemoryError("oracle allocation failed")
        max_edges = ncand.value
    cap = max(int(max_edges), 1)
    ou = np.empty(cap, np.uint32)
    ow = np.empty(cap, np.uint32)
    os_ = np.empty(cap, np.float32)
    rc = L.nlpo_predict_range2(offsets.ctypes.data, keys.ctypes.data, span, metric, hub, maxfactor2, min_score,
                               int(max_edges), u_begin, u_end, ou.ctypes.data, ow.ctypes.data,
                              os_.ctypes.data, ctypes.byref(cnt), ctypes.byref(ncand),
                              ctypes.byref(nnan), ctypes.byref(nw), ctypes.byref(nwg))
    if rc:
        raise MemoryError("oracle allocation failed")
    n = cnt.value
    info = dict(candidates=ncand.value, nan=nnan.value, wedges=nw.value, wedges_gt=nwg.value)
    return ou[:n].copy(), ow[:n].copy(), os_[:n].copy(), info


def predict_par(offsets, keys, metric, hub, max_edges=None, min_score=0.0, u_begin=0, u_end=None, maxfactor2=0,
                threads=0, arrays=True):
    """The same canonical top-k as predict(), computed by nlpo_predict_par (OpenMP
    over source chunks, four passes, nothing stored beyond the kept set): for
    the full-size configs.  arrays=False returns no edges, only the counts and
    the order-free digest of the kept set (info["digest"] = (sum, xor) of
    nlpo_edge_hash, compare with edge_digest())."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    span = len(offsets) - 1
    if u_end is None:
        u_end = span
    if isinstance(metric, str):
        metric = METRICS.index(metric)
    me = (1 << 64) - 1 if max_edges is None else int(max_edges)
    L = lib()
    stats = np.zeros(8, np.uint64)
    if arrays:
        if max_edges is None:  # size the buffers from a counting run
            rc = L.nlpo_predict_par(offsets.ctypes.data, keys.ctypes.data, span, metric, hub, maxfactor2,
                                    min_score, 0, u_begin, u_end, threads, None, None, None, stats.ctypes.data)
            if rc:
                raise MemoryError("oracle allocation failed")
            me = int(stats[1])
        cap = max(me, 1)
        ou, ow, os_ = np.empty(cap, np.uint32), np.empty(cap, np.uint32), np.empty(cap, np.float32)
        ptrs = (ou.ctypes.data, ow.ctypes.data, os_.ctypes.data)
    else:
        ptrs = (None, None, None)
    rc = L.nlpo_predict_par(offsets.ctypes.data, keys.ctypes.data, span, metric, hub, maxfactor2, min_score, me,
                            u_begin, u_end, threads, *ptrs, stats.ctypes.data)
    if rc:
        raise MemoryError("oracle allocation failed")
    n = int(stats[0])
    info = dict(candidates=int(stats[1]), nan=int(stats[2]), wedges=int(stats[3]), wedges_gt=int(stats[4]),
                kth_key=int(stats[5]), digest=(int(stats[6]), int(stats[7])), count=n)
    if not arrays:
        return None, None, None, info
    return ou[:n].copy(), ow[:n].copy(), os_[:n].copy(), info


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def edge_digest(u, w, s, chunk=1 << 24):
    """(sum, xor) of nlpo_edge_hash over the links (u, w, score): the order-free
    digest predict_par reports (uint64 wrapping arithmetic)."""
    tot, x = np.uint64(0), np.uint64(0)
    with np.errstate(over="ignore"):
        for i in range(0, len(u), chunk):
            uu = np.asarray(u[i:i + chunk], np.uint64)
            ww = np.asarray(w[i:i + chunk], np.uint64)
            ss = np.asarray(s[i:i + chunk], np.float32)
            b = ss.view(np.uint32).astype(np.uint64)
            b[np.isnan(ss)] = np.uint64(0x7fc00000)
            h = _mix64(((uu << np.uint64(32)) | ww) ^ (b * np.uint64(0x9E3779B97F4A7C15)))
            tot = tot + h.sum(dtype=np.uint64)
            x = x ^ np.bitwise_xor.reduce(h) if len(h) else x
    return int(tot), int(x)


def score_keys(scores):
    """Vectorised nlpo_score_key: order-preserving float -> uint32, NaN -> 0."""
    s = np.asarray(scores, dtype=np.float32).copy()
    s[s == 0] = 0.0  # -0 -> +0
    b = s.view(np.uint32)
    k = np.where(b & 0x80000000, ~b, b | 0x80000000).astype(np.uint32)
    k[np.isnan(s)] = 0
    return k


def read_csr(path):
    with open(path, "rb") as f:
        S, M = np.frombuffer(f.read(16), np.uint64)
        off = np.frombuffer(f.read(8 * (int(S) + 1)), np.uint64).copy()
        keys = np.frombuffer(f.read(4 * int(M)), np.uint32).copy()
    return off, keys


def write_csr(path, offsets, keys):
    with open(path, "wb") as f:
        np.array([len(offsets) - 1, len(keys)], np.uint64).tofile(f)
        np.asarray(offsets, np.uint64).tofile(f)
        np.asarray(keys, np.uint32).tofile(f)


def read_edges(path):
    """u64 n, then n x {u32 u, u32 w, f32 score} (ref_driver predict output)."""
    with open(path, "rb") as f:
        n = int(np.frombuffer(f.read(8), np.uint64)[0])
        rec = np.frombuffer(f.read(12 * n), np.uint32).reshape(n, 3) if n else np.zeros((0, 3), np.uint32)
    return rec[:, 0].copy(), rec[:, 1].copy(), rec[:, 2].copy().view(np.float32)


def read_deletions(path):
    with open(path, "rb") as f:
        n = int(np.frombuffer(f.read(8), np.uint64)[0])
        p = np.frombuffer(f.read(8 * n), np.uint32).reshape(n, 2)
    return p[:, 0].copy(), p[:, 1].copy()


def ref_predict(csr_path, metric, hub, max_edges=-1, mode="seq", threads=1, repeat=1, out=None, maxfactor2=0):
    """Run the compiled reference (oracle/_ref/ref_driver) -- only where it exists."""
    if isinstance(metric, str):
        metric = METRICS.index(metric)
    out = out or csr_path + ".pred.%d.%d.%s" % (metric, hub, mode)
    r = subprocess.run([REF_DRIVER, "predict", csr_path, str(metric), str(hub), str(max_edges), mode,
                        str(threads), str(repeat), out, str(maxfactor2)], check=True, capture_output=True, text=True)
    t, ts, n = r.stdout.split()
    u, w, s = read_edges(out)
    return u, w, s, dict(time_ms=float(t), scoring_ms=float(ts))


def wedges_gt(offsets, keys, hub, u_begin, u_end, threads=0):
    """Wedges (u, v, w), w > u, of the sources [u_begin, u_end) (nlpo_wedges_gt:
    one binary search of N(v) per (u, v) entry, predict.hxx:284-304)."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    return int(lib().nlpo_wedges_gt(offsets.ctypes.data, keys.ctypes.data, len(offsets) - 1, hub, u_begin, u_end,
                                    threads))
