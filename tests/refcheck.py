"""Full-size parity against the REFERENCE ITSELF, for the
k-filling calls of the full-size stand-ins (tests/test_gpu_c3.py, c4.py).

TEST INFRASTRUCTURE: the reference's own predictLinks<Metric>Omp<H> runs as
oracle/_ref/ref_driver (compiled from /root/reference/inc by oracle/Makefile in
the build container; the binary travels) on the same CSR, written to /dev/shm.
The comparison runs on the GPU with torch (sets of 1e8+ links), never through
the library under test.

The reference's tie order depends on its OpenMP schedule (predict.hxx:287,
332, 437), so the contract is:
  1. the same number of links and the same score multiset, bitwise;
  2. the same set of links strictly above the k-th score;
  3. every link at the k-th score (ours and the reference's) is in the
     reference's own tie set -- ALL its candidates at that score, taken from a
     second reference call with maxEdges = |above| + |ties| + 1 (our count of
     links at or above the k-th score, plus one): that call must come back
     with a link below the k-th score (or with fewer links than asked, every
     candidate), which proves the tie set complete whatever our count was;
  4. F1 (main.cxx:48-57, 199-206) of both lies within the tie bounds: the
     r = k - |above| boundary links chosen from the tie set T to minimise /
     maximise the matches with the deletions.
and, for OUR output only (the canonical contract of this library, which the
parallel oracle restates): the r boundary links are the r smallest (u, w) of
the reference's tie set, and the list is in canonical order (score key desc,
u asc, w asc) -- together with 1-2, the output is the oracle's bit for bit.
"""
import json
import os
import subprocess
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
REF_THREADS = int(os.environ.get("NLP_REF_THREADS", os.environ.get("OMP_NUM_THREADS", "16")))


def have_ref():
    return os.path.exists(REF_DRIVER)


def write_csr(off, keys):
    """The CSR as ref_driver reads it ([span, nnz] u64, offsets u64, keys u32),
    in /dev/shm when present.  Returns (path, TemporaryDirectory)."""
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else None
    tmp = tempfile.TemporaryDirectory(dir=shm)
    path = os.path.join(tmp.name, "g.csr")
    with open(path, "wb") as f:
        np.array([len(off) - 1, len(keys)], np.uint64).tofile(f)
        np.asarray(off, np.uint64).tofile(f)
        np.asarray(keys, np.uint32).tofile(f)
    return path, tmp


def ref_predict(csr, metric, H, max_edges, threads=REF_THREADS, timeout=600):
    """predictLinks<Metric>Omp<H>(G, {1, max_edges}) of the reference on the CSR
    file: (u, w, score) numpy arrays and its own time (ms)."""
    fd, out = tempfile.mkstemp(dir=os.path.dirname(csr), suffix=".edges")
    os.close(fd)
    try:
        env = dict(os.environ, OMP_NUM_THREADS=str(threads))
        t0 = time.time()
        r = subprocess.run([REF_DRIVER, "predict", csr, str(metric), str(H), str(max_edges), "omp", str(threads), "1",
                            out], capture_output=True, text=True, env=env, timeout=timeout)
        wall = time.time() - t0
        assert r.returncode == 0, r.stderr[-500:]
        t_ms, ts_ms, n = r.stdout.split()
        raw = np.fromfile(out, dtype=np.uint32)
    finally:
        os.unlink(out)
    n = int(n)
    assert int(raw[:2].view(np.uint64)[0]) == n
    rec = raw[2:].reshape(n, 3)
    return rec[:, 0].copy(), rec[:, 1].copy(), rec[:, 2].copy().view(np.float32), \
        dict(time_ms=float(t_ms), wall_s=wall, n=n)


def _t(x, dev):
    import torch
    if isinstance(x, torch.Tensor):
        return x.to(dev)
    return torch.as_tensor(np.ascontiguousarray(x)).to(dev)


def keys_t(s):
    """Order-preserving u32 score key (parity.keys_of) as int64, on the device."""
    import torch
    s = s.clone()
    s[s == 0] = 0.0
    b = s.view(torch.int32).long() & 0xffffffff
    k = torch.where(b >= 0x80000000, 0xffffffff - b, b | 0x80000000)
    k[torch.isnan(s)] = 0
    return k


def pk(u, w):
    return (u.long() << 32) | w.long()


def gpu_links(out_t, n):
    """(u, w, score) device tensors of the first n links of an [N, 3] int32 output tensor."""
    o = out_t[:n]
    return o[:, 0].long() & 0xffffffff, o[:, 1].long() & 0xffffffff, o[:, 2].contiguous().view(__import__("torch").float32)


def check_contract(gpu, ref_k, ref_ge, k, del_u, del_w, dev="cuda", asked=None):
    """Contract 1-4 of the module docstring.  gpu = device tensors (u, w, s);
    ref_k, ref_ge = numpy (u, w, s) of the reference's maxEdges = k call and
    of its tie-set call, which asked for `asked` links (None: ref_ge is the
    exact set at or above the k-th score, as the CPU fixtures cut it); del_u /
    del_w = the directed deletions (both directions).  Returns the numbers of
    the check."""
    import torch
    gu, gw, gs = gpu
    eu, ew, es = (_t(x, dev) for x in ref_ge[:3])
    eu, ew = (x.long() & 0xffffffff for x in (eu, ew))
    n = gu.numel()
    gk, ek = keys_t(gs), keys_t(es)
    assert not torch.isnan(es).any(), "NaN scores: the reference's order is undefined (SURVEY A.4)"
    if ref_k is not None:
        ru, rw, rs = (_t(x, dev) for x in ref_k[:3])
        ru, rw = (x.long() & 0xffffffff for x in (ru, rw))
        rk = keys_t(rs)
        assert ru.numel() == n, ("link counts differ", ru.numel(), n)
    else:
        # one reference call (the tie-set call): its top n scores are the reference's
        # top-n multiset whatever ties its own k-call would pick; its own k-call's
        # F1 is then not reported (common_ref None)
        assert asked is not None, "a single reference call must be the tie-set call"
        order = torch.argsort(ek, descending=True)[:n]
        ru, rw, rk = eu[order], ew[order], ek[order]
        assert ru.numel() == n, ("link counts differ", ru.numel(), n)
    assert torch.equal(torch.sort(gk).values, torch.sort(rk).values), "score multisets differ"
    kth = int(rk.min())
    ga = torch.sort(pk(gu, gw)[gk > kth]).values
    ra = torch.sort(pk(ru, rw)[rk > kth]).values
    assert torch.equal(ga, ra), "above-boundary sets differ (%d vs %d)" % (ga.numel(), ra.numel())
    # the reference's whole tie set at the k-th score
    if asked is not None:
        # asked = our count at or above the k-th score + 1: a complete set leaves room for one link below it
        assert ek.numel() < asked or int(ek.min()) < kth, \
            "the reference has more links at or above the k-th score than our output: a candidate was lost"
        keep = ek >= kth
        eu, ew, es, ek = eu[keep], ew[keep], es[keep], ek[keep]
    assert int(ek.min()) >= kth, "the tie-set call returned links below the k-th score"
    ea = torch.sort(pk(eu, ew)[ek > kth]).values
    assert torch.equal(ea, ra), "the two reference calls disagree above the k-th score"
    T = torch.sort(pk(eu, ew)[ek == kth]).values
    assert torch.unique(T).numel() == T.numel()
    gt = pk(gu, gw)[gk == kth]
    rt = pk(ru, rw)[rk == kth]
    assert bool(torch.isin(gt, T).all()), "tie links outside the reference's tie set"
    assert bool(torch.isin(rt, T).all()), "the reference's own ties outside its tie set"
    assert torch.unique(pk(gu, gw)).numel() == n, "duplicate links in the output"
    # canonical: the boundary links are the smallest (u, w) of T, the list in canonical order
    assert torch.equal(torch.sort(gt).values, T[:gt.numel()]), "boundary links are not the first ties in (u, w) order"
    if n > 1:
        dk, dp = gk[1:] - gk[:-1], pk(gu, gw)[1:] - pk(gu, gw)[:-1]
        assert bool(((dk < 0) | ((dk == 0) & (dp > 0))).all()), "output not in canonical order"
    # F1 (main.cxx:48-57): both directions of every link against the directed deletions
    D = torch.sort(pk(_t(del_u, dev).long() & 0xffffffff, _t(del_w, dev).long() & 0xffffffff)).values

    def contrib(u, w):  # per link: how many of (u, w), (w, u) are deletions
        return torch.isin(pk(u, w), D).long() + torch.isin(pk(w, u), D).long()

    def common(u, w):
        return int(contrib(u, w).sum())

    r = n - ga.numel()
    ca = common(ga >> 32, ga & 0xffffffff)
    ct = torch.sort(contrib(T >> 32, T & 0xffffffff)).values
    lo = ca + int(ct[:r].sum())
    hi = ca + int(ct[ct.numel() - r:].sum()) if r > 0 else ca
    cg = common(gu, gw)
    cr = common(ru, rw) if ref_k is not None else None
    assert lo <= cg <= hi, ("our matches outside the tie bounds", lo, cg, hi)
    assert cr is None or lo <= cr <= hi, ("the reference's matches outside the tie bounds", lo, cr, hi)
    nd = int(D.numel())

    def f1(c):
        p, rc = c / max(2 * n, 1), c / max(nd, 1)
        return 0.0 if p + rc == 0 else 2 * p * rc / (p + rc)

    return dict(k=k, n=n, kth_key=kth, above=int(ga.numel()), ties_total=int(T.numel()), ties_taken=r,
                common_gpu=cg, common_ref=cr, common_lo=lo, common_hi=hi,
                f1_gpu=f1(cg), f1_ref=f1(cr) if cr is not None else None, f1_lo=f1(lo), f1_hi=f1(hi),
                precision_gpu=cg / max(2 * n, 1), recall_gpu=cg / max(nd, 1))


def run_reference_check(c, csr, metric, H, name, single=False):
    """The whole check for one call on a bigconf.Config: our k-call, the
    reference's k-call, the count of candidates at or above the k-th score (our
    top-2k call), the reference's call with that many links, the contract.
    Writes one JSON line to $NLP_TEST_REPORT_DIR/refcheck.jsonl when set."""
    import torch
    out = c.out()
    n, t = c.G.predict_device(metric, H, c.k, out)
    gpu = gpu_links(out, n)
    kth = int(keys_t(gpu[2]).min()) if n else 0
    # how many candidates score >= the k-th score: our canonical top-m for a
    # growing m, with minScore one float below the k-th score (predict.hxx:311:
    # only scores above it are candidates), until the list stops short of m (it
    # then holds every candidate at or above the k-th score) -- the call keeps
    # no candidate below the k-th, so its buffers stay near k (the top-2k call
    # without the floor ran out of HBM on C4 AA H = 32's 6.6e9 candidates)
    s_k = float(gpu[2].min()) if n else 0.0
    floor = float(np.nextafter(np.float32(s_k), np.float32(-np.inf)))
    torch.cuda.empty_cache()
    m = min(int(t["candidates"]), c.k + c.k // 4 + 1)
    while True:
        out2 = c.out(m)
        n2, _ = c.G.predict_device(metric, H, m, out2, min_score=floor)
        k2 = keys_t(gpu_links(out2, n2)[2])
        n_ge = int((k2 >= kth).sum())
        assert n_ge == n2, "the minScore floor let a candidate below the k-th score through"
        if n2 < m or m >= int(t["candidates"]):
            break
        del out2, k2
        torch.cuda.empty_cache()
        m = min(int(t["candidates"]), 2 * m)
    del out2, k2
    torch.cuda.empty_cache()
    # single: only the tie-set call (the reference's top-n multiset and above-set
    # come from it) -- half the reference time for the long calls
    ref_k = None if single else ref_predict(csr, metric, H, c.k)
    ref_ge = ref_predict(csr, metric, H, n_ge + 1)
    res = check_contract(gpu, ref_k, ref_ge, c.k, c.del_u, c.del_w, asked=n_ge + 1)
    res.update(config=name, metric=metric, H=H, candidates=int(t["candidates"]), wedges=int(t["wedges"]), path=t["path"],
               chunks=int(t["chunks"]), order_route=int(t.get("order_route", 0)),
               ref_threads=REF_THREADS, ref_time_ms=ref_k[3]["time_ms"] if ref_k else None,
               ref_ge_time_ms=ref_ge[3]["time_ms"],
               gpu_ms=t["total_ms"])
    rd = os.environ.get("NLP_TEST_REPORT_DIR")
    if rd:
        os.makedirs(rd, exist_ok=True)
        with open(os.path.join(rd, "refcheck.jsonl"), "a") as f:
            f.write(json.dumps(res) + "\n")
    return res
