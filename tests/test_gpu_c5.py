"""BASELINE configs[4] / SURVEY §8(d) C5: the sk-2005-shaped stand-in with
0.01|E| removed, IHub (no hub cutoff) Common Neighbours -- the worst-case
intersection stress.  The whole call scans sum_v deg(v)^2 ~ 1e14 wedges: it is
an 8-GPU config (hours on one GPU), so here a bounded source range goes
through the HIP path (path 4, the hash accumulation) and is checked exactly
against the parallel oracle, plus size-independent properties: canonical
order, the wedge / candidate counters, and shard-merge equality (the range
split in two, each half predicted and merged by nlp_merge_blocks_device ==
the single-range result).  The full-call time is extrapolated from the
measured wedge rate (reported, not asserted)."""
import json
import os
import time

import numpy as np
import pytest

from bigconf import ORACLE_THREADS, Config
from parity import assert_canonical_equal, assert_canonical_order

pytestmark = pytest.mark.gpu

RANGE_WEDGES = 1.5e9  # wedges (all w, IHub) of the checked source range


@pytest.fixture(scope="module")
def c5(nlp):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = Config(nlp, "C5-sk-2005-ihub")
    # per-source IHub work W(u) = sum_{v in N(u)} deg(v), chunked on the device
    off, keys = c.off_t, c.keys_t
    deg = (off[1:] - off[:-1])
    m = keys.numel()
    pref = torch.zeros(m + 1, dtype=torch.int64, device=keys.device)
    carry = torch.zeros((), dtype=torch.int64, device=keys.device)
    for b in range(0, m, 1 << 27):
        e = min(m, b + (1 << 27))
        pref[b + 1:e + 1] = torch.cumsum(deg[keys[b:e].long()], 0) + carry
        carry = pref[e]
    W = (pref[off[1:]] - pref[off[:-1]]).cpu().numpy()
    del pref
    span = len(W)
    ua = span // 3
    cum = np.cumsum(W[ua:].astype(np.float64))
    ub = ua + int(np.searchsorted(cum, RANGE_WEDGES)) + 1
    c.range = (ua, min(ub, span))
    c.range_wedges = int(W[ua:ub].sum())
    c.total_wedges = int(np.sum(deg.double().cpu().numpy() ** 2))
    yield c
    c.close()


@pytest.mark.timeout(300)
def test_gpu_c5_ihub_range_vs_oracle(c5, oracle):
    ua, ub = c5.range
    out = c5.out()
    c5.G.predict_device(0, 0, c5.k, out, ua, ub)  # warm
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n, t = c5.G.predict_device(0, 0, c5.k, out, ua, ub)
    ms = (time.perf_counter() - t0) * 1e3
    assert t["path"] == 4
    u, w, s = c5.nlp.edges_from_tensor(out, n)
    eu, ew, es, oi = oracle.predict_par(c5.off, c5.keys, 0, 0, max_edges=c5.k, u_begin=ua, u_end=ub,
                                        threads=ORACLE_THREADS)
    assert_canonical_equal(eu, ew, es, u, w, s)
    assert_canonical_order(u, w, s)
    assert t["wedges"] == oi["wedges_gt"] and t["candidates"] == oi["candidates"]
    assert np.all((u >= ua) & (u < ub))
    # extrapolation of the full IHub call from this range's wedge rate (all wedges w > u: about half)
    rate = oi["wedges_gt"] / (ms * 1e-3)
    rep = dict(config="C5-sk-2005-ihub", range=[ua, ub], sources=ub - ua, range_wedges_gt=oi["wedges_gt"],
               range_candidates=oi["candidates"], predicted=n, gpu_ms=ms, wedges_per_s=rate,
               total_wedges_all=c5.total_wedges,
               full_call_estimate_s_1gpu=0.5 * c5.total_wedges / rate,
               full_call_estimate_s_8gpu=0.5 * c5.total_wedges / rate / 8)
    print(json.dumps(rep))
    d = os.environ.get("NLP_TEST_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "c5_range.json"), "w") as f:
            json.dump(rep, f)


@pytest.mark.timeout(300)
def test_gpu_c5_ihub_shards_merge_to_the_range_result(c5):
    import torch
    ua, ub = c5.range
    k = c5.k
    whole = c5.out()
    n, _ = c5.G.predict_device(0, 0, k, whole, ua, ub)
    mid = (ua + ub) // 2
    parts = []
    for a, b in ((ua, mid), (mid, ub)):
        blk = c5.out(k + 1)
        m, _ = c5.G.predict_device(0, 0, k, blk[1:], a, b)
        h = np.array([m & 0xFFFFFFFF, m >> 32, 0x4E4C5042], np.uint32).view(np.int32)
        blk[0] = torch.from_numpy(h).cuda()
        parts.append((blk, m))
    stride = max(m for _, m in parts) + 1
    blocks = torch.stack([b[:stride] for b, _ in parts])
    merged = c5.out()
    km = c5.G.merge_blocks_device(blocks, k, merged)
    assert km == n
    assert torch.equal(merged[:n], whole[:n])


@pytest.mark.timeout(600)
def test_gpu_c5_heaviest_shard_leading_wedges(c5, oracle):
    """The leading 1 % of the wedges of shard 0 of the 8 wedge-balanced shards
    of the whole call (dist.shard_ranges over dist.source_weights: the lowest
    ids, whose sources see the most w > u) -- ~5e10 wedges, far beyond what the
    oracle can score, so size-independent properties: the canonical order, every
    link in the range, the wedge counter equal to the exact count of w > u
    wedges (oracle.wedges_gt: one binary search of N(v) per (u, v) entry,
    predict.hxx:284-304), and the range split at its middle weight, the halves
    predicted and merged by nlp_merge_blocks_device, equal to the whole."""
    import torch
    import nlp_loader
    dmod = nlp_loader.load_sub("dist")
    span = len(c5.off) - 1
    w = dmod.source_weights(c5.off_t, c5.keys_t, 0)
    ranges = dmod.shard_ranges(span, 8, w)
    ua, ub = ranges[0]
    cw = torch.cumsum(torch.as_tensor(w, dtype=torch.float64).cpu()[ua:ub], 0)
    ub1 = ua + int(torch.searchsorted(cw, 0.01 * float(cw[-1]))) + 1
    mid = ua + int(torch.searchsorted(cw, 0.005 * float(cw[-1]))) + 1
    k = c5.k
    whole = c5.out()
    n, t = c5.G.predict_device(0, 0, k, whole, ua, ub1)
    u, ww, s = c5.nlp.edges_from_tensor(whole, n)
    assert t["path"] == 4 and n > 0
    assert_canonical_order(u, ww, s)
    assert np.all((u >= ua) & (u < ub1))
    exact = oracle.wedges_gt(c5.off, c5.keys, 0, ua, ub1, threads=ORACLE_THREADS)
    assert t["wedges"] == exact, (t["wedges"], exact)
    assert t["wedges"] >= 0.005 * 3.9e13 / 8  # about 1 % of a shard of the whole call's ~3.9e13
    parts = []
    for a, b in ((ua, mid), (mid, ub1)):
        blk = c5.out(k + 1)
        m, tm = c5.G.predict_device(0, 0, k, blk[1:], a, b)
        h = np.array([m & 0xFFFFFFFF, m >> 32, 0x4E4C5042], np.uint32).view(np.int32)
        blk[0] = torch.from_numpy(h).cuda()
        parts.append((blk, m, tm["wedges"]))
    assert parts[0][2] + parts[1][2] == t["wedges"]
    stride = max(m for _, m, _ in parts) + 1
    blocks = torch.stack([b[:stride] for b, _, _ in parts])
    merged = c5.out()
    km = c5.G.merge_blocks_device(blocks, k, merged)
    assert km == n
    assert torch.equal(merged[:n], whole[:n])
    d = os.environ.get("NLP_TEST_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "c5_shard0_leading.json"), "w") as f:
            json.dump(dict(shard0=[ua, ub], leading=[ua, ub1], wedges=t["wedges"], exact_wedges=exact,
                           candidates=t["candidates"], predicted=n, chunks=t["chunks"]), f)
