"""Synthetic inputs for the link-prediction path (host/device plumbing, not the
hot path).

The reference experiment (main.cxx:157-179, 241-245) reads a SuiteSparse graph,
symmetrizes it, removes self-loops and then deletes a random fraction of its
undirected edges.  The SuiteSparse graphs are not available offline, so the
bench and the large parity tests use deterministic Chung-Lu stand-ins with the
shape of each BASELINE.json config:

    endpoints i.i.d. with P(i) ~ (i+1)^-alpha, ids randomly permuted,
    self-loops dropped, (u, v) deduped, then symmetrized.

Vertex ids are 1..n and row 0 is empty, as in the reference's DiGraph
(mtx.hxx reads 1-based ids; Graph.hxx span() = n+1).

On a GPU the pairs go through the reference's own ingest and deletion batch
on the device instead (make_workload's ingest="reference"); the host-side
construction below is the "simple" variant the CPU tests use.

Deletions follow the reference's sampling shape (batch.hxx:29-58, 99-112):
a uniformly random vertex u in [1, n] (retried up to 5 times when deg(u)=0,
_utility.hxx:432), then a uniformly random entry of N(u); both directions are
deleted; duplicates are removed by tidy (batch.hxx:200-208).  Random numbers come
from a counter-based splitmix64 stream, so the workload is bit-identical on the
CPU and on any GPU (the draws are not the reference's minstd_rand0 sequence --
bit-exact replay of the reference's ingest is done by the oracle's ref_driver
for the golden fixtures instead).

Everything is vectorised torch so it runs on the GPU (bench) or the CPU (tests).
"""
import math

import numpy as np
import torch

# SURVEY.md §8(d) stand-ins: name -> (n, m, alpha, graph_seed, deletion fraction, metric, hub)
CONFIGS = {
    "C1-web-Google": (916_428, 5_105_039, 0.7, 11, 0.01, "JAC", 4),
    "C2-soc-LiveJournal1": (4_847_571, 68_993_773, 0.6, 12, 0.1, "JAC", 4),
    "C3-uk-2005": (39_459_925, 936_364_282, 0.7, 13, 0.1, "AA", 4),
    "C4-sk-2005": (50_636_154, 1_949_412_601, 0.7, 14, 0.1, "JAC", 4),
    "C5-sk-2005-ihub": (50_636_154, 1_949_412_601, 0.7, 14, 0.01, "CN", 0),
}


_M64 = (1 << 64) - 1


def _s64(c):
    """uint64 constant as a signed int64 Python int (torch has no uint64 arithmetic)."""
    return c - (1 << 64) if c >= (1 << 63) else c


def _srl(x, s):
    """Logical right shift of int64 tensor values."""
    return (x >> s) & ((1 << (64 - s)) - 1)


def splitmix64(x):
    """splitmix64 finaliser on int64 tensors (wrapping arithmetic): a
    counter-based generator, identical on CPU and GPU and independent of
    launch geometry (torch's Philox offsets are not)."""
    z = x + _s64(0x9E3779B97F4A7C15)
    z = (z ^ _srl(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _srl(z, 27)) * _s64(0x94D049BB133111EB)
    return z ^ _srl(z, 31)


def uniform(seed, stream, start, count, device):
    """count doubles in [0, 1) for counter indices [start, start+count) of (seed, stream)."""
    base = _s64(((seed * 0x100000001B3) ^ (stream * 0xC2B2AE3D27D4EB4F)) & _M64)
    idx = torch.arange(start, start + count, dtype=torch.int64, device=device)
    z = splitmix64(splitmix64(idx + base))
    return _srl(z, 11).to(torch.float64) * (1.0 / (1 << 53))


def permutation(n, seed, stream, device):
    """Deterministic random permutation of 0..n-1 (argsort of random 64-bit keys)."""
    base = _s64(((seed * 0x100000001B3) ^ (stream * 0xC2B2AE3D27D4EB4F)) & _M64)
    k = splitmix64(torch.arange(n, dtype=torch.int64, device=device) + base)
    return torch.sort(k, stable=True).indices


# Device sorts, boolean indexing and nonzero break beyond 2^31 items on this
# torch build: larger tensors go through the chunked helpers below.
BIG = 1 << 30


def masked(x, m, limit=None):
    """x[m] in chunks (boolean indexing breaks beyond 2^31 items)."""
    limit = limit or BIG
    if x.numel() <= limit:
        return x[m]
    return torch.cat([a[b] for a, b in zip(torch.split(x, limit), torch.split(m, limit))])


def nonzero1(m, limit=None):
    """torch.nonzero(m)[:, 0] of a 1-d mask, in chunks."""
    limit = limit or BIG
    if m.numel() <= limit:
        return torch.nonzero(m).squeeze(1)
    return torch.cat([torch.nonzero(c).squeeze(1) + i * limit for i, c in enumerate(torch.split(m, limit))])


def big_unique(x, limit=None):
    """torch.unique (sorted) for tensors beyond the device sort's 2^31-item
    limit: the value range is cut into buckets of at most ~limit items each."""
    limit = limit or BIG
    if x.numel() <= limit:
        return torch.unique(x)
    lo, hi = int(x.min()), int(x.max()) + 1
    nb = 2 * ((x.numel() + limit - 1) // limit)
    if hi - lo < 2 * nb:  # few distinct values: nothing to split on
        return torch.unique(x)
    edges = [lo + (hi - lo) * i // nb for i in range(nb + 1)]
    parts = []
    for a, b in zip(edges[:-1], edges[1:]):
        # boolean indexing breaks beyond 2^31 items: mask chunk by chunk
        sub = torch.cat([c[(c >= a) & (c < b)] for c in torch.split(x, limit)])
        parts.append(big_unique(sub, limit) if sub.numel() > limit else torch.unique(sub))
        del sub
    return torch.cat(parts)


def chung_lu_edges(n, m, alpha, seed, device="cpu"):
    """Return (src, dst) int64 tensors of m distinct directed edges, ids in 1..n.

    The CDF is computed on the host in float64 (sequential cumsum) so that every
    device sees the same values; all random draws come from splitmix64."""
    w = np.arange(1, n + 1, dtype=np.float64) ** (-alpha)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    cdf = torch.from_numpy(cdf).to(device)
    del w
    perm = permutation(n, seed, 1, device) + 1
    draws = int(m * 1.15) + 1024
    keys = []
    have = 0
    pos = 0  # counter position in the endpoint streams
    chunk = 1 << 26
    while True:
        todo = min(chunk, draws)
        u = torch.searchsorted(cdf, uniform(seed, 2, pos, todo, device)).clamp_(max=n - 1)
        v = torch.searchsorted(cdf, uniform(seed, 3, pos, todo, device)).clamp_(max=n - 1)
        pos += todo
        u = perm[u]
        v = perm[v]
        ok = u != v
        keys.append((u[ok] * (n + 1) + v[ok]))
        del u, v, ok
        have += todo
        if have >= draws:
            allk = big_unique(torch.cat(keys))
            keys = [allk]
            if allk.numel() >= m:
                break
            draws = int((m - allk.numel()) * 1.3) + 1024
            have = 0
    allk = keys[0]
    if allk.numel() > m and allk.numel() > BIG:
        allk = _select_m(allk, m, seed, device)
    elif allk.numel() > m:
        sel = permutation(allk.numel(), seed, 4, device)[:m]
        allk = torch.sort(allk[sel]).values
    return allk // (n + 1), allk % (n + 1)


def _select_m(allk, m, seed, device):
    """m of the sorted keys allk, chosen by the smallest random 64-bit tags
    (splitmix64 of the position), without sorting all of them (the device sort
    stops at 2^31 items): a histogram of the tags' top 16 bits fixes the cut,
    only the boundary bin is sorted.  Returns the chosen keys in sorted order."""
    base = _s64(((seed * 0x100000001B3) ^ (4 * 0xC2B2AE3D27D4EB4F)) & _M64)
    tag = splitmix64(torch.arange(allk.numel(), dtype=torch.int64, device=device) + base)
    top = _srl(tag, 48)
    cnt = torch.cumsum(torch.bincount(top, minlength=1 << 16), 0)
    b = int(torch.searchsorted(cnt, torch.tensor(m, device=device, dtype=cnt.dtype)))
    below = int(cnt[b - 1]) if b > 0 else 0
    keep = top < b
    inb = nonzero1(top == b)
    order = torch.sort(tag[inb]).indices[: m - below]
    keep[inb[order]] = True
    return masked(allk, keep)  # allk is sorted, so is the selection


def symmetric_csr(n, src, dst):
    """CSR (offsets int64 [n+2], keys int32 [M]) of the symmetrized, self-loop-free,
    deduplicated graph, span = n+1 (row 0 empty)."""
    span = n + 1
    a = torch.cat([src * span + dst, dst * span + src])
    a = big_unique(a)  # sorted
    rows = a // span
    keys = (a % span).to(torch.int32)
    del a
    counts = torch.bincount(rows, minlength=span)
    offsets = torch.zeros(span + 1, dtype=torch.int64, device=src.device)
    offsets[1:] = torch.cumsum(counts, 0)
    return offsets, keys


def csr_rows(offsets, M):
    span = offsets.numel() - 1
    deg = offsets[1:] - offsets[:-1]
    return torch.repeat_interleave(torch.arange(span, device=offsets.device), deg, output_size=M)


def delete_edges(offsets, keys, frac, seed, n=None):
    """Reference-shaped random undirected deletions (see module docstring).

    Returns (offsets', keys', del_u, del_w) where (del_u, del_w) are the sorted,
    unique directed deletions (both directions), i.e. main.cxx's `deletions0`;
    the reference predicts maxEdges = len(deletions0) // 2 links (main.cxx:50)."""
    dev = offsets.device
    span = offsets.numel() - 1
    n = span - 1 if n is None else n
    M = keys.numel()
    D = int(frac * M / 2)
    deg = offsets[1:] - offsets[:-1]
    # 5 tries per draw (retry(fn, 5), batch.hxx:110 / _utility.hxx:432)
    tries = 5
    u = (1 + torch.floor(n * uniform(seed, 5, 0, D * tries, dev).view(D, tries))).long()
    u.clamp_(max=span - 1)
    has = deg[u] > 0
    first = torch.argmax(has.to(torch.int8), dim=1)
    okrow = has.any(dim=1)
    u = u.gather(1, first[:, None])[:, 0][okrow]
    r = uniform(seed, 6, 0, u.numel(), dev)
    vi = torch.floor(r * deg[u].double()).long()
    v = keys[offsets[u] + vi].long()
    pairs = big_unique(torch.cat([u * span + v, v * span + u]))
    rows = csr_rows(offsets, M)
    ek = rows * span + keys.long()
    keep = torch.cat([pairs[torch.searchsorted(pairs, c).clamp_(max=pairs.numel() - 1)] != c
                      for c in torch.split(ek, BIG)])  # chunked: searchsorted stops at 2^31 items
    keys2 = masked(keys, keep)
    counts = torch.bincount(masked(rows, keep), minlength=span)
    off2 = torch.zeros(span + 1, dtype=torch.int64, device=dev)
    off2[1:] = torch.cumsum(counts, 0)
    return off2, keys2, (pairs // span).to(torch.int32), (pairs % span).to(torch.int32)


def make_workload(name_or_spec, device="cpu", scale=1.0, ingest=None):
    """Build (offsets, keys, del_u, del_w, spec) for a CONFIGS entry.

    `scale` shrinks n and m proportionally (tests use small scales).

    ingest = "reference" (the default on a GPU): the Chung-Lu pairs are the
    MatrixMarket file's lines and go through the reference's own ingest and
    deletion batch on the device (nlp_ingest_device / nlp_delete_edges_device,
    SURVEY §8(f) N1 + N2): symmetrize with its duplicate rule (the graph keeps
    the duplicate entries main.cxx's graph has), then generateEdgeDeletions
    with std::default_random_engine(seed + 1000) and batch size
    size_t(d |E| / 2) (main.cxx:164-169), tidied and applied one occurrence at
    a time.  ingest = "simple" (the default on the CPU): the deduplicated
    symmetric graph and the counter-based deletions above, for host tests."""
    spec = CONFIGS[name_or_spec] if isinstance(name_or_spec, str) else name_or_spec
    n, m, alpha, seed, d, metric, hub = spec
    n = max(16, int(math.ceil(n * scale)))
    m = max(16, int(math.ceil(m * scale)))
    if ingest is None:
        ingest = "reference" if str(device).startswith("cuda") else "simple"
    src, dst = chung_lu_edges(n, m, alpha, seed, device)
    if ingest == "reference":
        import nlp_amd
        src, dst = src.to(torch.int32), dst.to(torch.int32)
        if src.is_cuda:
            torch.cuda.synchronize()
            torch.cuda.empty_cache()  # the library allocates its scratch with hipMalloc
        off, keys = nlp_amd.ingest_device(src, dst, n)
        del src, dst
        if off.is_cuda:
            torch.cuda.empty_cache()
        batch = int(d * keys.numel() / 2)  # size_t(d * x.size()/2), main.cxx:166
        off2, keys2, du, dw, _ = nlp_amd.delete_edges_device(off, keys, batch, seed + 1000)
    else:
        off, keys = symmetric_csr(n, src, dst)
        del src, dst
        off2, keys2, du, dw = delete_edges(off, keys, d, seed + 1000, n=n)
    return off2, keys2, du, dw, dict(n=n, m=m, alpha=alpha, seed=seed, d=d, metric=metric, hub=hub,
                                     M_before=int(keys.numel()), M=int(keys2.numel()),
                                     k=int(du.numel()) // 2, ingest=ingest)
