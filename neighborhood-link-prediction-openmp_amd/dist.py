"""Multi-GPU link prediction: one process per GPU, source-vertex range shards,
one selection exchange over RCCL (torch.distributed backend "nccl" on ROCm).

SURVEY.md §8(e).  The reference has a single OpenMP team over source vertices
(predict.hxx:287, schedule(dynamic, 2048)) and merges per-thread heaps serially
(predict.hxx:431-460).  Here:

  1. every rank holds a full CSR replica (second-hop lists are arbitrary, so
     the adjacency cannot be partitioned) and predicts the canonical top-k of
     its own contiguous source range [u_begin, u_end)  -> nlp_predict_device;
     the ranges balance the per-source wedge estimate (source_weights);
  2. histogram-first selection (select_quota): every rank histograms the top
     16 bits of its result's score keys and one all_gather of the 65536-bin
     histograms (world rows) gives every rank the bin of the k-th key and each
     rank's count above it; a second all_gather of the low-16-bit histograms
     inside that bin gives the k-th key itself, each rank's count above it and
     its ties.  The tie quota is handed out in rank (= u) order, the canonical
     tie rule, on the device; only the shares (world integers) are read back.
     A rank's share of the global top-k is a PREFIX of its canonical list;
  3. ONE all_gather of exactly those prefixes (block stride = the largest
     share + 1 header entry): about 12 k bytes in total instead of every
     rank's whole local top-k;
  4. every rank merges in one kernel: block order is u order, so ranking each
     entry against the other blocks by score (ties: lower block first) gives
     exactly the single-GPU canonical result        -> nlp_merge_blocks_device.

Every rank ends with the identical global result (so rank 0 can report it
and any rank can evaluate F1).  The local predictor and the merge are
injectable so that the same orchestration runs under gloo on the CPU in the
tests (with the oracle standing in for the device kernels there); with the
gloo backend the collectives run on CPU copies of the small tensors.
"""
import time

import torch
import torch.distributed as dist


def shard_ranges(span, world, weights=None):
    """Contiguous source ranges [b, e) per rank.  With `weights` (per-vertex
    work, e.g. wedge counts) the split balances their prefix sum; otherwise it
    balances vertex counts."""
    if weights is None:
        return [(span * r // world, span * (r + 1) // world) for r in range(world)]
    w = torch.as_tensor(weights, dtype=torch.float64).cpu()
    c = torch.cumsum(w, 0)
    tot = float(c[-1]) if c.numel() else 0.0
    bounds = [0]
    for r in range(1, world):
        bounds.append(int(torch.searchsorted(c, torch.tensor(tot * r / world, dtype=torch.float64))))
    bounds.append(span)
    bounds = [min(max(b, 0), span) for b in bounds]
    for i in range(1, len(bounds)):
        bounds[i] = max(bounds[i], bounds[i - 1])
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def source_weights(off, keys, hub, chunk=1 << 27):
    """Per-source work estimate for balancing the shards (SURVEY.md §8(e):
    balance by the wedge prefix, not by vertex count): W(u) = sum of deg v over
    the surviving intermediates v in N(u) (deg v <= hub; hub = 0: all), times
    (span - u) / span, the share of second-hop vertices w > u when ids carry no
    order (predict.hxx:221 keeps only w > u, so low ids own more candidates).
    Computed on the CSR's device in chunks; identical on every rank (integer
    sums, then float64 elementwise).  Returns a float64 CPU tensor [span]."""
    off = off.to(torch.int64)
    span = off.numel() - 1
    deg = (off[1:] - off[:-1]).to(torch.int32)
    surv = deg >= 1 if hub <= 0 else (deg >= 1) & (deg <= hub)
    cdeg = torch.where(surv, deg, torch.zeros_like(deg))
    m = keys.numel()
    pref = torch.zeros(m + 1, dtype=torch.int64, device=keys.device)
    carry = torch.zeros((), dtype=torch.int64, device=keys.device)
    for b in range(0, m, chunk):
        e = min(m, b + chunk)
        c = cdeg[keys[b:e].to(torch.int64)].to(torch.int64)
        pref[b + 1:e + 1] = torch.cumsum(c, 0) + carry
        carry = pref[e]
    w = (pref[off[1:]] - pref[off[:-1]]).to(torch.float64)
    w *= (span - torch.arange(span, device=w.device, dtype=torch.float64)) / max(span, 1)
    return w.cpu()


BLOCK_MAGIC = 0x4E4C5042  # nlp.h NLP_BLOCK_MAGIC


class BlockOverflow(RuntimeError):
    """A gathered block held more entries than the exchange stride (count = the
    largest block count).  With the quota exchange the stride is exact, so this
    means the blocks were corrupted in transit."""

    def __init__(self, count):
        super().__init__("block count %d exceeds the exchange stride" % count)
        self.count = count


class Exchange:
    """Exchange state of one sharded job: the shard bounds (the weights' prefix
    sum is O(span), computed once)."""

    def __init__(self):
        self.ranges = None


def write_header(block, n):
    """Entry 0 of a block: {count lo, count hi, NLP_BLOCK_MAGIC} (nlp.h)."""
    import numpy as np
    h = np.array([n & 0xFFFFFFFF, n >> 32, BLOCK_MAGIC], np.uint32).view(np.int32)
    block[0].copy_(torch.from_numpy(h))


def block_counts(blocks):
    """Per-block counts from the headers of gathered blocks [world, stride, 3]."""
    h = blocks[:, 0, :2].to(torch.int64).cpu() & 0xFFFFFFFF
    return [int(lo) | (int(hi) << 32) for lo, hi in h.tolist()]


def _coll(t, group=None):
    """The tensor the collective runs on: gloo takes CPU tensors."""
    return t.cpu() if dist.get_backend(group) == "gloo" and t.is_cuda else t


def score_keys(edges, n):
    """Order-preserving uint32 keys (as int64) of the scores in edges[:n, 2]
    (int32 bit patterns): larger score -> larger key, -0 == +0, NaN -> 0 --
    the library's score_key (kernels.hpp) and the oracle's nlpo_score_key."""
    b = edges[:n, 2].to(torch.int64) & 0xFFFFFFFF
    b = torch.where(b == 0x80000000, torch.zeros_like(b), b)  # -0.0 -> +0.0
    neg = (b & 0x80000000) != 0
    k = torch.where(neg, (~b) & 0xFFFFFFFF, b | 0x80000000)
    nan = ((b & 0x7F800000) == 0x7F800000) & ((b & 0x007FFFFF) != 0)
    return torch.where(nan, torch.zeros_like(k), k)


HBINS = 1 << 16


def _hist16(idx, valid, device):
    """Counts of the 16-bit values idx[valid] (int64 [HBINS]) without a host
    sync: index_add_ into a fixed-size tensor (torch.bincount sizes its output
    from the data's maximum, which reads it back to the host)."""
    h = torch.zeros(HBINS + 1, dtype=torch.int64, device=device)
    if idx.numel():
        h.index_add_(0, torch.where(valid, idx, torch.full_like(idx, HBINS)), torch.ones_like(idx))
    return h[:HBINS]


def _all_gather_rows(x, group=None):
    """[world, len(x)] on x's device: one all_gather (gloo: on CPU copies)."""
    world = dist.get_world_size(group)
    send = _coll(x.contiguous(), group)
    recv = torch.empty(world * x.numel(), dtype=x.dtype, device=send.device)
    dist.all_gather_into_tensor(recv, send, group=group)
    return recv.to(x.device).view(world, x.numel())


def _kth_bin(per_rank, need):
    """Per-rank histograms [world, HBINS] and the number `need` (>= 1, device
    scalar) of entries wanted from the top: the bin holding the need-th largest
    entry over all ranks, and per rank the entries in bins above it."""
    from_top = torch.cumsum(per_rank.flip(1), 1)          # per rank, bins HBINS-1 .. 0
    tot_top = from_top.sum(0)
    j = torch.searchsorted(tot_top, need.view(1)).clamp_(max=HBINS - 1)  # first from-top bin reaching need
    above = torch.where(j > 0, from_top[:, (j - 1).clamp(min=0)].squeeze(1), torch.zeros_like(from_top[:, 0]))
    return (HBINS - 1 - j).squeeze(0), above


def select_quota(edges, n, max_edges, group=None):
    """Histogram-first global selection.  `edges[:n]` is this
    rank's canonical list (score key desc, then u, then w).  Returns (share,
    shares): how many leading entries of this rank's list belong to the
    canonical global top max_edges, and every rank's share (rank order).

    Two collectives and one host read: an all_gather of every rank's histogram
    of the top 16 key bits gives every rank the bin b of the k-th key and each
    rank's count above b; an all_gather of the histograms of the low 16 bits
    inside b gives the k-th key itself, each rank's count above it and its tie
    count, from which the tie quota is handed out in rank (= u) order -- the
    canonical tie rule.  Everything stays on the list's device until the shares
    (world integers) are read back to size the block exchange."""
    rank = dist.get_rank(group)
    dev = edges.device
    keys = score_keys(edges, n)
    ones = torch.ones_like(keys, dtype=torch.bool)
    hi = _all_gather_rows(_hist16(keys >> 16, ones, dev), group)          # [world, HBINS]
    counts = hi.sum(1)                                                     # per-rank list lengths
    total = counts.sum()
    take = torch.clamp(total, max=int(max_edges))
    b, above_hi = _kth_bin(hi, take.clamp(min=1))
    lo = _all_gather_rows(_hist16(keys & 0xFFFF, (keys >> 16) == b, dev), group)
    l, above_lo = _kth_bin(lo, (take - above_hi.sum()).clamp(min=1))
    above = above_hi + above_lo                                            # per rank: keys > the k-th key
    ties = lo[:, l]                                                        # per rank: keys == the k-th key
    quota = take - above.sum()
    before = torch.cumsum(ties, 0) - ties                                  # ties of the ranks before
    shares = above + torch.minimum(ties, (quota - before).clamp(min=0))
    shares = torch.where(take == total, counts, shares)                    # everything kept: no boundary key
    shares = [int(x) for x in shares.cpu().tolist()]
    return shares[rank], shares


def gather_blocks(block, stride, group=None):
    """One all_gather of every rank's first `stride` entries (header + its
    share) into [world, stride, 3].  A block shorter than the stride (a rank
    sized to its own smaller result) is padded, so every rank sends the same
    number of entries."""
    world = dist.get_world_size(group)
    send = block[:stride]
    if send.shape[0] < stride:
        pad = torch.zeros((stride, 3), dtype=block.dtype, device=block.device)
        pad[:send.shape[0]] = send
        send = pad
    send = _coll(send.contiguous(), group)
    recv = torch.empty((world * stride, 3), dtype=block.dtype, device=send.device)
    dist.all_gather_into_tensor(recv, send, group=group)
    return recv.to(block.device).view(world, stride, 3)


def predict_sharded(local_predict, merge, span, max_edges, group=None, weights=None, state=None):
    """Run the sharded pipeline on this rank.

    local_predict(u_begin, u_end) -> (block [>= max_edges + 1, 3] int32 tensor
        whose entries 1..n hold the shard's canonical result, n, info)
    merge(blocks [world, stride, 3], max_edges) -> (edges [>= k, 3], k)
    state: an Exchange kept across calls (the shard bounds).
    Returns (edges, k, info) -- identical on every rank."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    state = state if state is not None else Exchange()
    if state.ranges is None:
        state.ranges = shard_ranges(span, world, weights)
    ub, ue = state.ranges[rank]
    t0 = time.perf_counter()
    block, n, info = local_predict(ub, ue)  # synchronous: the shard's result is complete on return
    t1 = time.perf_counter()
    if block.shape[0] < min(n, max_edges) + 1:
        raise ValueError("local block must hold the result + 1 header entry")
    share, shares = select_quota(block[1:], n, max_edges, group)  # ends with a host read of the shares
    t2 = time.perf_counter()
    write_header(block, share)
    blocks = gather_blocks(block, max(shares) + 1, group)
    out, k = merge(blocks, max_edges)  # synchronous
    t3 = time.perf_counter()
    # predict_ms: this rank's shard (score + local top-k + order); the exchange that
    # replaces the reference's serial merge (predict.hxx:431-460) split into the
    # histogram selection and the block gather + merge
    info = dict(info or {}, shard=(ub, ue), blocks=blocks, stride=max(shares) + 1, shares=shares, local_count=n,
                predict_ms=(t1 - t0) * 1e3, select_xchg_ms=(t2 - t1) * 1e3, gather_merge_ms=(t3 - t2) * 1e3,
                exchange_ms=(t3 - t1) * 1e3)
    return out, k, info


def hip_local_predict(graph, metric, hub, max_edges, block, stream=None, min_score=0.0):
    """Local predictor bound to libnlp: the shard's result goes to entries
    1..n of the device block buffer (>= max_edges + 1 rows)."""
    def fn(ub, ue):
        n, t = graph.predict_device(metric, hub, max_edges, block[1:], ub, ue, min_score=min_score, stream=stream)
        return block, n, t
    return fn


def hip_merge(graph, out, stream=None):
    """Merge bound to libnlp (nlp_merge_blocks_device, one kernel over the gathered blocks)."""
    def fn(blocks, max_edges):
        try:
            k = graph.merge_blocks_device(blocks, max_edges, out, stream=stream)
        except Exception as e:  # NLP_ERR_CAPACITY carries the largest count
            if getattr(e, "status", None) == 5 and hasattr(e, "count"):
                raise BlockOverflow(e.count) from None
            raise
        return out, k
    return fn
