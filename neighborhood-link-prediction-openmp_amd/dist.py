"""Multi-GPU link prediction: one process per GPU, source-vertex range shards,
one exchange step over RCCL (torch.distributed backend "nccl" on ROCm).

SURVEY.md §8(e).  The reference has a single OpenMP team over source vertices
(predict.hxx:287, schedule(dynamic, 2048)) and merges per-thread heaps serially
(predict.hxx:431-460).  Here:

  1. every rank holds a full CSR replica (second-hop lists are arbitrary, so
     the adjacency cannot be partitioned) and predicts the canonical top-k of
     its own contiguous source range [u_begin, u_end)  -> nlp_predict_device;
  2. ONE all_gather over xGMI of fixed-stride blocks: entry 0 of a rank's
     block is a header with its count, entries 1..n its top-k list.  The
     stride is learnt once per job (one extra all_gather of the counts on the
     first call) and kept; a block that outgrows it is seen by every rank in
     the gathered headers, and all ranks regather with a larger stride;
  3. every rank merges in one kernel: block order is u order, so ranking each
     entry against the other blocks by score (ties: lower block first) gives
     exactly the single-GPU canonical result        -> nlp_merge_blocks_device.

Every rank ends with the identical global result (so rank 0 can report it
and any rank can evaluate F1).  The local predictor and the merge are
injectable so that the same orchestration runs under gloo on the CPU in the
tests (with the oracle standing in for the device kernels there).
"""
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
    largest block count); the exchange regathers with a larger stride."""

    def __init__(self, count):
        super().__init__("block count %d exceeds the exchange stride" % count)
        self.count = count


class Exchange:
    """Exchange state of one sharded job.  `cap` (entries per gathered block,
    header excluded) is identical on every rank: it is set from gathered data
    only, so every rank takes the same branch."""

    def __init__(self):
        self.cap = None
        self.ranges = None  # shard bounds, computed once (the weights' prefix sum is O(span))


def _grow(mx, max_edges):
    return int(min(max_edges, max(1024, mx + mx // 16)))


def write_header(block, n):
    """Entry 0 of a block: {count lo, count hi, NLP_BLOCK_MAGIC} (nlp.h)."""
    import numpy as np
    h = np.array([n & 0xFFFFFFFF, n >> 32, BLOCK_MAGIC], np.uint32).view(np.int32)
    block[0].copy_(torch.from_numpy(h))


def block_counts(blocks):
    """Per-block counts from the headers of gathered blocks [world, stride, 3]."""
    h = blocks[:, 0, :2].to(torch.int64).cpu() & 0xFFFFFFFF
    return [int(lo) | (int(hi) << 32) for lo, hi in h.tolist()]


def gather_blocks(block, cap, group=None):
    """One all_gather of every rank's first cap + 1 entries (header + result)
    into [world, cap + 1, 3]."""
    world = dist.get_world_size(group)
    stride = cap + 1
    recv = torch.empty((world * stride, 3), dtype=block.dtype, device=block.device)
    dist.all_gather_into_tensor(recv, block[:stride].contiguous(), group=group)
    return recv.view(world, stride, 3)


def predict_sharded(local_predict, merge, span, max_edges, group=None, weights=None, state=None):
    """Run the sharded pipeline on this rank.

    local_predict(u_begin, u_end) -> (block [>= max_edges + 1, 3] int32 tensor
        whose entries 1..n hold the shard's canonical result, n, info)
    merge(blocks [world, stride, 3], max_edges) -> (edges [>= k, 3], k); raises
        BlockOverflow when a header count exceeds stride - 1
    state: an Exchange kept across calls (the stride learnt by the first call);
        a fresh one costs one extra all_gather of the counts.
    Returns (edges, k, info) -- identical on every rank."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    state = state if state is not None else Exchange()
    if state.ranges is None:
        state.ranges = shard_ranges(span, world, weights)
    ub, ue = state.ranges[rank]
    block, n, info = local_predict(ub, ue)
    if block.shape[0] < max_edges + 1:
        raise ValueError("local block must hold max_edges + 1 entries")
    write_header(block, n)
    if state.cap is None:
        cnt = torch.tensor([n], dtype=torch.int64, device=block.device)
        counts = torch.empty(world, dtype=torch.int64, device=block.device)
        dist.all_gather_into_tensor(counts, cnt, group=group)
        state.cap = _grow(int(counts.max()), max_edges)
    while True:
        blocks = gather_blocks(block, state.cap, group)
        try:
            out, k = merge(blocks, max_edges)
            break
        except BlockOverflow as e:  # every rank sees the same headers, so all regather
            state.cap = _grow(e.count, max_edges)
    info = dict(info or {}, shard=(ub, ue), blocks=blocks, stride=state.cap + 1)
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
