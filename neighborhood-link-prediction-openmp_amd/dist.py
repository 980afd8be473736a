"""Multi-GPU link prediction: one process per GPU, source-vertex range shards,
one exchange step over RCCL (torch.distributed backend "nccl" on ROCm).

SURVEY.md §8(e).  The reference has a single OpenMP team over source vertices
(predict.hxx:287, schedule(dynamic, 2048)) and merges per-thread heaps serially
(predict.hxx:431-460).  Here:

  1. every rank holds a full CSR replica (second-hop lists are arbitrary, so
     the adjacency cannot be partitioned) and predicts the canonical top-k of
     its own contiguous source range [u_begin, u_end)  -> nlp_predict_device;
  2. one all_gather of the per-rank counts and one all_gather of the (padded)
     per-rank top-k lists over xGMI;
  3. every rank merges: the concatenation in rank order is in (u asc) order
     for equal scores, so a stable select by score gives exactly the
     single-GPU canonical result                   -> nlp_select_edges_device.

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


def gather_edges(local, n_local, group=None):
    """all_gather a [n_local, 3] int32 edge block from every rank (padded to the
    largest count).  Returns (concatenated [sum n, 3] tensor in rank order, counts)."""
    world = dist.get_world_size(group)
    dev = local.device
    cnt = torch.tensor([n_local], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    mx = max(counts) if counts else 0
    if mx == 0:
        return local[:0], counts
    pad = torch.zeros((mx, 3), dtype=local.dtype, device=dev)
    pad[:n_local] = local[:n_local]
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, counts)]), counts


def predict_sharded(local_predict, merge, span, max_edges, group=None, weights=None):
    """Run the sharded pipeline on this rank.

    local_predict(u_begin, u_end) -> (edges [n, 3] int32 tensor, n, info)
    merge(edges [N, 3], N, max_edges) -> (edges [k, 3], k)
    Returns (edges, k, info) -- identical on every rank."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    ub, ue = shard_ranges(span, world, weights)[rank]
    local, n, info = local_predict(ub, ue)
    allv, counts = gather_edges(local, n, group)
    out, k = merge(allv, int(sum(counts)), max_edges)
    info = dict(info or {}, shard=(ub, ue), counts=counts)
    return out, k, info


def hip_local_predict(graph, metric, hub, max_edges, out, stream=None, min_score=0.0):
    """Local predictor bound to libnlp (device output buffer `out` >= max_edges rows)."""
    def fn(ub, ue):
        n, t = graph.predict_device(metric, hub, max_edges, out, ub, ue, min_score=min_score, stream=stream)
        return out, n, t
    return fn


def hip_merge(graph, out, stream=None):
    def fn(allv, n, max_edges):
        k = graph.select_edges_device(allv, n, max_edges, out, stream=stream)
        return out, k
    return fn
