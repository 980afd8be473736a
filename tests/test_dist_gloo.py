"""The multi-GPU orchestration (dist.py) with world_size 2 and 3 over gloo on
the CPU.  The per-rank device predictor is replaced by the oracle here (there is
no GPU in this container; tests/test_gpu_dist.py runs the same chain with the
HIP predictor and merge on the GPU box); the shard ranges, the histogram-first
quota selection, the all_gather of the shares and the rank-order merge rule are
the production code.  The result must equal the single-process canonical top-k
exactly."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _edges_tensor(u, w, s):
    a = np.zeros((len(u), 3), np.int32)
    a[:, 0] = u.view(np.int32)
    a[:, 1] = w.view(np.int32)
    a[:, 2] = s.view(np.int32)
    return torch.from_numpy(a)


def _canonical_merge(blocks, k):
    """Reference merge rule over the gathered blocks: headers checked like
    nlp_merge_blocks_device (overflow -> BlockOverflow), then a stable sort of
    the rank-ordered concatenation by score key descending, first k."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import nlp_loader
    from parity import keys_of
    dmod = nlp_loader.load_sub("dist")
    b = blocks.numpy()
    stride = b.shape[1]
    hdr = b[:, 0, :].view(np.uint32)
    counts = [int(h[0]) | (int(h[1]) << 32) for h in hdr]
    assert all(int(h[2]) == dmod.BLOCK_MAGIC for h in hdr)
    if max(counts) > stride - 1:
        raise dmod.BlockOverflow(max(counts))
    a = np.concatenate([b[r, 1:1 + c] for r, c in enumerate(counts)])
    s = a[:, 2].view(np.float32)
    kk = keys_of(s).astype(np.int64)
    order = np.lexsort((np.arange(len(kk)), -kk))[:k]
    return torch.from_numpy(a[order].copy()), len(order)


def _worker(rank, world, port, name, metric, hub, q, k_override=None):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import nlp_loader
        import pyoracle
        dmod = nlp_loader.load_sub("dist")
        g = dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False))
        off, keys = g["offsets"], g["keys"]
        k = int(g["k"][0]) if k_override is None else k_override

        def local(ub, ue):
            u, w, s, info = pyoracle.predict(off, keys, metric, hub, max_edges=k, u_begin=ub, u_end=ue)
            block = torch.zeros((k + 1, 3), dtype=torch.int32)
            block[1:1 + len(u)] = _edges_tensor(u, w, s)
            return block, len(u), info

        state = dmod.Exchange()
        outs = []
        for _ in range(2):  # the second call reuses the shard bounds
            out, n, info = dmod.predict_sharded(local, _canonical_merge, len(off) - 1, k, state=state)
            outs.append(out[:n].numpy().copy())
        assert np.array_equal(outs[0], outs[1])
        q.put((rank, outs[1], info["shard"], dmod.block_counts(info["blocks"]), info["shares"], info["local_count"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,metric,hub,k,world", [("g3k", 1, 4, None, 2), ("g3k", 7, 8, None, 2),
                                                     ("g300", 0, 0, None, 2), ("g3k", 1, 4, 50, 2),
                                                     ("g3k", 0, 0, 333, 3), ("g300", 1, 4, 10 ** 6, 3)])
def test_sharded_predict_equals_single_process(oracle, golden, name, metric, hub, k, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, metric, hub, q, k)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda x: x[0])
    g = golden[name]
    k = int(g["k"][0]) if k is None else k
    eu, ew, es, _ = oracle.predict(g["offsets"], g["keys"], metric, hub, max_edges=k)
    for rank, a, shard, counts, shares, local in res:
        assert np.array_equal(a[:, 0].view(np.uint32), eu)
        assert np.array_equal(a[:, 1].view(np.uint32), ew)
        assert np.array_equal(a[:, 2].view(np.uint32), es.view(np.uint32))
        assert counts == shares  # the gathered blocks hold exactly the quota shares
    assert all(res[i][2][1] == res[i + 1][2][0] for i in range(world - 1))  # contiguous shards
    assert sum(res[0][4]) == len(eu)  # the shares add up to the global top-k: nothing else crossed the wire
    assert all(res[r][4][r] <= res[r][5] for r in range(world))
