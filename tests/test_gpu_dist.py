"""The multi-GPU chain end to end with the HIP predictor: dist.predict_sharded
(wedge-balanced source ranges, histogram-first quota selection, all_gather of
the shares, nlp_merge_blocks_device) in 2 and 3 processes on the one GPU of
the box.  RCCL refuses two ranks on one device, so the collectives run over
gloo on CPU copies of the small tensors (dist._coll); the local predictions
and the merge are the library's, on cuda:0.  Every rank's result must equal
the single-process prediction bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


GRAPHS = {"small": (30000, 10, 5), "1M": (1_000_000, 12, 9)}


def _worker(rank, world, port, cases, q, backend="gloo", graph="small"):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import nlp_loader
        from test_gpu_parity import random_csr
        nlp = nlp_loader.load()
        dmod = nlp_loader.load_sub("dist")
        res = []
        if graph in GRAPHS:
            off, keys = random_csr(*GRAPHS[graph])
            G = nlp.Graph(off, keys, device=0)
            off_t = torch.from_numpy(off.astype(np.int64))
            keys_t = torch.from_numpy(keys.view(np.int32))
        else:  # a bench config's stand-in, generated on the device (identical on every rank)
            off_t, keys_t = _standin(graph)
            G = nlp.Graph.from_device(off_t, keys_t)
        span = off_t.numel() - 1
        with G:
            for metric, hub, k in cases:
                block = torch.empty((k + 1, 3), dtype=torch.int32, device="cuda")
                out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
                st = dmod.Exchange()
                w = dmod.source_weights(off_t, keys_t, hub)
                edges, n, info = dmod.predict_sharded(dmod.hip_local_predict(G, metric, hub, k, block),
                                                      dmod.hip_merge(G, out), span, k, state=st, weights=w)
                res.append((edges[:n].cpu().numpy().copy(), info["shares"]))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _standin(name):
    """The CONFIGS entry's stand-in graph on cuda:0 (graphgen: Chung-Lu pairs,
    the reference's ingest and deletion batch on the device)."""
    import torch
    import nlp_loader
    gg = nlp_loader.load_sub("graphgen")
    off, keys, _, _, _ = gg.make_workload(gg.CONFIGS[name], "cuda")
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return off, keys


def _run_chain(nlp, world, cases, backend="gloo", graph="small"):
    import torch
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from test_gpu_parity import random_csr
    if graph in GRAPHS:
        off, keys = random_csr(*GRAPHS[graph])
        G = nlp.Graph(off, keys)
    else:
        sys.path.insert(0, ROOT)
        off_t, keys_t = _standin(graph)
        G = nlp.Graph.from_device(off_t, keys_t)
        del off_t, keys_t
    want = []
    with G:
        for metric, hub, k in cases:
            out = torch.empty((k, 3), dtype=torch.int32, device="cuda")
            n, _ = G.predict_device(metric, hub, k, out)
            want.append(out[:n].cpu().numpy().copy())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q, backend, graph)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=400) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res in got:
        for (a, shares), b, (metric, hub, k) in zip(res, want, cases):
            assert np.array_equal(a, b), (rank, metric, hub)
            assert sum(shares) == len(b)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_sharded_chain_equals_single_gpu(nlp, world):
    _run_chain(nlp, world, [(1, 4, 2000), (7, 8, 5000), (0, 0, 3000), (1, 16, 10 ** 6)])


@pytest.mark.timeout(300)
def test_gpu_sharded_chain_h16_1m_vertices(nlp):
    """H = 16 on a 1 M-vertex graph (k-filling: more candidates than k), 2 ranks."""
    _run_chain(nlp, 2, [(1, 16, 400_000), (7, 16, 300_000)], graph="1M")


@pytest.mark.timeout(300)
def test_gpu_sharded_chain_nccl_world1(nlp):
    """The production backend: RCCL ("nccl") with the tensors on cuda:0 -- the
    histogram all_gathers, the quota and the block exchange never leave the
    device except for the shares (one rank: RCCL refuses two ranks on one GPU)."""
    _run_chain(nlp, 1, [(1, 4, 2000), (1, 16, 400_000)], backend="nccl", graph="1M")


@pytest.mark.timeout(500)
def test_gpu_sharded_chain_c2_standin(nlp):
    """The exchange at a bench config's size: the C2 (soc-LiveJournal1) stand-in,
    4.8 M vertices, 1.4e8 entries, generated by every rank on the device; 2
    ranks, Jaccard and Adamic-Adar at H = 16 with k beyond one rank's share,
    every rank's merged list equal to the single-process call bit for bit."""
    _run_chain(nlp, 2, [(1, 16, 3_000_000), (7, 16, 1_000_000), (0, 4, 200_000)], graph="C2-soc-LiveJournal1")
