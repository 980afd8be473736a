"""Host-side logic on the CPU: synthetic workload generator, shard ranges, the
parity helpers themselves."""
import numpy as np
import pytest
import torch

import nlp_loader

gg = nlp_loader.load_sub("graphgen")
dmod = nlp_loader.load_sub("dist")


@pytest.fixture(scope="module")
def small():
    return gg.make_workload("C2-soc-LiveJournal1", "cpu", 0.002)


def test_workload_is_a_sorted_symmetric_simple_graph(small):
    off, keys, du, dw, info = small
    off = off.numpy()
    keys = keys.numpy().astype(np.int64)
    span = len(off) - 1
    assert off[0] == 0 and off[-1] == len(keys) and np.all(np.diff(off) >= 0)
    assert off[1] == 0, "vertex 0 must be absent (1-based ids)"
    rows = np.repeat(np.arange(span), np.diff(off))
    assert np.all(keys < span) and np.all(keys >= 1)
    assert not np.any(rows == keys), "self-loops must be removed (selfLoop.hxx:304-311)"
    same = rows[1:] == rows[:-1]
    assert np.all(keys[1:][same] > keys[:-1][same]), "rows sorted, no duplicates"
    fwd = set((rows * span + keys).tolist())
    rev = set((keys * span + rows).tolist())
    assert fwd == rev, "graph must be symmetric"
    assert info["M"] == len(keys)


def test_deletions_removed_both_directions(small):
    off, keys, du, dw, info = small
    span = off.numel() - 1
    rows = torch.repeat_interleave(torch.arange(span), off[1:] - off[:-1])
    present = set((rows * span + keys.long()).tolist())
    dels = (du.long() * span + dw.long()).tolist()
    assert len(dels) == 2 * info["k"]
    assert not (set(dels) & present)
    d = set(dels)
    assert all((v * span + u) in d for u, v in zip(du.tolist(), dw.tolist()))
    assert info["M_before"] - info["M"] == len(dels)


def test_workload_is_deterministic():
    a = gg.make_workload("C1-web-Google", "cpu", 0.01)
    b = gg.make_workload("C1-web-Google", "cpu", 0.01)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])


def test_uniform_stream_properties():
    u = gg.uniform(3, 1, 0, 200000, "cpu")
    assert float(u.min()) >= 0.0 and float(u.max()) < 1.0
    assert abs(float(u.mean()) - 0.5) < 0.01
    # counter-based: a slice equals the same slice of a longer draw
    assert torch.equal(gg.uniform(3, 1, 1000, 10, "cpu"), u[1000:1010])
    p = gg.permutation(1000, 5, 2, "cpu")
    assert torch.equal(torch.sort(p).values, torch.arange(1000))


def test_shard_ranges_cover_and_balance():
    for span, world in ((10, 3), (4_847_572, 8), (5, 8)):
        r = dmod.shard_ranges(span, world)
        assert r[0][0] == 0 and r[-1][1] == span
        assert all(r[i][1] == r[i + 1][0] for i in range(world - 1))
    w = np.zeros(100)
    w[:10] = 100.0  # heavy head
    r = dmod.shard_ranges(100, 4, weights=w)
    assert r[0][0] == 0 and r[-1][1] == 100 and r[0][1] <= 10
