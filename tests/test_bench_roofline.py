"""bench.py's roofline pairs one kernel's algorithmic bytes with that same
kernel's device time (CPU: synthetic per-call timing fields)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_roofline_pairs_bytes_and_time_of_one_kernel():
    b = _bench()
    ids = sorted(b.HOT_KERNELS)[:2]
    # calls alternate between two dominant kernels: kernel A 20 us / 200 kB, kernel B 18 us / 330 kB
    lasts = [dict(hot_kernel=ids[0], hot_ms=0.020, hot_bytes=200000), dict(hot_kernel=ids[1], hot_ms=0.018,
                                                                            hot_bytes=330000)] * 5
    acc = dict(hot_ms=sum(x["hot_ms"] for x in lasts) / 10, hot_bytes=sum(x["hot_bytes"] for x in lasts) / 10)
    hot = {}
    for one in lasts:
        e = hot.setdefault(one["hot_kernel"], [0.0, 0, 0])
        e[0] += one["hot_ms"]
        e[1] += one["hot_bytes"]
        e[2] += 1
    acc["_hot"] = hot
    r = b.roofline_of(acc, lasts[-1], "none", 1, 1, 4)
    assert r["kernel"] == b.HOT_KERNELS[ids[0]]  # the longer one, not the last call's
    assert r["algorithmic_bytes"] == 200000 and abs(r["kernel_ms"] - 0.020) < 1e-12
    assert abs(r["achieved"] - 200000 / 0.020e-3 / 1e9) < 1e-6
