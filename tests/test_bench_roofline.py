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


def test_build_roofline_names_the_entry_pass():
    """roofline_build: the amortized value's largest build kernel, its phase
    time and 26 algorithmic bytes per entry; traffic from the committed PMC
    record of the config (C4 holds one), none for an unknown config."""
    b = _bench()
    r = b.build_roofline({"entry_classes": 200.0, "transpose": 100.0}, 10 ** 9, "C4-sk-2005", 1)
    assert r["kernel"] == "k_hp_entry_classes" and r["algorithmic_bytes"] == 26 * 10 ** 9
    assert abs(r["achieved"] - 26e9 / 0.2 / 1e9) < 1e-9 and abs(r["frac"] - r["achieved"] / b.HBM_PEAK_GBS) < 1e-12
    assert r["traffic"] and r["traffic_frac"] > r["frac"]
    assert b.build_roofline({"entry_classes": 200.0}, 10 ** 9, "none", 1)["traffic"] is None
    assert b.build_roofline({}, 10 ** 9, "C4-sk-2005", 1) is None
