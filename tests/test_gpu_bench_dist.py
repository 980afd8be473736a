"""bench.py's N > 1 path, executed: the driver launches `torch.distributed.run
--nproc-per-node N bench.py --gpus N` on an 8-GPU node; here the same launcher
runs 2 ranks on the box's one GPU over gloo (NLP_DIST_BACKEND=gloo -- RCCL
refuses two ranks on one device), on the C1 (web-Google-shaped) config.  The
line must parse, carry every rank's shard and exchange times, and predict
exactly what the world-1 run predicts (the sharded chain is the reference's
one OpenMP team plus its serial merge, predict.hxx:284-339, 431-460).
Unmeasured on multi-GPU hardware: this checks the code path, not RCCL/xGMI."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "3", "--warmup", "1", "--config", "C1-web-Google", "--no-cpu-baseline", "--no-dropin",
        "--sweep", "", "--work-point", "16", "--wp-steps", "2", "--wp-warmup", "1"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _line(cmd, env):
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(900)
def test_gpu_bench_two_ranks_gloo_equals_world1():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ)
    one = _line([sys.executable, "bench.py", "--gpus", "1"] + ARGS, env)
    env2 = dict(env, NLP_DIST_BACKEND="gloo")
    two = _line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                 "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2"] + ARGS,
                env2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["predicted"] == one["predicted"] > 0
    assert two["value"] > 0 and two["ms_per_step"] > 0 and two["amortized_ms_per_call"] > two["ms_per_step"]
    pr = two["per_rank"]
    for key in ("predict_ms", "select_xchg_ms", "gather_merge_ms", "exchange_ms"):
        assert len(pr[key]) == 2 and all(x >= 0 for x in pr[key]), key
    assert pr["imbalance"] is not None and pr["imbalance"] >= 1.0
    assert pr["exchange_ms_max"] == max(pr["exchange_ms"])
    wp1, wp2 = one["work_point"], two["work_point"]
    assert wp1["H"] == wp2["H"] == 16
    assert wp2["predicted"] == wp1["predicted"] > 0
    assert len(wp2["per_rank"]["predict_ms"]) == 2
    # F1 is a property of the predicted set, which is the same for both runs
    assert wp2["f1"] == pytest.approx(wp1["f1"], rel=0, abs=0)
    assert two["graph_create_phases_ms"]["upload"] >= 0
