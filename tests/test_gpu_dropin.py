"""The reference's own experiment driver on the GPU: main.cxx, unmodified,
compiled with inc/predict.hxx swapped for include/nlp/predict.hxx
(oracle/_ref/main_dropin, built by oracle/Makefile in the container where the
reference lies; the binary travels like oracle/_ref/ref_driver).  It ingests
with the reference's code (readMtxOmpW, symmetrizeOmp, removeSelfLoopsOmpU,
its own random deletion batch) and makes its 99 calls (PREDICT_LINKS_ALL,
main.cxx:67-80, 212-220) through the drop-in header.  main.cxx seeds its
deletions from std::random_device, so the check is structural: every call's
log line parses with process.js's regex (main.cxx:205), the nine metrics x
eleven thresholds in the reference's order, precision / recall in [0, 1] and
P <= 1 / R consistent with |predictions| <= k."""
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_ref", "main_dropin")

# process.js:5-8 (the reference's log parser)
RX = re.compile(r"^\{\-(.+?)\/\+(.+?) batchf, (.+?) threads\} -> \{(.+?)ms, (.+?)ms scoring, (.+?) precision, "
                r"(.+?) recall\} (\w+)$")
METRICS = ["CommonNeighbors", "JaccardCoefficient", "SorensenIndex", "SaltonCosineSimilarity", "HubPromoted",
           "HubDepressed", "LeichtHolmeNermanScore", "AdamicAdarCoefficient", "ResourceAllocationScore"]
HUBS = [0, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024]


@pytest.mark.timeout(300)
def test_gpu_reference_main_runs_on_the_dropin_header(nlp, tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.skip("oracle/_ref/main_dropin not built (needs the reference headers in the build container)")
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_golden import chung_lu_mtx
    mtx = str(tmp_path / "g.mtx")
    chung_lu_mtx(mtx, 3000, 20000, 0.6, 3)
    r = subprocess.run([EXE, mtx, "0", "0"], capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    assert re.search(r"\(removeSelfLoops\)", r.stdout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{-")]
    assert len(lines) == 9 * 11
    for i, ln in enumerate(lines):
        m = RX.match(ln)
        assert m, ln
        want = "predictLinks%sOmp%d" % (METRICS[i // 11], HUBS[i % 11])
        assert m.group(8) == want
        p, rc = float(m.group(6)), float(m.group(7))
        assert 0 <= p <= 1 and 0 <= rc <= 1
        assert float(m.group(4)) >= 0 and float(m.group(5)) >= 0
