"""Summarise NLP_STAMP phase stamps (s_memrealtime, 100 MHz) of the last call.

    NLP_STAMP=gpurun_out/st.bin NLP_HOT_STAGE=5 python bench.py ...
    python tools/stamps.py gpurun_out/st.bin [nphases]
"""
import sys

import numpy as np

rec = 8 * 65536
a = np.fromfile(sys.argv[1], dtype=np.uint64)
nph = int(sys.argv[2]) if len(sys.argv) > 2 else 8
last = a[-rec:].reshape(65536, 8)[:, :nph].astype(np.int64)
blocks = last[last[:, 0] != 0]
# phases that were stamped by every block
ok = [i for i in range(nph) if (blocks[:, i] != 0).all()]
ok.sort(key=lambda i: blocks[:, i].mean())  # phases in time order
t0 = blocks[:, 0].min()
print("blocks %d, phases stamped %s" % (len(blocks), ok))
print("start offset: mean %.2f us max %.2f us" % ((blocks[:, 0] - t0).mean() / 100, (blocks[:, 0] - t0).max() / 100))
for i, j in zip(ok, ok[1:]):
    d = (blocks[:, j] - blocks[:, i]) / 100.0
    print("phase %d->%d: mean %.2f us  p50 %.2f  max %.2f" % (i, j, d.mean(), np.median(d), d.max()))
print("span %.2f us" % ((blocks[:, ok[-1]].max() - t0) / 100))
if nph > 7 and 7 in ok and 0 in ok:
    d = (blocks[:, 0] - blocks[:, 7]) / 100.0
    e0 = blocks[:, 7].min()
    print("entry (phase 7) -> phase 0: mean %.2f us max %.2f; entry spread %.2f us; entry -> last end %.2f us"
          % (d.mean(), d.max(), (blocks[:, 7].max() - e0) / 100, (blocks[:, ok[-2] if ok[-1] == 7 else ok[-1]].max() - e0) / 100))
