"""Summarise NLP_STAMP phase stamps (s_memrealtime, 100 MHz) of the last call.

    NLP_STAMP=gpurun_out/st.bin python bench.py ...
    python tools/stamps.py gpurun_out/st.bin [nphases]
"""
import sys

import numpy as np

rec = 8 * 65536
a = np.fromfile(sys.argv[1], dtype=np.uint64)
nph = int(sys.argv[2]) if len(sys.argv) > 2 else 8
CLOCK = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else []  # slots holding sp_clock
last = a[-rec:].reshape(65536, 8)[:, :nph].astype(np.int64)
blocks = last[last[:, 0] != 0]
# phases stamped by at least one block, in time order; each step over the
# blocks that stamped both of its phases (early-exit blocks stamp fewer)
ok = [i for i in range(nph) if (blocks[:, i] != 0).any() and i not in CLOCK]
ok.sort(key=lambda i: blocks[blocks[:, i] != 0, i].mean() - blocks[blocks[:, i] != 0, 0].mean())
t0 = blocks[:, 0].min()
full = (blocks[:, ok] != 0).all(axis=1)
print("blocks %d (%d stamped every phase), phases %s" % (len(blocks), full.sum(), ok))
print("start offset: mean %.2f us max %.2f us" % ((blocks[:, 0] - t0).mean() / 100, (blocks[:, 0] - t0).max() / 100))
for i, j in zip(ok, ok[1:]):
    both = (blocks[:, i] != 0) & (blocks[:, j] != 0)
    d = (blocks[both, j] - blocks[both, i]) / 100.0
    print("phase %d->%d (%d blocks): mean %.2f us  p50 %.2f  max %.2f" % (i, j, both.sum(), d.mean(), np.median(d), d.max()))
last = blocks[:, ok][blocks[:, ok] != 0].max()
if CLOCK and (blocks[:, CLOCK] != 0).all(axis=1).any():  # sp_clock pair: shader clock rate
    c = (blocks[:, CLOCK] != 0).all(axis=1) & (blocks[:, 4] != 0)
    f = (blocks[c, 7] - blocks[c, 6]) / ((blocks[c, 4] - blocks[c, 0]) / 100.0)
    print("shader clock: mean %.0f MHz  min %.0f  max %.0f" % (f.mean(), f.min(), f.max()))
print("span %.2f us" % ((last - t0) / 100))
if nph > 7 and 7 in ok and 0 in ok:
    d = (blocks[:, 0] - blocks[:, 7]) / 100.0
    e0 = blocks[:, 7].min()
    print("entry (phase 7) -> phase 0: mean %.2f us max %.2f; entry spread %.2f us; entry -> last end %.2f us"
          % (d.mean(), d.max(), (blocks[:, 7].max() - e0) / 100, (blocks[:, ok[-2] if ok[-1] == 7 else ok[-1]].max() - e0) / 100))
