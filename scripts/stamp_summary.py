"""Summarise FG_STAMP s_memtime stamps (diagnostic builds): per stage, for the wave of
group 0 and of group 1 on one SIMD: memory section (t1-t0), barrier wait into the compute
section (t2-t1), compute issue (t3-t2), barrier wait out (t4-t3); cycles."""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64)[:16 * 2 * 2 * 32 * 6].reshape(16, 2, 2, 32, 6).astype(np.int64)
ok = (a[..., 0] > 0) & (a[..., 4] > 0)
for g in range(2):
    sel = a[:, :, g][ok[:, :, g]]
    d = np.diff(sel, axis=-1)
    per = np.diff(sel[:, 0])
    print(f"group {g}: n={len(sel)}  mem {np.median(d[:, 0]):.0f}  wait-in {np.median(d[:, 1]):.0f}  "
          f"mfma {np.median(d[:, 2]):.0f}  wait-out {np.median(d[:, 3]):.0f}  (median cycles; total "
          f"{np.median(d.sum(-1)):.0f})")

# per-tile stamps (wave 0 of workgroups 0..63, tiles 0..15): setup, K loop, epilogue, gap
t = np.fromfile(sys.argv[1], dtype=np.uint64)[16384:16384 + 64 * 64].reshape(64, 16, 4).astype(np.int64)
okt = (t[..., 0] > 0) & (t[..., 3] > 0)
sel = t[okt]
if len(sel):
    d = np.diff(sel, axis=-1)
    gap = (t[:, 1:, 0] - t[:, :-1, 3])[okt[:, 1:] & okt[:, :-1]]
    tot = np.median(d.sum(-1)) + (np.median(gap) if len(gap) else 0)
    print(f"tiles: n={len(sel)}  setup {np.median(d[:, 0]):.0f}  K loop {np.median(d[:, 1]):.0f}  "
          f"epilogue {np.median(d[:, 2]):.0f}  gap to next {np.median(gap) if len(gap) else 0:.0f}  "
          f"(median s_memtime ticks; K loop share {np.median(d[:, 1]) / tot:.3f})")
