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
