"""Pretest survival of the batch filter with bf16 vs int8 row/query splits (VERDICT r3 #3:
"measure the pretest survival per 16x64 block before writing the epilogue").

CPU model of the certified bound of fgemm_kernel (cwq_mfma.hip fg_bounds2) on the C3
workload's distribution (X ~ N(0,I), 768-d, half perturbed / half fresh queries), on a
row subset: per (query, row) the squared distance S and the bound's half-width in S units
  bf16: 2 (|x_hi| beta + |x_lo| delta),  beta = |mu_lo| + gamma |mu_hi|, delta = |mu_hi| + |mu_lo|
  int8: 2 (|x_q| beta8 + |x_r| delta8) + 2^-21 |x'.mu'|   (per-row / per-query scale s = max|v|/127,
        the split v = s q + r formed exactly -- the per-call int8 pass)
A row survives the filter when S - w <= S_(K) + w_(K) -- the threshold after tightening is
the K-th best upper bound of the candidates (in S units).  K is scaled to the subset so
that the survivors per query estimate the full 1M-row case.  Reported: survivors per
query (x 1M / rows) and the fraction of 16-query x 64-row MFMA blocks holding a survivor
(the blocks whose epilogue leaves the one-max-per-element fast path).

    python scripts/i8_batch_survival.py [--rows 262144] [--queries 256]
"""
import argparse

import numpy as np


def bf16_split(v):
    """hi = bf16(v) (round to nearest even on the top 16 bits of fp32), lo = v - hi."""
    u = v.astype(np.float32).view(np.uint32)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    hi = r.view(np.float32)
    return hi, (v - hi).astype(np.float32)


def i8_split(v):
    s = np.abs(v).max(axis=1, keepdims=True) / 127.0
    q = np.clip(np.rint(v / s), -127, 127)
    hi = s * q
    return hi, v - hi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=262_144)
    ap.add_argument("--queries", type=int, default=256)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--full", type=int, default=1_000_000)
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    N, Q, D = args.rows, args.queries, args.dim
    X = rng.standard_normal((N, D), dtype=np.float32)
    c = X.mean(0)
    Xc = X - c
    pick = rng.choice(N, Q // 2, replace=False)
    qs = np.concatenate([X[pick] + 0.1 * rng.standard_normal((Q // 2, D), dtype=np.float32),
                         rng.standard_normal((Q - Q // 2, D), dtype=np.float32)]) - c
    K = max(1, int(round(args.k * N / args.full)))   # the subset's K-th ~ the full set's k-th
    gamma = (D + 64) * 2.0 ** -23
    out = {}
    dots = qs.astype(np.float64) @ Xc.astype(np.float64).T
    S = (qs.astype(np.float64) ** 2).sum(1)[:, None] + (Xc.astype(np.float64) ** 2).sum(1)[None, :] - 2 * dots
    for name in ("bf16", "int8"):
        if name == "bf16":
            rh, rl = bf16_split(Xc)
            xh, xl = bf16_split(qs)
            beta = np.linalg.norm(rl, axis=1) + gamma * np.linalg.norm(rh, axis=1)
            extra = 0.0
        else:
            rh, rl = i8_split(Xc.astype(np.float64))
            xh, xl = i8_split(qs.astype(np.float64))
            beta = np.linalg.norm(rl, axis=1)
            extra = 2.0 ** -21 * np.abs(dots)
        delta = np.linalg.norm(rh, axis=1) + np.linalg.norm(rl, axis=1)
        w = 2 * (np.linalg.norm(xh, axis=1)[:, None] * beta[None, :] +
                 np.linalg.norm(xl, axis=1)[:, None] * delta[None, :]) + 2 * extra
        ub = S + w
        thr = np.partition(ub, K - 1, axis=1)[:, K - 1]          # K-th best upper bound (S units)
        surv = (S - w) <= thr[:, None]
        per_q = surv.sum(1) * (args.full / N)
        nb_q, nb_r = Q // 16, N // 64
        blocks = surv[:nb_q * 16, :nb_r * 64].reshape(nb_q, 16, nb_r, 64).any(axis=(1, 3))
        out[name] = (np.median(per_q), per_q.mean(), blocks.mean(), float(np.median(w)))
        print(f"{name}: survivors per query (scaled to {args.full} rows) median {out[name][0]:.0f} mean "
              f"{out[name][1]:.0f}; 16x64 blocks with a survivor {100 * out[name][2]:.2f}%; median half-width "
              f"{out[name][3]:.3f} (S units)", flush=True)
    print(f"int8 / bf16: survivors x{out['int8'][1] / out['bf16'][1]:.2f}, active blocks "
          f"x{out['int8'][2] / out['bf16'][2]:.2f}", flush=True)


if __name__ == "__main__":
    main()
