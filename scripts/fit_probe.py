"""GPU ifit (add path) throughput: inserts/s of CobwebWrapper's
incremental fit (CU scoring on libcwq, host-driven operation choice) for N(0,I) data
(a flat tree: every insert scores all root children, the reference's O(N^2 D) case)
and clustered data (hierarchical trees).  GPU only.

    python scripts/fit_probe.py --n 2000 --dim 768 --clusters 0
"""
import argparse
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def depth_stats(root):
    n, mx, stack = 0, 0, [(root, 0)]
    nint = 0
    while stack:
        x, d = stack.pop()
        n += 1
        mx = max(mx, d)
        if x.children:
            nint += 1
        stack.extend((c, d + 1) for c in x.children)
    return n, nint, mx, len(root.children)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--clusters", type=int, default=0, help="0: X ~ N(0,I); else Gaussian clusters (sd 0.3)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--host", action="store_true", help="the host-driven fitter (CWQ_FIT_DEVICE=0)")
    args = ap.parse_args()
    if args.host:
        os.environ["CWQ_FIT_DEVICE"] = "0"
    pkg = cobweb_pkg.load()
    rng = np.random.default_rng(args.seed)
    if args.clusters:
        C = rng.standard_normal((args.clusters, args.dim)).astype(np.float32) * 2.0
        X = (C[rng.integers(0, args.clusters, args.n)] +
             0.3 * rng.standard_normal((args.n, args.dim))).astype(np.float32)
    else:
        X = rng.standard_normal((args.n, args.dim)).astype(np.float32)
    random.seed(args.seed)
    w = pkg.CobwebWrapper(corpus=None, corpus_embeddings=X[:8])   # warm up libcwq + the device pool
    torch.cuda.synchronize()
    random.seed(args.seed)
    t0 = time.perf_counter()
    w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(args.n)], corpus_embeddings=X)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n, nint, mx, rootc = depth_stats(w.tree.root)
    mode = "host-driven" if args.host else "device-resident"
    print(f"ifit ({mode}) n={args.n} d={args.dim} clusters={args.clusters}: {dt:.2f} s  {args.n / dt:.0f} inserts/s  "
          f"{1e3 * dt / args.n:.2f} ms/insert  tree: {n} nodes ({nint} internal), depth {mx}, root children {rootc}",
          flush=True)


if __name__ == "__main__":
    main()
