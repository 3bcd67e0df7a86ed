"""Recall of the Fast top-k against fp64 brute force (exact L2 ranking) at a given
synthetic size; also reports the fp32-GEMM ground truth bench.py uses.  GPU only.

    python scripts/recall_check.py --n 10000000 --dim 1024 --queries 64
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--queries", type=int, default=64)
    ap.add_argument("--k", type=int, default=10)
    a = ap.parse_args()
    pkg = cobweb_pkg.load()
    dev = torch.device("cuda", 0)
    X = pkg.synth.synthetic_corpus(a.n, a.dim, seed=0, device=dev)
    fs = pkg.synth.flat_synth(X)
    ix = pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device=dev)
    del fs
    Q, tg = pkg.synth.synthetic_queries(X, a.queries, seed=1)
    ids, sc = ix.score_topk(Q, a.k)
    ids = ids.cpu()
    r64, r32, r3264 = 0.0, 0.0, 0.0
    xn = (X * X).sum(1)
    for i in range(a.queries):
        q = Q[i]
        d64 = torch.zeros(a.n, dtype=torch.float64, device=dev)
        for c in range(0, a.dim, 128):
            d64 += ((X[:, c:c + 128].double() - q[c:c + 128].double()) ** 2).sum(1)
        gt64 = torch.topk(-d64, a.k).indices.cpu()
        gt32 = torch.topk(-(xn - 2 * (X @ q)), a.k).indices.cpu()
        s_ours, s64, s32 = set(ids[i].tolist()), set(gt64.tolist()), set(gt32.tolist())
        r64 += len(s_ours & s64) / a.k
        r32 += len(s_ours & s32) / a.k
        r3264 += len(s32 & s64) / a.k
        if i < 4 and s_ours != s64:
            miss = sorted(s64 - s_ours)
            print(f"q{i}: ours-only {sorted(s_ours - s64)} d64 {[round(float(d64[j]), 4) for j in sorted(s_ours - s64)]}"
                  f" missed {miss} d64 {[round(float(d64[j]), 4) for j in miss]}", flush=True)
    n = a.queries
    print(f"N={a.n} D={a.dim}: recall vs fp64 L2 {r64 / n:.4f}; vs fp32-GEMM GT {r32 / n:.4f}; "
          f"fp32-GEMM GT vs fp64 {r3264 / n:.4f}", flush=True)


if __name__ == "__main__":
    main()
