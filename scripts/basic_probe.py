"""Throughput of the Basic query (best-first categorize, A4: `CobwebIndex.categorize`) and
of all-leaf rank scores (A8) on synthetic trees: flat-synth N x D or root -> G random
clusters -> leaves.  Prints ms per call and queries/s, plus the fraction of queries the
heap replay resolved without the dense re-run.  GPU only.

    python scripts/basic_probe.py --n 1000000 --dim 768 --queries 2000 --clusters 1024
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--queries", type=int, default=2000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--clusters", type=int, default=0)
    ap.add_argument("--balanced", default=None, help="B,L: a depth-L tree of branching B (synth.balanced_synth)")
    ap.add_argument("--rank-queries", type=int, default=64)
    ap.add_argument("--max-nodes", type=int, default=100_000,
                    help="categorize max_nodes (the wrapper's max_init_search); raise it so found-k = 1")
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    dev = torch.device("cuda", 0)
    X = pkg.synth.synthetic_corpus(args.n, args.dim, seed=0, device=dev)
    if args.balanced:
        b, lv = (int(v) for v in args.balanced.split(","))
        fs = pkg.synth.balanced_synth(X, b, lv)
    elif args.clusters:
        g = torch.Generator(device=dev)
        g.manual_seed(7)
        labels = torch.randint(0, args.clusters, (args.n,), generator=g, device=dev)
        fs = pkg.synth.two_level_synth(X, labels)
    else:
        fs = pkg.synth.flat_synth(X)
    ix = pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device=dev)
    del fs
    Q, _ = pkg.synth.synthetic_queries(X, args.queries, seed=1)
    del X
    torch.cuda.empty_cache()
    tree = (f"balanced {args.balanced}" if args.balanced else f"two-level G={args.clusters}" if args.clusters
            else "flat")
    dt, (nodes, found, calls) = timed(lambda: ix.categorize(Q, args.k, args.max_nodes), args.reps)
    ok = float((found == args.k).float().mean())
    print(f"categorize ({tree}, {args.n}x{args.dim}, k={args.k}, max_nodes={args.max_nodes}): {dt * 1e3:.2f} ms per "
          f"{args.queries} queries  {args.queries / dt:.0f} q/s  found-k fraction {ok:.3f}  mean log_prob calls "
          f"{float(calls.float().mean()):.0f}  resolved {ix.last_categorize_stats()}", flush=True)
    Qr = Q[:args.rank_queries]
    dt, out = timed(lambda: ix.rank_scores(Qr), args.reps)
    print(f"rank_scores ({tree}): {dt * 1e3:.2f} ms per {Qr.shape[0]} queries  {Qr.shape[0] / dt:.0f} q/s  "
          f"output {tuple(out.shape)}", flush=True)


if __name__ == "__main__":
    main()
