"""A/B of the isotropic-row strategies at the bench workload (flat-synth N x D,
Q queries, k): exact fp32 scan (filter 0) vs bf16-MFMA filter + exact rerank
(filter 1).  Prints wall time per call, phase timings, fallback counts and whether
ids/scores are bit-identical.  GPU only.

    python scripts/filter_probe.py --n 1000000 --dim 768 --queries 10000
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--queries", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="0,1")
    ap.add_argument("--clusters", type=int, default=0, help="0: flat tree; G: root -> G random clusters -> leaves")
    ap.add_argument("--balanced", default=None, help="B,L: a depth-L tree of branching B (synth.balanced_synth)")
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    dev = torch.device("cuda", 0)
    X = pkg.synth.synthetic_corpus(args.n, args.dim, seed=0, device=dev)
    if args.balanced:
        b, lv = (int(v) for v in args.balanced.replace("x", ",").split(","))
        fs = pkg.synth.balanced_synth(X, b, lv)
        print(f"balanced tree: branching {b}, depth {lv}: {fs['n_internal']} internal nodes", flush=True)
    elif args.clusters:
        g = torch.Generator(device=dev)
        g.manual_seed(7)
        labels = torch.randint(0, args.clusters, (args.n,), generator=g, device=dev)
        fs = pkg.synth.two_level_synth(X, labels)
    else:
        fs = pkg.synth.flat_synth(X)
    ix = pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device=dev)
    print(f"filter rows {ix.filter_info()}; cut {ix.cut_info()}", flush=True)
    del fs
    Q, _ = pkg.synth.synthetic_queries(X, args.queries, seed=1)
    del X
    torch.cuda.empty_cache()
    res = {}
    for mode in [int(m) for m in args.modes.split(",")]:
        ix.set_filter(mode)
        ids, sc = ix.score_topk(Q, args.k)          # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            ids, sc = ix.score_topk(Q, args.k)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        st = ix.last_stats()
        ix.set_timing(True)
        ix.score_topk(Q, args.k)
        tm = ix.last_timing()
        ix.set_timing(False)
        res[mode] = (ids.cpu(), sc.cpu())
        print(f"mode {mode}: {dt * 1e3:.2f} ms/call  {args.queries / dt:.0f} q/s  stats {st}  timing "
              f"{ {k: round(v, 3) for k, v in tm.items()} }", flush=True)
    if 0 in res and 1 in res:
        print("ids equal:", torch.equal(res[0][0], res[1][0]), " scores equal:", torch.equal(res[0][1], res[1][1]),
              flush=True)


if __name__ == "__main__":
    main()
