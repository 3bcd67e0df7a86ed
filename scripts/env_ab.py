"""In-process A/B of run-time knobs (environment variables read per call) on the Fast
path: the variants run interleaved, round after round, in ONE process on one tree, and
each call's fgemm time (HIP events) and wall time are recorded; ids/scores of every
variant are compared with the first.  GPU only.

    python scripts/env_ab.py --variants "CWQ_FG_QG=8;CWQ_FG_QG=4" --rounds 5
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def parse(v):
    env = {}
    for item in v.split("&"):
        item = item.strip()
        if item:
            key, val = item.split("=", 1)
            env[key] = val
    return env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--queries", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", required=True, help="';'-separated variants of '&'-separated KEY=VAL")
    args = ap.parse_args()
    variants = [parse(v) for v in args.variants.split(";")]
    keys = sorted({k for v in variants for k in v})
    pkg = cobweb_pkg.load()
    dev = torch.device("cuda", 0)
    X = pkg.synth.synthetic_corpus(args.n, args.dim, seed=0, device=dev)
    fs = pkg.synth.flat_synth(X)
    ix = pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device=dev)
    del fs
    Q, _ = pkg.synth.synthetic_queries(X, args.queries, seed=1)
    del X
    torch.cuda.empty_cache()

    def setenv(v):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(v)

    ref = None
    wall = [[] for _ in variants]
    fg = [[] for _ in variants]
    for vi, v in enumerate(variants):   # warm-up + equality check
        setenv(v)
        ids, sc = ix.score_topk(Q, args.k)
        torch.cuda.synchronize()
        if ref is None:
            ref = (ids.cpu(), sc.cpu())
        else:
            print(f"variant {v}: ids equal {torch.equal(ref[0], ids.cpu())} scores equal {torch.equal(ref[1], sc.cpu())}",
                  flush=True)
    for r in range(args.rounds):
        for vi, v in enumerate(variants):
            setenv(v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                ix.score_topk(Q, args.k)
            torch.cuda.synchronize()
            wall[vi].append((time.perf_counter() - t0) / args.reps * 1e3)
            ix.set_timing(True)
            ix.score_topk(Q, args.k)
            fg[vi].append(ix.last_timing().get("fgemm_ms", float("nan")))
            ix.set_timing(False)
        print(f"round {r}: " + "  ".join(f"{wall[i][-1]:.2f}/{fg[i][-1]:.2f}" for i in range(len(variants))), flush=True)
    for vi, v in enumerate(variants):
        print(f"{v}: call ms median {statistics.median(wall[vi]):.3f} min {min(wall[vi]):.3f}; "
              f"fgemm ms median {statistics.median(fg[vi]):.3f} min {min(fg[vi]):.3f}", flush=True)


if __name__ == "__main__":
    main()
