"""In-process A/B of run-time knobs on the per-call path (one score_topk call of --nq queries
at a time, host sync after each, as the reference harness): variants interleaved round
after round in ONE process on one tree; per variant the median us/call, the stream
filter's candidates and exact reranks per query, and whether ids/scores equal the first
variant's.  GPU only.

    python scripts/percall_ab.py --variants "CWQ_STREAM_I8=0;CWQ_STREAM_I8=1" --calls 200
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
    return dict(item.strip().split("=", 1) for item in v.split("&") if item.strip())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--nq", type=int, default=1)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--balanced", default=None, help="B,L: a depth-L tree of branching B (synth.balanced_synth)")
    ap.add_argument("--variants", required=True, help="';'-separated variants of '&'-separated KEY=VAL")
    args = ap.parse_args()
    variants = [parse(v) for v in args.variants.split(";")]
    keys = sorted({k for v in variants for k in v})
    pkg = cobweb_pkg.load()
    dev = torch.device("cuda", 0)
    X = pkg.synth.synthetic_corpus(args.n, args.dim, seed=0, device=dev)
    if args.balanced:
        b, L = (int(v) for v in args.balanced.replace("x", ",").split(","))
        fs = pkg.synth.balanced_synth(X, b, L, seed=1)
    else:
        fs = pkg.synth.flat_synth(X)
    ix = pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device=dev)
    del fs
    Q, _ = pkg.synth.synthetic_queries(X, args.calls * args.nq, seed=1)
    del X
    torch.cuda.empty_cache()
    batches = [Q[i * args.nq:(i + 1) * args.nq].contiguous() for i in range(args.calls)]

    def setenv(v):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(v)

    def run_all():
        ids, sc, cand, ex = [], [], [], []
        for qb in batches:
            i, s = ix.score_topk(qb, args.k)
            st = ix.last_stats()
            ids.append(i)
            sc.append(s)
            cand.append(st["candidates"])
            ex.append(st["exact_reranks"])
        torch.cuda.synchronize()
        return torch.cat(ids).cpu(), torch.cat(sc).cpu(), cand, ex, st

    ref = None
    for v in variants:   # warm-up (builds what a variant builds) + equality check
        setenv(v)
        ids, sc, cand, ex, st = run_all()
        line = (f"variant {v}: path {st['path']} candidates/query median {statistics.median(cand)} max {max(cand)}; "
                f"exact reranks/query median {statistics.median(ex)} max {max(ex)}; fallbacks {st['fallback_queries']}")
        if ref is None:
            ref = (ids, sc)
        else:
            line += f"; ids equal {torch.equal(ref[0], ids)} scores equal {torch.equal(ref[1], sc)}"
        print(line, flush=True)
    us = [[] for _ in variants]
    for r in range(args.rounds):
        for vi, v in enumerate(variants):
            setenv(v)
            torch.cuda.synchronize()
            t = []
            for qb in batches:
                t0 = time.perf_counter()
                ix.score_topk(qb, args.k)
                torch.cuda.synchronize()
                t.append((time.perf_counter() - t0) * 1e6)
            us[vi].append(statistics.median(t))
        print(f"round {r}: " + "  ".join(f"{us[i][-1]:.1f}" for i in range(len(variants))), flush=True)
    for vi, v in enumerate(variants):
        print(f"{v}: us/call median {statistics.median(us[vi]):.1f} min {min(us[vi]):.1f}", flush=True)


if __name__ == "__main__":
    main()
