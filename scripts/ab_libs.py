"""In-process A/B of libcwq builds on the bench workload (flat-synth N x D, Q queries).

Each library gets its own index over the same data; the builds then run in
interleaved rounds (A B C A B C ...), so clock/DVFS drift hits every arm alike.
Reports per-arm median call time and median summed fgemm launch time, and checks
that every arm returns the same ids/scores.  GPU only.

    python scripts/ab_libs.py --libs rag-cobweb_amd/libcwq.so,rag-cobweb_amd/libcwq_b.so

An arm may carry run-time knobs: `lib.so@CWQ_FG_CUTS=32,128;CWQ_FG_SAMPLE_DIV=128` sets
those variables while that arm's index is built and while it runs (arms are separated
by spaces when knobs contain commas: pass --libs once per arm).
"""
import argparse
import contextlib
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


@contextlib.contextmanager
def env(kv):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True, action="append")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--queries", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--share-index", action="store_true",
                    help="one index for every arm (same library; knobs read per call only)")
    ap.add_argument("--clusters", type=int, default=0, help="0: flat tree; G: root -> G random clusters -> leaves")
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    L = pkg._lib
    dev = torch.device("cuda", 0)
    X = pkg.synth.synthetic_corpus(args.n, args.dim, seed=0, device=dev)
    if args.clusters:
        g = torch.Generator(device=dev)
        g.manual_seed(7)
        labels = torch.randint(0, args.clusters, (args.n,), generator=g, device=dev)
        fs = pkg.synth.two_level_synth(X, labels)
    else:
        fs = pkg.synth.flat_synth(X)
    Q, _ = pkg.synth.synthetic_queries(X, args.queries, seed=1)
    del X
    paths = args.libs[0].split(",") if len(args.libs) == 1 and "@" not in args.libs[0] else args.libs
    knobs = {}
    for p in paths:
        kv = p.split("@", 1)[1] if "@" in p else ""
        knobs[p] = dict(x.split("=", 1) for x in kv.split(";") if x)
    arms = []
    for p in paths:
        if args.share_index and arms:
            arms.append(arms[0])
            continue
        with env(knobs[p]):
            L._lib = L.load_library(os.path.abspath(p.split("@")[0]), strict=False)
            ix = pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device=dev)
            ix.set_filter(1)
            ix.score_topk(Q, args.k)
        arms.append(ix)
    del fs
    torch.cuda.empty_cache()
    call = {p: [] for p in paths}
    fg = {p: [] for p in paths}
    ref = None
    for r in range(args.rounds):
        for p, ix in zip(paths, arms):
            with env(knobs[p]):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ids, sc = ix.score_topk(Q, args.k)
                torch.cuda.synchronize()
                call[p].append((time.perf_counter() - t0) * 1e3)
                ix.set_timing(True)
                ix.score_topk(Q, args.k)
                fg[p].append(ix.last_timing()["fgemm_ms"])
                ix.set_timing(False)
                if ref is None:
                    ref = (ids.cpu(), sc.cpu())
                elif not (torch.equal(ref[0], ids.cpu()) and torch.equal(ref[1], sc.cpu())):
                    print(f"MISMATCH {p} round {r}", flush=True)
        print(f"round {r}: " + "  ".join(f"{os.path.basename(p)[:60]} {call[p][-1]:.2f}/{fg[p][-1]:.3f}" for p in paths),
              flush=True)
    base = statistics.median(fg[paths[0]])
    for p in paths:
        mc, mf = statistics.median(call[p]), statistics.median(fg[p])
        print(f"{os.path.basename(p)[:60]}: call {mc:.3f} ms ({args.queries / mc * 1e3:.0f} q/s)  fgemm {mf:.3f} ms "
              f"(x{base / mf:.3f} vs first)  min {min(fg[p]):.3f}", flush=True)


if __name__ == "__main__":
    main()
