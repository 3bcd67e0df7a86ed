"""rank_scores (A8) timing: all-sentence scores for nq queries over the flat-synth
C3 tree (1M x 768), like cobweb_rank_scores (CobwebWrapper.py:267-294).  GPU only.

    python scripts/rank_probe.py --n 1000000 --nq 16,64,256
    python scripts/rank_probe.py --libs rag-cobweb_amd/libcwq_base.so,rag-cobweb_amd/libcwq.so
        (A/B of library builds in one process, rounds interleaved; outputs compared bitwise)
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
    ap.add_argument("--nq", default="16,64,256")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--libs", default="", help="comma-separated libcwq builds to A/B")
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    dev = torch.device("cuda", 0)
    X = pkg.synth.synthetic_corpus(args.n, args.dim, seed=0, device=dev)
    fs = pkg.synth.flat_synth(X)
    Q, _ = pkg.synth.synthetic_queries(X, max(int(v) for v in args.nq.split(",")), seed=1)
    del X
    if args.libs:
        L = pkg._lib
        arms = []
        for path in args.libs.split(","):
            L._lib = L.load_library(os.path.abspath(path))
            arms.append((os.path.basename(path), L._lib, pkg.index.CobwebIndex(
                fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device=dev)))
        del fs
        torch.cuda.empty_cache()
        for nq in [int(v) for v in args.nq.split(",")]:
            q = Q[:nq].contiguous()
            ts = {a[0]: [] for a in arms}
            ref = None
            for r in range(args.reps + 1):
                for name, lib, ix in arms:
                    L._lib = lib
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    out = ix.rank_scores(q)
                    torch.cuda.synchronize()
                    if r:
                        ts[name].append(time.perf_counter() - t0)
                    if ref is None:
                        ref = out.clone()
                    elif not torch.equal(ref, out):
                        print(f"MISMATCH {name} nq={nq}", flush=True)
                    del out
            print(f"nq={nq}: " + "  ".join(f"{n} {sorted(v)[len(v) // 2] * 1e3:.3f} ms" for n, v in ts.items()),
                  flush=True)
        print("done", flush=True)
        return
    ix = pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device=dev)
    del fs
    torch.cuda.empty_cache()
    for nq in [int(v) for v in args.nq.split(",")]:
        q = Q[:nq].contiguous()
        out = ix.rank_scores(q)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            out = ix.rank_scores(q)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        med = sorted(ts)[len(ts) // 2]
        fl = 4.0 * args.n * args.dim * nq
        print(f"rank_scores n={args.n} d={args.dim} nq={nq}: {med * 1e3:.3f} ms  {nq / med:.0f} q/s  "
              f"{fl / med / 1e12:.1f} TFLOP/s (4*N*D per query)  out {out.numel() * 4 / 1e9:.2f} GB", flush=True)
        del out
    print("done", flush=True)


if __name__ == "__main__":
    main()
