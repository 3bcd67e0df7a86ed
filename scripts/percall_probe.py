"""Per-call latency of the Fast query at small batch sizes -- the reference harness's
mode: `evaluate_retrieval` times one `cobweb_predict_fast(q, k)` per query
(benchmark_utils.py:801-805).  For nq in --nq, times `CobwebIndex.score_topk` per call
(host sync after every call, like the harness) with each isotropic-row strategy, and
reports us/call and the HBM bandwidth implied by the bytes one pass must read
(fp32 leaf means 4*N*D, or the bf16 filter operand 2*N*D).  GPU only.

    python scripts/percall_probe.py --n 1000000 --dim 768 --nq 1,8,64
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
    ap.add_argument("--nq", default="1,8,64,256")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--modes", default="0,-1,1")
    ap.add_argument("--wrapper", action="store_true", help="also time the drop-in cobweb_predict_fast(q, k)")
    ap.add_argument("--balanced", default=None, help="B,L (or BxL): a depth-L tree of branching B (synth.balanced_synth)")
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    dev = torch.device("cuda", 0)
    X = pkg.synth.synthetic_corpus(args.n, args.dim, seed=0, device=dev)
    if args.balanced:
        b, L = (int(v) for v in args.balanced.replace("x", ",").split(","))   # "4,9" or "4x9"
        fs = pkg.synth.balanced_synth(X, b, L, seed=1)
    else:
        fs = pkg.synth.flat_synth(X)
    ix = pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device=dev)
    del fs
    Q, _ = pkg.synth.synthetic_queries(X, max(int(v) for v in args.nq.replace("+", ",").split(",")), seed=1)
    del X
    torch.cuda.empty_cache()
    fp32_bytes = 4.0 * args.n * args.dim
    bf16_bytes = 2.0 * args.n * args.dim
    ref = {}
    for nq in [int(v) for v in args.nq.replace("+", ",").split(",")]:
        q = Q[:nq].contiguous()
        for mode in [int(m) for m in args.modes.split(",")]:
            ix.set_filter(mode)
            ids, sc = ix.score_topk(q, args.k)
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                ids, sc = ix.score_topk(q, args.k)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            med = ts[len(ts) // 2]
            st = ix.last_stats()
            same = ""
            if nq in ref:
                same = " ids==exact" if torch.equal(ref[nq][0], ids) and torch.equal(ref[nq][1], sc) else " DIFF"
            if mode == 0:
                ref[nq] = (ids.clone(), sc.clone())
            print(f"n={args.n} d={args.dim} nq={nq:5d} mode={mode:2d} filter_used={int(st['filter_used'])}: "
                  f"median {med * 1e6:9.1f} us/call  min {ts[0] * 1e6:9.1f}  {nq / med:10.0f} q/s  "
                  f"fp32-pass {fp32_bytes / med / 1e9:7.0f} GB/s  bf16-pass {bf16_bytes / med / 1e9:7.0f} GB/s{same}",
                  flush=True)
        ix.set_filter(-1)
    print("done", flush=True)


if __name__ == "__main__":
    main()
