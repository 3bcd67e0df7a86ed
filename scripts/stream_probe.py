"""Phase timings (HIP events) of the small-batch stream path at C3 for a few batch sizes.
GPU only.   python scripts/stream_probe.py --nq 1,16,64"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--nq", default="1,16,64")
    ap.add_argument("--k", type=int, default=10)
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    X = pkg.synth.synthetic_corpus(args.n, args.dim, seed=0, device="cuda:0")
    fs = pkg.synth.flat_synth(X)
    ix = pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device="cuda:0")
    del fs
    Q, _ = pkg.synth.synthetic_queries(X, 64, seed=1)
    del X
    torch.cuda.empty_cache()
    nl = ix.info["leaf_rows"]
    for nq in [int(v) for v in args.nq.split(",")]:
        q = Q[:nq].contiguous()
        for _ in range(3):
            ix.score_topk(q, args.k)
        ix.set_timing(True)
        tms = []
        for _ in range(10):
            ix.score_topk(q, args.k)
            tms.append(ix.last_timing())
        ix.set_timing(False)
        st = ix.last_stats()
        med = {k: sorted(t[k] for t in tms)[5] for k in tms[0]}
        gbs = nl * (2 * args.dim + 32) / (med["fgemm_ms"] * 1e-3) / 1e9
        print(f"nq={nq:3d} path={st['path']} call {med['call_ms']:.3f} ms: internal {med['internal_ms']:.3f} "
              f"probe {med['sample_ms']:.3f} filter {med['fgemm_ms']:.3f} ({gbs:.0f} GB/s) rerank {med['rerank_ms']:.3f} "
              f"merge+expand+flags {med['merge_ms']:.3f}  cand/q {st['candidates']} exact/q {st['exact_reranks']} "
              f"probe rows {st['sample_rows']}", flush=True)


if __name__ == "__main__":
    main()
