"""Basic one query per call on the bench's flat-synth tree (root -> N leaves), host memory in
and out (cwq_categorize_host, the harness's call shape): median latency; run under the
timeline step of gpu_run.sh for a kernel breakdown.  GPU only."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--calls", type=int, default=30)
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    X = pkg.synth.synthetic_corpus(args.n, args.dim, seed=0, device=torch.device("cuda", 0))
    t = pkg.synth.flat_synth(X)
    ix = pkg.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    Q, _ = pkg.synth.synthetic_queries(X, args.calls, seed=1)
    Qh = Q.cpu().numpy().astype(np.float32)
    del X, t
    ts = []
    for i in range(args.calls):
        t0 = time.perf_counter()
        nodes, found, calls = ix.categorize_host(Qh[i:i + 1], args.k, 100000)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"flat {args.n}x{args.dim} Basic per call (categorize_host, k={args.k}): median {ts[len(ts) // 2] * 1e6:.1f} us; "
          f"found {int(found[0])}, calls {int(calls[0])}; stats {ix.last_categorize_stats()}", flush=True)
    print("done", flush=True)


if __name__ == "__main__":
    main()
