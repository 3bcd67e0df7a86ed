"""Diagnostic: categorize on a flat D=32 tree -- list keys, root bottleneck, how queries
resolve (count / replay / DENSE).  GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402

pkg = cobweb_pkg.load()
X = pkg.synth.synthetic_corpus(30_000, 32, seed=31)
t = pkg.synth.flat_synth(X)
ix = pkg.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
Q, _ = pkg.synth.synthetic_queries(X, 300, seed=32)
for filt in (-1, 0):
    ix.set_filter(filt)
    for k in (10, 64):
        nodes, found, calls = ix.categorize(Q, k)
        torch.cuda.synchronize()
        print("filter", filt, "k", k, ix.last_categorize_stats(), "found", found[:6].tolist(), "calls", calls[:6].tolist(),
              flush=True)
lp = ix.node_logprob(Q[:4], full=True)
print("root lp", lp[:, 0].tolist())
top = torch.topk(lp[:, 1:], 12, dim=1)
print("top leaf lp", top.values[:, :12].tolist())
