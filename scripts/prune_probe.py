"""Group pruning diagnostics (cwq_prune.hip): a clustered two-level tree, one batch and one
one-query Fast call with CWQ_PRUNE_DEBUG=1 (bounds, thresholds, pair counts on stderr),
then pruned vs unpruned vs exact-scan results and times.
    python scripts/prune_probe.py [--n 60000 --dim 128 --clusters 150 --nq 256]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=60_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--clusters", type=int, default=150)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--k", type=int, default=10)
    a = ap.parse_args()
    pkg = cobweb_pkg.load()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(51)
    C = 2.0 * torch.randn((a.clusters, a.dim), generator=g, device="cuda:0")
    lab = torch.randint(0, a.clusters, (a.n,), generator=g, device="cuda:0")
    X = (C[lab] + 0.3 * torch.randn((a.n, a.dim), generator=g, device="cuda:0")).contiguous()
    h = a.nq // 2
    Q = torch.cat([X[:h] + 0.05 * torch.randn((h, a.dim), generator=g, device="cuda:0"),
                   C[torch.randint(0, a.clusters, (a.nq - h,), generator=g, device="cuda:0")] +
                   0.3 * torch.randn((a.nq - h, a.dim), generator=g, device="cuda:0")]).contiguous()
    t = pkg.synth.two_level_synth(X, lab)
    ix = pkg.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    print("filter", ix.filter_info(), flush=True)
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, a.k)
    ix.set_filter(-1)
    os.environ["CWQ_PRUNE_DEBUG"] = "1"
    ids1, s1 = ix.score_topk(Q, a.k)
    torch.cuda.synchronize()
    print("batch", ix.last_prune_stats(), ix.last_stats(), "== exact", torch.equal(ids0, ids1) and torch.equal(s0, s1),
          flush=True)
    ids2, s2 = ix.score_topk(Q[:1].contiguous(), a.k)
    torch.cuda.synchronize()
    print("nq=1", ix.last_prune_stats(), ix.last_stats(), "== exact", torch.equal(ids0[:1], ids2), flush=True)
    del os.environ["CWQ_PRUNE_DEBUG"]
    for mode in ("0", None, "0", None):
        if mode:
            os.environ["CWQ_GROUP_PRUNE"] = mode
        else:
            os.environ.pop("CWQ_GROUP_PRUNE", None)
        for nq in (a.nq, 1, 64):
            q = Q[:nq].contiguous()
            ix.score_topk(q, a.k)
            torch.cuda.synchronize()
            ts = []
            for _ in range(20):
                t0 = time.perf_counter()
                ix.score_topk(q, a.k)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            print(f"prune {'off' if mode else 'on '} nq {nq}: {ts[10] * 1e6:.1f} us  {ix.last_prune_stats()}", flush=True)


if __name__ == "__main__":
    main()
