"""The tree-adaptive cut on the synthetic broad-rooted trees of
tests/test_gpu_cut.py: cut shape, Fast batch / per-call times with the filter and pruning
stats, pruned vs unpruned vs depth-1 cut, == exact scan.  CWQ_PRUNE_DEBUG=1 prints the
first queries' KUB / threshold.
    python scripts/cut_probe.py --n 48000 --dim 96 --fan 8,4,6 [--k 10]
GPU only."""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cobweb_pkg  # noqa: E402
from test_gpu_cut import broad_tree  # noqa: E402


def med(f, reps):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def legs(ix, Q, k, tag):
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, k)
    t_scan = med(lambda: ix.score_topk(Q, k), 5)
    ix.set_filter(-1)
    for prune in ("0", "1"):
        os.environ["CWQ_GROUP_PRUNE"] = prune
        ids, sc = ix.score_topk(Q, k)
        same = torch.equal(ids, ids0) and torch.equal(sc, s0)
        t = med(lambda: ix.score_topk(Q, k), 7)
        st, ps = ix.last_stats(), ix.last_prune_stats()
        pc = {}
        for nq in (1, 64):
            ts = []
            for a in range(0, 64 if nq == 1 else 256, nq):
                q = Q[a:a + nq].contiguous()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ix.score_topk(q, k)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            pc[nq] = round(ts[len(ts) // 2] * 1e6, 1)
        print(f"[{tag}] prune={prune} batch {Q.shape[0]}: {t * 1e3:.3f} ms (exact scan {t_scan * 1e3:.3f}); == exact "
              f"{same}; cand {st['candidates']} reranks {st['exact_reranks']} fallback {st['fallback_queries']}; "
              f"prune {ps}; per call us {pc}", flush=True)
    os.environ.pop("CWQ_GROUP_PRUNE", None)


def basic(ix, Q, k, tag):
    ref = None
    for name, env in (("materialised", {"CWQ_CAT_LAZY": "0", "CWQ_CAT_DIRECT": "0"}),
                      ("lazy-heap", {"CWQ_CAT_LAZY_RUNS": "0", "CWQ_CAT_DIRECT": "0"}),
                      ("lazy-runs", {"CWQ_CAT_DIRECT": "0"}), ("direct", {"CWQ_CAT_DIRECT": "1"}), ("auto", {})):
        for key in ("CWQ_CAT_LAZY", "CWQ_CAT_LAZY_RUNS", "CWQ_CAT_DIRECT"):
            os.environ.pop(key, None)
        os.environ.update(env)
        got = ix.categorize(Q, k, 100000)
        t = med(lambda: ix.categorize(Q, k, 100000), 3)
        st = ix.last_categorize_stats()
        ts = []
        for i in range(16):
            q = Q[i:i + 1].contiguous()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ix.categorize(q, k, 100000)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        same = ref is None or all(torch.equal(a, b) for a, b in zip(ref, got))
        ref = ref or got
        print(f"[{tag}] Basic {name} batch {Q.shape[0]}: {t * 1e3:.3f} ms; one query per call median "
              f"{ts[8] * 1e6:.1f} us; == materialised {same}; calls/query {float(got[2].float().mean()):.0f}; {st}; "
              f"last call lazy {ix.last_lazy_stats()}", flush=True)
    for key in ("CWQ_CAT_LAZY", "CWQ_CAT_LAZY_RUNS", "CWQ_CAT_DIRECT"):
        os.environ.pop(key, None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=48000)
    ap.add_argument("--dim", type=int, default=96)
    ap.add_argument("--fan", default="8,4,6")
    ap.add_argument("--direct", type=float, default=0.03)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--depth1", action="store_true", help="also the depth-1 cut forced on")
    ap.add_argument("--basic", action="store_true", help="Basic batch / per call, lazy vs materialised DENSE")
    ap.add_argument("--basic-only", action="store_true")
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    fan = tuple(int(x) for x in args.fan.replace("x", ",").split(","))
    t, Q = broad_tree(pkg, args.n, args.dim, fan, 62, direct=args.direct, nq=args.nq)
    variants = [("adaptive", {})]
    if args.depth1:
        variants.append(("depth-1", {"CWQ_GROUP_CUT": "1", "CWQ_GROUP_CENTRE": "1"}))
    for tag, env in variants:
        os.environ.update(env)
        ix = pkg.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
        for key in env:
            os.environ.pop(key, None)
        print(f"[{tag}] cut {ix.cut_info()} filter {ix.filter_info()} info {ix.info}", flush=True)
        if not args.basic_only:
            legs(ix, Q, args.k, tag)
        if args.basic:
            basic(ix, Q, args.k, tag)
        ix.close()


if __name__ == "__main__":
    main()
