"""GPU ifit (add path) throughput: inserts/s of CobwebWrapper's
incremental fit (the device-resident insert loop, cwq_fitdev.hip) for N(0,I) data (a flat
tree: every insert scores all root children, the reference's O(N^2 D) case) and clustered
data (hierarchical trees).  Rows go in chunks (one add_sentences call each, progress
printed per chunk); with --compare-every, a short chunk at that cadence is also run with
one workgroup (CWQ_FIT_HELPERS=0, the round-3 loop) and the tree it builds is checked
against the chip-wide fit's (same rows, same random() state).  GPU only.

    python scripts/fit_probe.py --n 20000 --dim 768 --clusters 0 --chunk 2000 --compare-every 5000
"""
import argparse
import copy
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def depth_stats(root):
    n, mx, stack = 0, 0, [(root, 0)]
    nint = 0
    while stack:
        x, d = stack.pop()
        n += 1
        mx = max(mx, d)
        if x.children:
            nint += 1
        stack.extend((c, d + 1) for c in x.children)
    return n, nint, mx, len(root.children)


def arrays(root):
    out, q, h = [], [root], 0
    while h < len(q):
        x = q[h]
        h += 1
        out.append(x)
        q.extend(x.children)
    pos = {id(x): i for i, x in enumerate(out)}
    return ([-1 if x.parent is None else pos[id(x.parent)] for x in out], np.stack([x.mean for x in out]),
            np.stack([x.meanSq for x in out]), [list(x.sentence_id) for x in out])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--clusters", type=int, default=0, help="0: X ~ N(0,I); else Gaussian clusters (sd 0.3)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--chunk", type=int, default=0, help="rows per add_sentences call (0: one call)")
    ap.add_argument("--compare-every", type=int, default=0,
                    help="every this many rows, also time --compare-rows rows with one workgroup")
    ap.add_argument("--compare-rows", type=int, default=200)
    ap.add_argument("--host", action="store_true", help="the host-driven fitter (CWQ_FIT_DEVICE=0)")
    args = ap.parse_args()
    if args.host:
        os.environ["CWQ_FIT_DEVICE"] = "0"
    pkg = cobweb_pkg.load()
    rng = np.random.default_rng(args.seed)
    if args.clusters:
        C = rng.standard_normal((args.clusters, args.dim)).astype(np.float32) * 2.0
        X = (C[rng.integers(0, args.clusters, args.n)] +
             0.3 * rng.standard_normal((args.n, args.dim))).astype(np.float32)
    else:
        X = rng.standard_normal((args.n, args.dim)).astype(np.float32)
    random.seed(args.seed)
    w = pkg.CobwebWrapper(corpus=None, corpus_embeddings=X[:8])   # warm up libcwq + the device pool
    torch.cuda.synchronize()
    random.seed(args.seed)
    chunk = args.chunk or args.n
    w = None
    t_all, done = 0.0, 0
    mode = "host-driven" if args.host else f"device-resident, helpers={os.environ.get('CWQ_FIT_HELPERS', 'CUs-1')}"
    next_cmp = args.compare_every
    while done < args.n:
        m = min(chunk, args.n - done)
        if next_cmp and done >= next_cmp and done + args.compare_rows <= args.n:
            # the same rows from the same tree and random() state with one workgroup
            tree0, st0 = copy.deepcopy(w.tree), random.getstate()
            rows = X[done:done + args.compare_rows]
            fan = len(w.tree.root.children)
            os.environ["CWQ_FIT_HELPERS"] = "0"
            w1 = pkg.CobwebWrapper.__new__(pkg.CobwebWrapper)
            w1.__dict__.update(w.__dict__)
            w1.tree = tree0
            w1.sentences, w1.sentence_to_node = list(w.sentences), dict(w.sentence_to_node)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            w1.add_sentences([f"s{i}" for i in range(done, done + len(rows))], rows)
            torch.cuda.synchronize()
            t1 = time.perf_counter() - t0
            st1 = random.getstate()
            del os.environ["CWQ_FIT_HELPERS"]
            random.setstate(st0)
            t0 = time.perf_counter()
            w.add_sentences([f"s{i}" for i in range(done, done + len(rows))], rows)
            torch.cuda.synchronize()
            t2 = time.perf_counter() - t0
            same = random.getstate() == st1 and all(
                (np.array_equal(a, b) if isinstance(a, np.ndarray) else a == b)
                for a, b in zip(arrays(w.tree.root), arrays(w1.tree.root)))
            # the insert kernel's own time (cwq_fit_insert; the call also loads the tree into
            # the device pool and exports it back -- a fixed cost per add_sentences call)
            k1 = getattr(w1, "last_fit_stats", {}).get("kernel_s", float("nan"))
            k2 = getattr(w, "last_fit_stats", {}).get("kernel_s", float("nan"))
            print(f"  at {done} rows (root fan-out {fan}): {len(rows)} inserts -- one workgroup "
                  f"{1e3 * t1 / len(rows):.3f} ms/insert, chip-wide {1e3 * t2 / len(rows):.3f} ms/insert "
                  f"= {t1 / t2:.1f}x per call; insert kernel {1e3 * k1 / len(rows):.3f} vs {1e3 * k2 / len(rows):.3f} "
                  f"ms/insert = {k1 / k2:.1f}x; trees and random() state identical: {same}", flush=True)
            done += len(rows)
            t_all += t2
            next_cmp += args.compare_every
            del w1, tree0
            continue
        t0 = time.perf_counter()
        if w is None:
            w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(m)], corpus_embeddings=X[:m])
        else:
            w.add_sentences([f"s{i}" for i in range(done, done + m)], X[done:done + m])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        t_all += dt
        done += m
        fan = len(w.tree.root.children)
        print(f"  rows {done - m}..{done}: {m / dt:.0f} inserts/s ({1e3 * dt / m:.3f} ms/insert), root fan-out now "
              f"{fan}", flush=True)
    n, nint, mx, rootc = depth_stats(w.tree.root)
    print(f"ifit ({mode}) n={args.n} d={args.dim} clusters={args.clusters}: {t_all:.2f} s  {args.n / t_all:.0f} inserts/s  "
          f"{1e3 * t_all / args.n:.2f} ms/insert  tree: {n} nodes ({nint} internal), depth {mx}, root children {rootc}",
          flush=True)


if __name__ == "__main__":
    main()
