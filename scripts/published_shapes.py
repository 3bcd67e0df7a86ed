"""Fast and Basic per-query latency, one query per call, at the shapes BASELINE.md publishes
ms/q for -- the reference harness's mode (benchmark_utils.py:576-581, 801-805: a numpy
query into cobweb_predict_fast / cobweb_predict, sentence strings out, timed per call).

Trees are built the reference's way, by the drop-in's device ifit (CobwebWrapper(corpus,
embeddings), CobwebWrapper.py:13-80):
  g8        tests/golden/g8_c1_d384.npz: config C1's own shape (1,500 x 384) and its 300
            queries; the device ifit rebuilds the reference's 1,591-node tree
  qqp1k     1,000 x 1,024, k = 10   (published Fast 5.86 / Basic 4.70 ms/q)
  qqp10k    10,000 x 1,024, k = 20  (published Fast 68.19; PCA+ICA Fast 53.05 / Basic 1,418.06)
  marco40k  40,000 x 768, k = 50    (published PCA+ICA Fast 253.16; QQP-40k PCA+ICA Basic 5,631.52)
The synthetic corpora are Gaussian clusters (no datasets offline); the published numbers are
the reference on CPU (BASELINE.md rows cited).  GPU only.

    python scripts/published_shapes.py [--shapes g8,qqp1k,qqp10k,marco40k] [--calls 200] [--json out.json]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# name: (n, dim, clusters, k, published {leg: (ms/q)})
SHAPES = {
    "g8": (1500, 384, 0, 10, {"fast": (29.76, "Cobweb Fast, QQP N=1500 (train split), BASELINE.md:26")}),
    "qqp1k": (1000, 1024, 10, 10, {"fast": (5.86, "Cobweb Fast, QQP N=1000, BASELINE.md:24"),
                                   "basic": (4.70, "Cobweb Basic, QQP N=1000, BASELINE.md:25")}),
    "qqp10k": (10000, 1024, 20, 20, {"fast": (68.19, "Cobweb Fast, QQP N=10000, BASELINE.md:28"),
                                     "basic": (1418.06, "Cobweb PCA+ICA (categorize), QQP N=10000, BASELINE.md:30")}),
    "marco40k": (40000, 768, 40, 50, {"fast": (253.16, "Cobweb PCA+ICA Fast, MS-MARCO N=40000, BASELINE.md:35"),
                                      "basic": (5631.52, "Cobweb PCA+ICA (categorize), QQP N=40000, BASELINE.md:33")}),
}


def corpus(n, d, nc, nq, seed=5):
    rng = np.random.default_rng(seed)
    C = rng.standard_normal((nc, d)).astype(np.float32) * 2.0
    X = (C[rng.integers(0, nc, n)] + 0.3 * rng.standard_normal((n, d))).astype(np.float32)
    pick = rng.choice(n, nq // 2, replace=False)
    Qp = X[pick] + 0.1 * rng.standard_normal((nq // 2, d))
    Qf = C[rng.integers(0, nc, nq - nq // 2)] + 0.3 * rng.standard_normal((nq - nq // 2, d))
    return X, np.concatenate([Qp, Qf]).astype(np.float32)


def per_call(fn, Qn, calls):
    fn(Qn[0])
    ts, errs = [], 0
    for i in range(calls):
        t0 = time.perf_counter()
        try:
            fn(Qn[i % len(Qn)])
        except IndexError:   # Basic: fewer than k nodes found (CobwebTorchTree.py:289), as the reference
            errs += 1
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return {"median_ms": round(ts[len(ts) // 2] * 1e3, 4), "p10_ms": round(ts[len(ts) // 10] * 1e3, 4),
            "mean_ms": round(float(np.mean(ts)) * 1e3, 4), "calls": calls, "index_errors": errs}


def run_shape(pkg, name, calls):
    n, d, nc, k, pub = SHAPES[name]
    if name == "g8":
        z = np.load(os.path.join(ROOT, "tests", "golden", "g8_c1_d384.npz"))
        X, Qn, k = z["X"].astype(np.float32), z["Xq"].astype(np.float32), int(z["k"])
        ref_nodes = int(z["parent"].shape[0])
    else:
        X, Qn = corpus(n, d, nc, 300)
        ref_nodes = None
    random.seed(0)
    t0 = time.perf_counter()
    w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(len(X))], corpus_embeddings=X)
    torch.cuda.synchronize()
    t_fit = time.perf_counter() - t0
    w.build_prediction_index()
    inf = w._index.info
    out = {"shape": name, "n": int(X.shape[0]), "dim": int(X.shape[1]), "k": k,
           "tree": {"nodes": inf["n_nodes"], "internal": inf["internal_nodes"], "max_depth": inf["max_depth"],
                    "root_children": len(w.tree.root.children), "device_ifit_s": round(t_fit, 3)}}
    if ref_nodes is not None:
        out["tree"]["reference_tree_nodes"] = ref_nodes
    random.seed(1)
    out["fast"] = per_call(lambda q: w.cobweb_predict_fast(q, k), Qn, calls)
    random.seed(1)
    out["basic"] = per_call(lambda q: w.cobweb_predict(q, k), Qn, calls)
    Q = torch.from_numpy(Qn).cuda()
    ix = w._index
    ix.score_topk(Q, k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ix.score_topk(Q, k)
    torch.cuda.synchronize()
    out["fast_batch_ms_per_q"] = round((time.perf_counter() - t0) * 1e3 / len(Qn), 5)
    for leg in ("fast", "basic"):
        if leg in pub:
            ms, row = pub[leg]
            out[leg]["published_ms_per_q"] = ms
            out[leg]["published_row"] = row
            out[leg]["speedup_vs_published"] = round(ms / out[leg]["median_ms"], 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="g8,qqp1k,qqp10k,marco40k")
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    res = []
    for name in args.shapes.replace("+", ",").split(","):
        r = run_shape(pkg, name, args.calls)
        res.append(r)
        t = r["tree"]
        print(f"{name}: {r['n']}x{r['dim']} k={r['k']}; device ifit {t['device_ifit_s']:.2f} s -> {t['nodes']} nodes "
              f"(depth {t['max_depth']}, root children {t['root_children']}"
              + (f", reference tree {t['reference_tree_nodes']}" if "reference_tree_nodes" in t else "") + ")", flush=True)
        for leg in ("fast", "basic"):
            x = r[leg]
            pub = (f"; published {x['published_ms_per_q']} ms/q ({x['published_row']}) -> "
                   f"{x['speedup_vs_published']}x") if "published_ms_per_q" in x else ""
            print(f"  {leg:5s} per call: median {x['median_ms']:.3f} ms, p10 {x['p10_ms']:.3f}, mean {x['mean_ms']:.3f}"
                  f" ({x['index_errors']} IndexError){pub}", flush=True)
        print(f"  fast batch (the shape's 300 queries in one call): {r['fast_batch_ms_per_q']:.4f} ms/q", flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
