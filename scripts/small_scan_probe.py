"""Exact Fast top-k on small flat-synth corpora with many queries: the lane-per-query
scan (scan_small_kernel) vs the row-sliced scan (CWQ_SCAN_SMALL=0), in one process,
interleaved.  GPU only.

    python scripts/small_scan_probe.py --shapes 1500x384x64/300,8000x768x1000
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def timed(ix, q, k, reps):
    ix.score_topk(q, k)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ix.score_topk(q, k)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="1500x384x64/300/1000/3000,4000x768x300/1000/3000,"
                    "8000x768x1000/3000/10000,16000x384x300/1000/10000,16000x768x300/3000")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    dev = torch.device("cuda", 0)
    for sh in args.shapes.split(","):
        n, d, nqs = sh.split("x")
        n, d = int(n), int(d)
        nqs = [int(v) for v in nqs.split("/")]
        X = pkg.synth.synthetic_corpus(n, d, seed=0, device=dev)
        fs = pkg.synth.flat_synth(X)
        ix = pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device=dev)
        Qa, _ = pkg.synth.synthetic_queries(X, max(nqs), seed=1)
        ix.set_filter(0)
        for nq in nqs:
            Q = Qa[:nq].contiguous()
            res = {}
            for rnd in range(2):
                for mode in ("1", "0", ""):
                    os.environ["CWQ_SCAN_SMALL"] = mode
                    res.setdefault(mode, []).append(timed(ix, Q, args.k, args.reps))
            os.environ["CWQ_SCAN_SMALL"] = "1"
            ids1, s1 = ix.score_topk(Q, args.k)
            os.environ["CWQ_SCAN_SMALL"] = "0"
            ids0, s0 = ix.score_topk(Q, args.k)
            os.environ.pop("CWQ_SCAN_SMALL")
            same = bool(torch.equal(ids1, ids0) and torch.equal(s1, s0))
            t1, t0, ta = (min(res[m]) * 1e3 for m in ("1", "0", ""))
            print(f"{n}x{d} nq={nq} k={args.k}: small {t1:.3f} ms  row-sliced {t0:.3f} ms  auto {ta:.3f} ms  "
                  f"small/rs {t1 / t0:.2f}  auto {nq / ta * 1e3:.0f} q/s  identical={same}", flush=True)
        ix.close()
        del X, fs, Qa
        torch.cuda.empty_cache()
    print("done", flush=True)


if __name__ == "__main__":
    main()
