"""Throughput of the PCA + ICA whitening transform (F4) on one MI355X: n x 768 -> 256
(the C5 shape), fp32 MFMA GEMMs, inputs resident in HBM.  GPU only.

    python scripts/whiten_probe.py --n 2000000
"""
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
    ap.add_argument("--n", type=int, default=2_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--p", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    pkg = cobweb_pkg.load()
    rng = np.random.default_rng(0)
    comps = np.linalg.qr(rng.standard_normal((a.d, a.p)))[0].T.astype(np.float32)
    unmix = np.linalg.qr(rng.standard_normal((a.p, a.p)))[0].astype(np.float32)
    w = pkg.whitening.PCAICAWhiteningModel(np.zeros(a.d, np.float32), comps, unmix,
                                           np.ones(a.p, np.float32), 1e-8, device="cuda:0")
    X = torch.randn((a.n, a.d), device="cuda:0")
    w.transform(X)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        w.transform(X)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    flops = 2.0 * a.n * a.p * (a.d + a.p)
    print(f"whiten {a.n}x{a.d}->{a.p}: {dt * 1e3:.2f} ms, {a.n / dt / 1e6:.1f} M rows/s, "
          f"{flops / dt / 1e12:.1f} TFLOP/s fp32 (peak 157.3), {4.0 * a.n * (a.d + a.p) / dt / 1e9:.0f} GB/s in+out")


if __name__ == "__main__":
    main()
