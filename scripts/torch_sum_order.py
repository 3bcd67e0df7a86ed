"""The summation order of torch's CPU float32 sum (ATen's cascade sum as this torch build
runs it), restated in numpy float32 steps and checked bit for bit against torch.sum.  The
reference's category utility is KL sums over torch tensors (CobwebTorchTree.py:344-356), so
the fitters (cwq_refmath.h torch_sum2) add the KL terms in exactly this order.

    python scripts/torch_sum_order.py
"""
import numpy as np

F32 = np.float32


def _ceil_log2(x):
    return 0 if x <= 1 else int(np.ceil(np.log2(x)))


def torch_order_sum(x, W=8):
    """8-wide vectors: 4 vector accumulators over rows of 4 vectors with cascade levels of
    2^max(4, ceil_log2(rows)/4) rows; leftover vectors into accumulator 0; accumulators
    added in order; then the scalar tail from 0 and the W lanes in order.  Fewer than W
    elements: the same 4-accumulator form over scalars."""
    x = np.asarray(x, np.float32)
    n = len(x)
    if n < W:
        acc = [F32(0)] * 4
        nr = n // 4
        for r in range(nr):
            for k in range(4):
                acc[k] = F32(acc[k] + x[r * 4 + k])
        for d in range(nr * 4, n):
            acc[0] = F32(acc[0] + x[d])
        for k in range(1, 4):
            acc[0] = F32(acc[0] + acc[k])
        return acc[0]
    vec_size = n // W
    size_ilp = vec_size // 4
    lp = max(4, _ceil_log2(size_ilp) // 4)
    step, mask = 1 << lp, (1 << lp) - 1
    lev = [[np.zeros(W, np.float32) for _ in range(4)] for _ in range(4)]
    row = lambda i, k: x[(i * 4 + k) * W:(i * 4 + k + 1) * W]
    i = 0
    while i + step <= size_ilp:
        for _ in range(step):
            for k in range(4):
                lev[0][k] = (lev[0][k] + row(i, k)).astype(np.float32)
            i += 1
        for j in range(1, 4):
            for k in range(4):
                lev[j][k] = (lev[j][k] + lev[j - 1][k]).astype(np.float32)
                lev[j - 1][k] = np.zeros(W, np.float32)
            if i & (mask << (j * lp)):
                break
    while i < size_ilp:
        for k in range(4):
            lev[0][k] = (lev[0][k] + row(i, k)).astype(np.float32)
        i += 1
    ps = [lev[0][k] for k in range(4)]
    for j in range(1, 4):
        for k in range(4):
            ps[k] = (ps[k] + lev[j][k]).astype(np.float32)
    for v in range(size_ilp * 4, vec_size):
        ps[0] = (ps[0] + x[v * W:(v + 1) * W]).astype(np.float32)
    for k in range(1, 4):
        ps[0] = (ps[0] + ps[k]).astype(np.float32)
    s = F32(0)
    for d in range(vec_size * W, n):
        s = F32(s + x[d])
    for lane in range(W):
        s = F32(s + ps[0][lane])
    return s


def check(sizes=(5, 7, 8, 9, 16, 17, 32, 48, 100, 129, 384, 513, 768, 1024, 4096), trials=200, seed=3):
    import torch
    rng = np.random.default_rng(seed)
    out = {}
    for n in sizes:
        ok = 0
        for _ in range(trials):
            x = (rng.standard_normal(n) * rng.uniform(0.1, 10)).astype(np.float32)
            ok += torch_order_sum(x) == F32(torch.from_numpy(x).sum().item())
        out[n] = ok / trials
    return out


if __name__ == "__main__":
    import torch
    print("cpu capability", torch.backends.cpu.get_cpu_capability())
    for n, frac in check().items():
        print(f"n={n}: restatement == torch.sum on {100 * frac:.1f}% of random vectors")
