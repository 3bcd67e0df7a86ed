"""F3: the batched metrics equal the reference harness definitions
(benchmark_utils.py:619-833), including sklearn's tie-averaged nDCG."""
import numpy as np
import pytest
import torch

sk = pytest.importorskip("sklearn.metrics")


def ref_metrics(retrieved, targets, top_k):
    """The reference's per-query loop (benchmark_utils.py:801-831), verbatim semantics."""
    ks = sorted(k for k in [2, 3, 5, 10, 20, 50, 100] if k <= top_k)
    m = {f"{p}@{k}": 0.0 for p in ("recall", "mrr", "ndcg") for k in ks}
    for row, target in zip(retrieved, targets):
        row = [d for d in row if d >= 0]
        for k in ks:
            top = row[:k]
            if target in top:
                m[f"recall@{k}"] += 1
                m[f"mrr@{k}"] += 1 / (top.index(target) + 1)
            rel = [1 if d == target else 0 for d in top]
            if sum(rel) > 0:
                m[f"ndcg@{k}"] += sk.ndcg_score([sorted(rel, reverse=True)], [rel])
    n = len(targets)
    return {k: round(v / n, 4) for k, v in m.items()}


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_metrics_match_reference_loop(pkg, seed):
    rng = np.random.default_rng(seed)
    Q, top_k = 200, 10
    retrieved = rng.integers(0, 15, (Q, top_k))          # small key space -> duplicates / multi-hits
    retrieved[rng.random((Q, top_k)) < 0.05] = -1
    retrieved = np.sort(retrieved, axis=1)[:, ::-1].copy()   # keep -1 padding at the end
    targets = rng.integers(0, 15, Q)
    got = pkg.harness.retrieval_metrics(torch.from_numpy(retrieved), torch.from_numpy(targets), top_k)
    ref = ref_metrics(retrieved.tolist(), targets.tolist(), top_k)
    for key in ref:
        assert abs(got[key] - ref[key]) <= 1e-4, (key, got[key], ref[key])


def test_brute_force_matches_numpy(pkg):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((500, 16)).astype(np.float32)
    Q = rng.standard_normal((20, 16)).astype(np.float32)
    ip = pkg.harness.brute_force_topk(X, Q, 5, "ip").numpy()
    l2 = pkg.harness.brute_force_topk(X, Q, 5, "l2").numpy()
    np.testing.assert_array_equal(ip, np.argsort(-(Q @ X.T), 1)[:, :5])
    d = ((Q[:, None, :] - X[None]) ** 2).sum(-1)
    np.testing.assert_array_equal(l2, np.argsort(d, 1)[:, :5])


def test_brute_force_exact_chunked(pkg):
    """The float64 row-chunked path gives the exact ranking, chunk boundaries included."""
    rng = np.random.default_rng(5)
    X = rng.standard_normal((3001, 48)).astype(np.float32)
    Q = rng.standard_normal((37, 48)).astype(np.float32)
    Xd, Qd = X.astype(np.float64), Q.astype(np.float64)
    for metric in ("ip", "l2"):
        got = pkg.harness.brute_force_topk(X, Q, 7, metric, exact=True, row_chunk=500).numpy()
        s = Qd @ Xd.T if metric == "ip" else -((Qd[:, None, :] - Xd[None]) ** 2).sum(-1)
        ref = np.argsort(-s, axis=1, kind="stable")[:, :7]
        assert np.array_equal(np.sort(got, 1), np.sort(ref, 1)), metric
