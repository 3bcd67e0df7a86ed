"""The internal pass of a one-query call (raw_split_kernel: D split over the workgroup's
waves, partials folded in slice order from LDS) gives the scan kernel's sums bit for bit:
the exact internal prefixes (prefix_bounds' exact column) and the Fast / Basic results of
one-query calls equal those with CWQ_RAW_SPLIT=0, on deep, clustered and wide trees and at
dimensions that are not a multiple of 64."""
import os

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg


def _with(env, fn):
    old = {n: os.environ.get(n) for n in env}
    os.environ.update(env)
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        for n, v in old.items():
            if v is None:
                del os.environ[n]
            else:
                os.environ[n] = v


@pytest.mark.parametrize("dim", [48, 96, 768])
def test_raw_split_equals_scan(gpu, dim):
    X = gpu.synth.synthetic_corpus(12_000, dim, seed=41)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(42)
    trees = [gpu.synth.balanced_synth(X, 4, 5),
             gpu.synth.two_level_synth(X, torch.randint(0, 150, (X.shape[0],), generator=g, device="cuda:0"))]
    for t in trees:
        ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
        Q, _ = gpu.synth.synthetic_queries(X, 6, seed=43)
        for i in range(Q.shape[0]):
            q1 = Q[i:i + 1].contiguous()
            ex_a = _with({"CWQ_RAW_SPLIT": "0"}, lambda: ix.prefix_bounds(q1)[2].clone())
            ex_b = _with({}, lambda: ix.prefix_bounds(q1)[2].clone())
            assert torch.equal(ex_a, ex_b), (dim, i)
            fa = _with({"CWQ_RAW_SPLIT": "0"}, lambda: ix.score_topk(q1, 10))
            fb = _with({}, lambda: ix.score_topk(q1, 10))
            assert torch.equal(fa[0], fb[0]) and torch.equal(fa[1], fb[1]), (dim, i)
            ca = _with({"CWQ_RAW_SPLIT": "0"}, lambda: ix.categorize(q1, 10, 100000))
            cb = _with({}, lambda: ix.categorize(q1, 10, 100000))
            for x, y in zip(ca, cb):
                assert torch.equal(x, y), (dim, i)
        ix.close()
