"""Edge cases of the Fast path on the GPU, against the CPU oracle (flat_synth_index +
rank_scores_vec, CobwebWrapper.py:210-265) and across strategies: an empty query batch,
a one-leaf tree, odd and tiny dimensions (D = 1, 3, 17, 100: every padding path of the
bf16 operand, the fp32 scan and the stream filter), k = 1 / k = N / k > N, identical
rows (score collisions: ties go to the lower sentence id), and queries far outside
the corpus.  Every strategy (exact scan, batch filter, stream filter) must return the
same ids and bit-identical scores; scores within 1e-5 of the oracle."""
import numpy as np
import pytest

from oracle import cobweb_oracle as O
from test_gpu_parity import rel_err, topk_equiv, RTOL

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg


def flat_index(pkg, X):
    fs = pkg.synth.flat_synth(X)
    return pkg.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device="cuda:0")


def all_modes(ix, Q, k):
    """(ids, scores) per strategy: exact scan, forced filter (stream path for <= 64
    queries, batch filter above), automatic."""
    out = {}
    for mode in (0, 1, -1):
        ix.set_filter(mode)
        ids, sc = ix.score_topk(Q, k)
        out[mode] = (ids.cpu(), sc.cpu(), ix.last_stats())
    ix.set_filter(-1)
    return out


def check_oracle(X, Q, k, ids, scores):
    idx = O.flat_synth_index(X.cpu().numpy())
    pa = O.path_arrays(idx)
    n = X.shape[0]
    for qi, x in enumerate(Q.cpu().numpy()):
        ref = O.rank_scores_vec(x, idx, pa).astype(np.float64)
        order = np.lexsort((np.arange(n), -ref))
        m = min(k, n)
        topk_equiv(ids[qi][:m].numpy(), order[:m], ref)
        assert rel_err(scores[qi][:m].numpy(), ref[ids[qi][:m].numpy()]) < RTOL
        assert np.all(ids[qi][m:].numpy() == -1)


def test_empty_query_batch(gpu):
    X = gpu.synth.synthetic_corpus(3000, 64, seed=1)
    ix = flat_index(gpu, X)
    for mode in (0, 1, -1):
        ix.set_filter(mode)
        ids, sc = ix.score_topk(torch.empty((0, 64), device="cuda:0"), 10)
        assert tuple(ids.shape) == (0, 10) and tuple(sc.shape) == (0, 10)


def test_one_leaf_tree(gpu):
    X = gpu.synth.synthetic_corpus(1, 32, seed=2)
    ix = flat_index(gpu, X)
    Q = gpu.synth.synthetic_corpus(5, 32, seed=3)
    for k in (1, 4):
        res = all_modes(ix, Q, k)
        for mode, (ids, sc, _) in res.items():
            assert torch.equal(ids, res[0][0]) and torch.equal(sc, res[0][1]), mode
        check_oracle(X, Q, k, res[0][0], res[0][1])


@pytest.mark.parametrize("N,D,nq,k", [(20000, 1, 300, 10), (20000, 3, 40, 5), (20000, 17, 300, 10),
                                      (20000, 17, 7, 10), (18000, 100, 64, 33), (18000, 100, 65, 1)])
def test_odd_dimensions(gpu, N, D, nq, k):
    """D not a multiple of 16/32: zero padding of the fp32 scan layout, the bf16 operand
    (whole 64-deep stages) and the stream filter's fragments must not change a key."""
    X = gpu.synth.synthetic_corpus(N, D, seed=N + D)
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, nq, seed=D)
    res = all_modes(ix, Q, k)
    assert res[1][2]["filter_used"]
    for mode in (1, -1):
        assert torch.equal(res[mode][0], res[0][0]) and torch.equal(res[mode][1], res[0][1]), mode
    sel = torch.arange(0, nq, max(1, nq // 6))
    check_oracle(X, Q[sel], k, res[0][0][sel], res[0][1][sel])


@pytest.mark.parametrize("nq", [3, 300])
def test_k_equals_and_exceeds_n(gpu, nq):
    """k = N and k > N: the full ranking, -1 past the sentence count (the reference's
    `k >= num_leaves` branch returns every leaf, CobwebWrapper.py:243-249)."""
    N, D = 50, 48
    X = gpu.synth.synthetic_corpus(N, D, seed=5)
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, nq, seed=6)
    for k in (N, N + 7):
        res = all_modes(ix, Q, k)
        for mode in (1, -1):
            assert torch.equal(res[mode][0], res[0][0]) and torch.equal(res[mode][1], res[0][1])
        check_oracle(X, Q[:3], k, res[0][0][:3], res[0][1][:3])


@pytest.mark.parametrize("nq", [1, 40, 400])
def test_identical_rows(gpu, nq):
    """Blocks of exactly identical corpus rows (score collisions): every strategy breaks
    the ties the same way (lower sentence id first), also when the tie group is wider
    than k and straddles the k-th place."""
    N, D = 24000, 64
    X = gpu.synth.synthetic_corpus(N, D, seed=8)
    X[100:140] = X[99]          # 41 identical rows
    X[5000:5003] = X[7000]      # a second group elsewhere, same key as row 7000
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, nq, seed=9)
    Q[0] = X[99] + 0.01         # query 0 ranks the 41-row group first
    for k in (10, 64):
        res = all_modes(ix, Q, k)
        for mode in (1, -1):
            assert torch.equal(res[mode][0], res[0][0]) and torch.equal(res[mode][1], res[0][1]), (k, mode)
        ids0 = res[0][0][0].numpy()
        assert list(ids0[:10]) == list(range(99, 109))     # ties: ascending ids
        check_oracle(X, Q[:1], k, res[0][0][:1], res[0][1][:1])


def test_far_queries(gpu):
    """Queries 1e3 standard deviations away from every row: keys of order -1e9, where the
    bf16 bounds are widest in absolute terms; the answer must still be the exact one."""
    N, D = 30000, 96
    X = gpu.synth.synthetic_corpus(N, D, seed=10)
    ix = flat_index(gpu, X)
    Q = gpu.synth.synthetic_corpus(20, D, seed=11) * 1000.0
    res = all_modes(ix, Q, 10)
    for mode in (1, -1):
        assert torch.equal(res[mode][0], res[0][0]) and torch.equal(res[mode][1], res[0][1]), mode
    check_oracle(X, Q[:4], 10, res[0][0][:4], res[0][1][:4])
