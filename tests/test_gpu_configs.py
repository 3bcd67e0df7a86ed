"""BASELINE configurations on the GPU at (or at the per-GPU shape of) their full sizes.

* C3 (configs[2]): 1M x 768 flat-synth, the bench's 10k-query batch -- the filter's
  ids AND scores bit-identical to the exact fp32 scan; the oracle on sampled queries;
  properties of the whole batch (targets first, descending scores, split invariance).
* C4 per-GPU shard shape (configs[3]): 1M x 1024 (the filter bound at D = 1024), a
  strong-scaling query split over 8 "ranks" equals the whole batch.
* C5 (configs[4]): PCA + ICA whitening 768 -> 256 (`cwq_whiten`, src/whitening/
  pca_ica.py:30-51) feeding flat and two-level trees; Fast (filter == scan, oracle) and
  Basic (categorize pop order + log_prob calls vs the oracle) on the whitened index.

Oracle: oracle/cobweb_oracle.py on the same arrays (the node statistics come from the
GPU Welford builder, which is bit-identical to the reference's increment_counts --
tests/test_gpu_parity.py)."""
import numpy as np
import pytest

from oracle import cobweb_oracle as O
from test_gpu_parity import RTOL, rel_err, topk_equiv

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg


def flat_oracle_scores(mean_np, var_np, x):
    """rank_scores of a flat tree (root + leaves, paths [0, 1 + i]) for one query,
    vectorised: every path has length 2 and default level weights (coefficient 1/2)."""
    lp = O.node_logprob_prime(x, mean_np, var_np)
    c = O.path_weight(0, 2, O.DEFAULT_LEVEL_WEIGHTS)
    return (c * lp[0] + c * lp[1:]).astype(np.float32)


def check_against_oracle(ids, scores, ref):
    topk_equiv(ids, O.topk_ids_scores(ref, len(ids))[0], ref.astype(np.float64))
    assert rel_err(scores, ref[ids]) < RTOL


def filter_vs_scan(ix, Q, k):
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, k)
    assert not ix.last_stats()["filter_used"]
    ix.set_filter(-1)
    ids1, s1 = ix.score_topk(Q, k)
    st = ix.last_stats()
    return ids0, s0, ids1, s1, st


def test_c3_full_size(gpu):
    N, D, NQ, k = 1_000_000, 768, 10_000, 10
    X = gpu.synth.synthetic_corpus(N, D, seed=0)
    t = gpu.synth.flat_synth(X)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    Q, targets = gpu.synth.synthetic_queries(X, NQ, seed=1)
    ids0, s0, ids1, s1, st = filter_vs_scan(ix, Q, k)
    assert st["filter_used"] and st["filter_queries"] == NQ
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    ids, s = ids1.cpu().numpy(), s1.cpu().numpy()
    tg = targets.cpu().numpy()
    assert np.all(ids[:len(tg), 0] == tg)                      # perturbed corpus rows find their source first
    assert np.all(np.diff(s, axis=1) <= 0)
    for a, b in [(0, 256), (4999, 5301), (9744, 10000)]:        # batch split invariance (tile edges)
        i2, s2 = ix.score_topk(Q[a:b], k)
        assert torch.equal(i2, ids1[a:b]) and torch.equal(s2, s1[a:b])
    mean_np, var_np = t["mean"].cpu().numpy(), t["var"].cpu().numpy()
    Qn = Q.cpu().numpy()
    for qi in [0, 1, 2500, 4999, 5000, 5001, 7777, 9999]:       # perturbed and fresh queries
        check_against_oracle(ids[qi], s[qi], flat_oracle_scores(mean_np, var_np, Qn[qi]))
    ix.close()


def test_c4_shard_shape_d1024(gpu):
    N, D, NQ, k = 1_000_000, 1024, 4096, 10
    X = gpu.synth.synthetic_corpus(N, D, seed=3)
    t = gpu.synth.flat_synth(X)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    Q, targets = gpu.synth.synthetic_queries(X, NQ, seed=4)
    ids0, s0, ids1, s1, st = filter_vs_scan(ix, Q, k)
    assert st["filter_used"] and st["fallback_queries"] <= NQ // 100, st
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    # the strong-scaling split of bench --preset c4 (dist.shard_bounds over 8 ranks)
    for r in range(8):
        lo, hi = gpu.dist.shard_bounds(NQ, r, 8)
        i2, s2 = ix.score_topk(Q[lo:hi], k)
        assert torch.equal(i2, ids1[lo:hi]) and torch.equal(s2, s1[lo:hi])
    tg = targets.cpu().numpy()
    assert np.all(ids1.cpu().numpy()[:len(tg), 0] == tg)
    mean_np, var_np = t["mean"].cpu().numpy(), t["var"].cpu().numpy()
    Qn = Q.cpu().numpy()
    for qi in [0, 2047, 2048, 4095]:
        check_against_oracle(ids1[qi].cpu().numpy(), s1[qi].cpu().numpy(), flat_oracle_scores(mean_np, var_np, Qn[qi]))
    ix.close()


def _whitening_768_to_256(n_fit=20_000, seed=11):
    """PCA (numpy SVD on a fitting sample) to 256 dims and a random orthogonal 256 x 256
    unmixing, on correlated 768-d data -- the transform's shape and arithmetic are those of
    PCAICAWhiteningModel (the ICA fit itself is offline scikit-learn and not under test)."""
    rng = np.random.default_rng(seed)
    A = (rng.standard_normal((768, 768)) / np.sqrt(768)).astype(np.float32)
    scale = np.linspace(3.0, 0.2, 768).astype(np.float32)
    Xf = (rng.standard_normal((n_fit, 768)).astype(np.float32) * scale) @ A
    mean = Xf.mean(0).astype(np.float32)
    _, sv, vt = np.linalg.svd((Xf - mean).astype(np.float64), full_matrices=False)
    comps = vt[:256].astype(np.float32)
    ev = (sv[:256] ** 2 / (n_fit - 1)).astype(np.float32)
    unmix = np.linalg.qr(rng.standard_normal((256, 256)))[0].astype(np.float32)
    return A, scale, mean, comps, ev, unmix


def test_c5_whitened_d256(gpu):
    N, NQ, k = 400_000, 2048, 10
    A, scale, mean, comps, ev, unmix = _whitening_768_to_256()
    W = gpu.whitening.PCAICAWhiteningModel(mean, comps, unmix, ev, 1e-8, device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(12)
    At, st_ = torch.from_numpy(A).cuda(), torch.from_numpy(scale).cuda()
    raw = (torch.randn((N, 768), generator=g, device="cuda:0") * st_) @ At
    X = W.transform(raw)                                          # cwq_whiten, 768 -> 256
    assert X.shape == (N, 256)
    sample = raw[::4001].cpu().numpy()
    ref_w = O.whiten_transform(sample, mean, comps, ev, unmix, 1e-8)
    got_w = X[::4001].cpu().numpy()
    assert float(np.max(np.abs(got_w - ref_w).max(1) / np.abs(ref_w).max(1))) < 1e-5
    Q, targets = gpu.synth.synthetic_queries(X, NQ, seed=13)
    # flat tree over the whitened corpus
    t = gpu.synth.flat_synth(X)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    ids0, s0, ids1, s1, st = filter_vs_scan(ix, Q, k)
    assert st["filter_used"]
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    tg = targets.cpu().numpy()
    assert np.all(ids1.cpu().numpy()[:len(tg), 0] == tg)
    mean_np, var_np = t["mean"].cpu().numpy(), t["var"].cpu().numpy()
    Qn = Q.cpu().numpy()
    for qi in [0, 1023, 1024, 2047]:
        check_against_oracle(ids1[qi].cpu().numpy(), s1[qi].cpu().numpy(), flat_oracle_scores(mean_np, var_np, Qn[qi]))
    ix.close()
    del t
    # two-level tree (root -> 1024 clusters -> leaves) on the first 100k whitened rows:
    # Fast through the filter's multi-parent tiles, and Basic (categorize) vs the oracle
    Nh = 100_000
    Xh = X[:Nh].contiguous()
    lab = torch.randint(0, 1024, (Nh,), generator=g, device="cuda:0")
    t2 = gpu.synth.two_level_synth(Xh, lab)
    ix2 = gpu.index.CobwebIndex(t2["mean"], t2["var"], t2["parent"], t2["node_of_sentence"], device="cuda:0")
    Qh, _ = gpu.synth.synthetic_queries(Xh, 512, seed=14)
    ids0, s0, ids1, s1, st = filter_vs_scan(ix2, Qh, k)
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    parent = t2["parent"]
    nos = t2["node_of_sentence"]
    mean2, var2 = t2["mean"].cpu().numpy(), t2["var"].cpu().numpy()
    paths = [[0, int(parent[j]), int(j)] for j in nos]
    idx = O.FlatIndex(mean2, var2, parent, paths)
    pa = (np.array(paths, np.int64), np.full((Nh, 3), O.path_weight(0, 3, O.DEFAULT_LEVEL_WEIGHTS), np.float32))
    Qhn = Qh.cpu().numpy()
    for qi in [0, 255, 256, 511]:
        ref = O.rank_scores_vec(Qhn[qi], idx, pa)
        check_against_oracle(ids1[qi].cpu().numpy(), s1[qi].cpu().numpy(), ref)
    # Basic: pop order and log_prob call counts
    cnt = t2["count"].cpu().numpy()
    m2 = t2["meanSq"].cpu().numpy()
    node_sid = np.full(len(parent), -1, np.int64)
    node_sid[nos] = np.arange(Nh)
    has = node_sid >= 0
    sid_ptr = np.concatenate([[0], np.cumsum(has)]).astype(np.int64)
    sid_list = node_sid[has]
    tree = O.OTree(256)
    tree.root = O.tree_from_arrays(parent, cnt, mean2, m2, sid_ptr, sid_list)
    nodes, found, calls = ix2.categorize(Qh[:4], k)
    bfs = {id(n): i for i, n in enumerate(O.bfs_nodes(tree.root))}
    for qi in range(4):
        got, ncalls = tree.categorize(Qhn[qi], k, order=bfs)
        assert [bfs[id(n)] for n in got] == nodes[qi].cpu().tolist(), qi
        assert int(found[qi]) == k and int(calls[qi]) == ncalls
    ix2.close()
