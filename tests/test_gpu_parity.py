"""GPU parity: libcwq (through the C-ABI) against the reference's golden vectors and
the CPU oracle.  Tolerances: scores within 1e-5 relative (north star); top-k ids
identical except swaps the reference itself cannot separate (gap < 1e-5*|score|);
categorize pop order and log_prob call counts identical."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import cobweb_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
RTOL = 1e-5
HIER = ["g1_hier_d32", "g4_twolevel_d48", "g5_hier_d384", "g2_flat_d768"]


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    m = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), m)
    return float(np.max(np.abs(a[m] - b[m]) / np.maximum(np.abs(b[m]), 1e-30))) if m.any() else 0.0


def topk_equiv(ids, ref_ids, ref_scores, rtol=RTOL):
    ids, ref_ids = list(ids), list(ref_ids)
    for a, b in zip(ids, ref_ids):
        if a != b:
            sa, sb = ref_scores[a], ref_scores[b]
            assert abs(sa - sb) <= rtol * max(abs(sa), abs(sb)), (a, b, sa, sb)


def index_from_golden(pkg, g, weights=None):
    var = O.compute_var(g["meanSq"], g["count"][:, None])
    var[g["count"] == 0] = O.PRIOR_VAR
    nos = np.full(int(g["n_sent"]), -1, np.int64)
    for i in range(len(g["parent"])):
        for s in g["sid_list"][g["sid_ptr"][i]:g["sid_ptr"][i + 1]]:
            nos[s] = i
    return pkg.index.CobwebIndex(g["mean"], var, g["parent"], nos, weights, device="cuda:0")


@pytest.fixture(scope="module")
def gpu(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg


@pytest.mark.parametrize("name", HIER)
def test_node_logprob(gpu, name):
    g = load_golden(name)
    ix = index_from_golden(gpu, g)
    lp = ix.node_logprob(g["Xq"]).cpu().numpy()
    assert rel_err(lp, g["node_lp"]) < RTOL
    lpf = ix.node_logprob(g["Xq"][:4], full=True).cpu().numpy()
    assert rel_err(lpf, g["node_log_prob"]) < RTOL


@pytest.mark.parametrize("name", HIER)
def test_rank_scores_and_fast_topk(gpu, name):
    g = load_golden(name)
    ix = index_from_golden(gpu, g)
    rs = ix.rank_scores(g["Xq"]).cpu().numpy()
    assert rel_err(rs, g["rank_scores"]) < RTOL
    k = int(g["k"])
    ids, scores = ix.score_topk(g["Xq"], k)
    ids, scores = ids.cpu().numpy(), scores.cpu().numpy()
    for qi in range(len(g["Xq"])):
        ref = g["rank_scores"][qi].astype(np.float64)
        topk_equiv(ids[qi], g["fast_ids"][qi], ref)
        assert rel_err(scores[qi], ref[ids[qi]]) < RTOL


@pytest.mark.parametrize("name", HIER)
def test_categorize(gpu, name):
    g = load_golden(name)
    ix = index_from_golden(gpu, g)
    k = int(g["k"])
    nodes, found, calls = ix.categorize(g["Xq"], k)
    nodes, found, calls = nodes.cpu().numpy(), found.cpu().numpy(), calls.cpu().numpy()
    np.testing.assert_array_equal(found, k)
    np.testing.assert_array_equal(nodes, g["cat_nodes"])
    np.testing.assert_array_equal(calls, g["cat_calls"])


@pytest.mark.parametrize("pre", ["0", "1"])
@pytest.mark.parametrize("name", HIER)
def test_categorize_lazy_replay_goldens(gpu, name, pre, monkeypatch):
    """The exact lazy replay straight from the internal pass (CWQ_CAT_DIRECT=1, no lists),
    both run-merge kernels (CWQ_LAZY_PRE=0: packed arena; 1: one load round trip per pop),
    against the reference's own pop order and log_prob call counts -- goldens with internal
    nodes and an anisotropic leaf (g1, g4) exercise the lazily scored anisotropic rows; whole
    batch and one query per call; k past the retrievable leaves and a tiny max_nodes end as
    the reference's IndexError cases do."""
    g = load_golden(name)
    ix = index_from_golden(gpu, g)
    monkeypatch.setenv("CWQ_CAT_DIRECT", "1")
    monkeypatch.setenv("CWQ_LAZY_PRE", pre)
    k = int(g["k"])
    nodes, found, calls = ix.categorize(g["Xq"], k)
    assert ix.last_lazy_stats()["direct"] + ix.last_categorize_stats()["dense_reruns"] == len(g["Xq"])
    np.testing.assert_array_equal(found.cpu().numpy(), k)
    np.testing.assert_array_equal(nodes.cpu().numpy(), g["cat_nodes"])
    np.testing.assert_array_equal(calls.cpu().numpy(), g["cat_calls"])
    for qi in range(min(4, len(g["Xq"]))):
        n1, f1, c1 = ix.categorize(g["Xq"][qi:qi + 1], k)
        np.testing.assert_array_equal(n1.cpu().numpy()[0], g["cat_nodes"][qi])
        assert int(c1[0]) == int(g["cat_calls"][qi])
    if "err_k_too_big" in g:
        x = g["Xq"][:1]
        for kk, mx, key in [(int(g["n_leaf_nodes"]) + 1, 100000, "err_k_too_big"), (k, 4, "err_max_nodes")]:
            _, found, _ = ix.categorize(x, kk, mx)
            assert (int(found[0]) < kk) == bool(g[key])


@pytest.mark.parametrize("name", ["g1_hier_d32", "g5_hier_d384", "g2_flat_d768"])
def test_categorize_index_errors(gpu, name):
    """k > retrievable leaves, and a tiny max_nodes: n_found < k exactly where the
    reference raises IndexError (CobwebTorchTree.py:264-289)."""
    g = load_golden(name)
    ix = index_from_golden(gpu, g)
    x = g["Xq"][:1]
    for kk, mx, key in [(int(g["n_leaf_nodes"]) + 1, 100000, "err_k_too_big"), (int(g["k"]), 4, "err_max_nodes")]:
        _, found, _ = ix.categorize(x, kk, mx)
        assert (int(found[0]) < kk) == bool(g[key])


def test_level_weights(gpu):
    g = load_golden("g1_hier_d32")
    for w, key in [([1.0, 2.0, 0.5], "rank_scores_w3"), (list(g["weights_exp"]), "rank_scores_exp")]:
        ix = index_from_golden(gpu, g, w)
        assert rel_err(ix.rank_scores(g["Xq"]).cpu().numpy(), g[key]) < RTOL
    g = load_golden("g4_twolevel_d48")
    ix = index_from_golden(gpu, g, [0.25, 1.0, 3.0])
    assert rel_err(ix.rank_scores(g["Xq"]).cpu().numpy(), g["rank_scores_w3"]) < RTOL


@pytest.mark.parametrize("k", [1, 10, 16, 17, 64, 65, 300, 5000])
def test_topk_all_k_paths(gpu, k):
    """k <= 16 (DPP lists), 17..64 (wave lists), > 64 (materialise + sort), k >= N
    (full ranking, -1 padding past the sentence count)."""
    g = load_golden("g1_hier_d32")
    ix = index_from_golden(gpu, g)
    ids, scores = ix.score_topk(g["Xq"][:6], k)
    ids = ids.cpu().numpy()
    n = int(g["n_sent"])
    for qi in range(6):
        ref = g["rank_scores"][qi].astype(np.float64)
        order = np.lexsort((np.arange(n), -ref))
        m = min(k, n)
        topk_equiv(ids[qi][:m], order[:m], ref)
        assert np.all(ids[qi][m:] == -1)


def test_flat_synth_matches_reference_injected_index(gpu):
    """G3: the reference's own cobweb_predict_indexed on an injected flat index; the
    root stats of the GPU synthesiser are bit-identical to the reference Welford."""
    g = load_golden("g3_flat_inject_d32")
    X = torch.from_numpy(g["X"]).cuda()
    t = gpu.synth.flat_synth(X)
    cnt, mu, m2 = (v.cpu().numpy() for v in t["root"])
    assert cnt[0] == g["root_count"]
    np.testing.assert_array_equal(mu[0], g["root_mean"])
    np.testing.assert_array_equal(m2[0], g["root_meanSq"])
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    assert ix.info["isotropic_rows"] == len(g["X"])
    lp = ix.node_logprob(g["Xq"]).cpu().numpy()
    assert rel_err(lp, g["node_lp"]) < RTOL
    rs = ix.rank_scores(g["Xq"]).cpu().numpy()
    assert rel_err(rs, g["rank_scores"]) < RTOL
    ids, _ = ix.score_topk(g["Xq"], int(g["k"]))
    for qi, row in enumerate(ids.cpu().numpy()):
        topk_equiv(row, g["fast_ids"][qi], g["rank_scores"][qi].astype(np.float64))


def test_two_level_synth_vs_oracle(gpu):
    """Paths of length 3 on a synthesised two-level tree, against the oracle."""
    rng = np.random.default_rng(7)
    N, D, G = 6000, 80, 37
    C = rng.normal(0, 2, (G, D)).astype(np.float32)
    lab = rng.integers(0, G, N)
    X = (C[lab] + rng.standard_normal((N, D))).astype(np.float32)
    t = gpu.synth.two_level_synth(torch.from_numpy(X).cuda(), torch.from_numpy(lab))
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], [1.0, 0.5, 2.0],
                               device="cuda:0")
    root = O.ONode(D)
    root.count, root.mean, root.meanSq = O.F32(0), np.zeros(D, np.float32), np.zeros(D, np.float32)
    # oracle tree: same BFS layout
    mean = t["mean"].cpu().numpy()
    var = t["var"].cpu().numpy()
    paths = []
    nos = t["node_of_sentence"]
    par = t["parent"]
    for s in range(N):
        p, j = [], int(nos[s])
        while j >= 0:
            p.append(j)
            j = int(par[j])
        paths.append(p[::-1])
    ref_idx = O.FlatIndex(mean, var, par, paths, [1.0, 0.5, 2.0])
    Xq = np.concatenate([X[:8] + 0.05 * rng.standard_normal((8, D)).astype(np.float32),
                         (2 * rng.standard_normal((8, D))).astype(np.float32)])
    rs = ix.rank_scores(Xq).cpu().numpy()
    ref = O.rank_scores_batch(Xq, ref_idx)
    assert rel_err(rs, ref) < RTOL
    ids, _ = ix.score_topk(Xq, 10)
    for qi, row in enumerate(ids.cpu().numpy()):
        topk_equiv(row, O.topk_ids_scores(ref[qi], 10)[0], ref[qi].astype(np.float64))
    # Welford cluster stats: bit-identical to sequential numpy Welford over members
    for gid in [0, 5, G - 1]:
        members = np.sort(np.nonzero(lab == gid)[0])
        node = O.welford_rows(X[members])
        v = O.compute_var(node.meanSq, node.count)
        np.testing.assert_array_equal(mean[1 + gid], node.mean)
        np.testing.assert_array_equal(var[1 + gid], v)


def test_large_flat_properties(gpu):
    """Full-size-style property checks on a 200k x 768 flat tree: each perturbed
    corpus query finds its source row first; scores agree with the oracle on
    sampled queries; batch results do not depend on the batch split."""
    N, D = 200_000, 768
    X = gpu.synth.synthetic_corpus(N, D, seed=0)
    Q, targets = gpu.synth.synthetic_queries(X, 512, seed=1)
    t = gpu.synth.flat_synth(X)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    del t
    ids, scores = ix.score_topk(Q, 10)
    ids_np = ids.cpu().numpy()
    tg = targets.cpu().numpy()
    assert np.all(ids_np[:len(tg), 0] == tg)
    # descending scores
    s = scores.cpu().numpy()
    assert np.all(np.diff(s, axis=1) <= 0)
    # split invariance
    ids2, scores2 = ix.score_topk(Q[100:300], 10)
    np.testing.assert_array_equal(ids2.cpu().numpy(), ids_np[100:300])
    np.testing.assert_array_equal(scores2.cpu().numpy(), s[100:300])
    # oracle on 3 queries (full-size scan in numpy)
    Xn = X.cpu().numpy()
    ref_idx = O.flat_synth_index(Xn[:50_000])
    ix_small = gpu.index.CobwebIndex(**{k: v for k, v in gpu.synth.flat_synth(X[:50_000]).items()
                                        if k in ("mean", "var", "parent", "node_of_sentence")}, device="cuda:0")
    Qn = Q[[0, 1, 400]].cpu().numpy()
    got, gs = ix_small.score_topk(Qn, 10)
    for qi in range(3):
        ref = O.rank_scores(Qn[qi], ref_idx)
        topk_equiv(got[qi].cpu().numpy(), O.topk_ids_scores(ref, 10)[0], ref.astype(np.float64))
        assert rel_err(gs[qi].cpu().numpy(), ref[got[qi].cpu().numpy()]) < RTOL
