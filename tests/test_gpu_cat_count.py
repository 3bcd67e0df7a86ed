"""Basic categorize by counting (cat_count_kernel) == the exact heap replay.

The counting path resolves a query from the bottleneck order: every node with path
bottleneck b > G is popped before any node with b <= G, so the search up to
the group G that ends it is a SET (a count and a children sum over the internal nodes),
and only the group at G is replayed with the heap keys of CobwebTorchTree.py:243-285.
Here it must give exactly what the full heap replay gives (CWQ_CAT_COUNT=0): retrieved
nodes in pop order, n_found, log_prob call counts -- on two-level and deep trees, with
max_nodes cutting before / inside / after the retrievals, k from 1 to 64, perturbed
queries (a leaf closer than its parent: b ties along the path) and duplicated rows
(retrievals sharing one b: left to the replay).  The G1/G2/G4/G5 reference goldens go
through the counting path in tests/test_gpu_parity.py.  Lists that end inside a
bottleneck tie (a cluster of more than 64 leaves under one node) go through the two-level
replay (simulate_two_kernel), checked here against the DENSE re-run on device-ifit trees
of clustered data, where nearly every query's list ends in such a tie."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg


def _run(ix, Q, k, max_nodes, **env):
    old = {n: os.environ.get(n) for n in env}
    os.environ.update(env)
    try:
        out = ix.categorize(Q, k, max_nodes)
        torch.cuda.synchronize()
        return out, ix.last_categorize_stats()
    finally:
        for n, v in old.items():
            if v is None:
                del os.environ[n]
            else:
                os.environ[n] = v


def _both(ix, Q, k, max_nodes):
    """Counting path (default) and heap replay (CWQ_CAT_COUNT=0), both with the
    two-level replay of tied lists, against the replay whose every uncertified query
    goes DENSE (CWQ_CAT_COUNT=0 CWQ_CAT_TWO=0)."""
    ref, _ = _run(ix, Q, k, max_nodes, CWQ_CAT_COUNT="0", CWQ_CAT_TWO="0")
    rep, _ = _run(ix, Q, k, max_nodes, CWQ_CAT_COUNT="0")
    got, st = _run(ix, Q, k, max_nodes)
    for leg, res in (("replay", rep), ("count", got)):
        for name, a, b in zip(("nodes", "n_found", "n_calls"), ref, res):
            if not torch.equal(a, b):
                bad = (a != b).reshape(a.shape[0], -1).any(1).nonzero().flatten()[:4].tolist()
                raise AssertionError(f"{leg}: {name} differs (k={k}, max_nodes={max_nodes}, stats {st}) at queries "
                                     f"{bad}: dense {[a[i].tolist() for i in bad]} {leg} {[b[i].tolist() for i in bad]}; "
                                     f"found {[int(ref[1][i]) for i in bad]}, calls {[int(ref[2][i]) for i in bad]} vs "
                                     f"{[int(res[2][i]) for i in bad]}")
    return st


def _trees(pkg):
    g = torch.Generator(device="cuda:0")
    g.manual_seed(21)
    X = pkg.synth.synthetic_corpus(60_000, 48, seed=22)
    X[1000:1010] = X[2000]                                   # duplicated rows: equal b among retrievals
    lab = torch.randint(0, 600, (X.shape[0],), generator=g, device="cuda:0")
    yield "two-level G=600", pkg.synth.two_level_synth(X, lab), X
    lab = torch.randint(0, 20_000, (X.shape[0],), generator=g, device="cuda:0")
    yield "two-level G=20000", pkg.synth.two_level_synth(X, lab), X
    yield "balanced 4/6", pkg.synth.balanced_synth(X, 4, 6), X
    yield "balanced 10/3", pkg.synth.balanced_synth(X, 10, 3), X


def test_count_equals_replay(gpu):
    totals = {"by_count": 0, "by_replay": 0}
    for name, t, X in _trees(gpu):
        ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
        Q, _ = gpu.synth.synthetic_queries(X, 512, seed=23)
        Q[5] = X[2000]                                       # exactly on the duplicated row
        Q[6] = X[1000] + 1e-3
        n_int = ix.info["internal_nodes"]
        for k, mx in [(10, 100000), (1, 100000), (64, 100000), (10, n_int // 2), (10, n_int + 5), (5, 7),
                      (10, 2), (64, n_int + 40)]:
            try:
                st = _both(ix, Q, k, mx)
            except AssertionError as e:
                raise AssertionError(f"{name}: {e}") from None
            totals["by_count"] += st["by_count"]
            totals["by_replay"] += st["by_replay"]
        ix.close()
    # the counting path must carry the bulk of the queries
    assert totals["by_count"] > 0.8 * (totals["by_count"] + totals["by_replay"]), totals


def test_count_flat_tree_and_small(gpu):
    X = gpu.synth.synthetic_corpus(30_000, 32, seed=31)
    t = gpu.synth.flat_synth(X)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=32)
    for k, mx in [(10, 100000), (64, 100000), (10, 5), (10, 1), (1, 2)]:
        st = _both(ix, Q, k, mx)
        if k < 64:   # k = 64 = the list length: its last entry sits at the list's cut-off (DENSE)
            assert st["by_count"] >= 0.9 * Q.shape[0], (k, mx, st)
    ix.close()
    # a tree smaller than the list (every leaf in it): the search exhausts the heap
    t = gpu.synth.two_level_synth(X[:40].contiguous(), torch.arange(40, device="cuda:0") % 3)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    for k, mx in [(10, 100000), (39, 100000), (40, 100000), (41, 100000), (10, 3)]:
        if k <= 64:
            _both(ix, Q[:50], k, mx)
    ix.close()


@pytest.mark.parametrize("filt", [-1, 0])
def test_two_level_replay_on_clustered_ifit_tree(gpu, filt):
    """A device-ifit tree of 40 Gaussian clusters (C2's generator at 64 dims): the leaves of
    the query's cluster share the cluster node's lp as their bottleneck, so the top-64 list
    ends inside that tie for nearly every query.  Two-level replay == DENSE on every query
    (pop order, n_found, calls), for the filter and the exact-scan lists, and it must
    resolve most of them."""
    import random
    rng = np.random.default_rng(5)
    n, d, nc = 20_000, 64, 40
    C = rng.standard_normal((nc, d)).astype(np.float32) * 2.0
    X = (C[rng.integers(0, nc, n)] + 0.3 * rng.standard_normal((n, d))).astype(np.float32)
    random.seed(5)
    w = gpu.CobwebWrapper(corpus=None, corpus_embeddings=X)
    w.build_prediction_index()
    ix = w._index
    ix.set_filter(filt)
    Qn = np.concatenate([X[:192] + 0.05 * rng.standard_normal((192, d)),
                         C[rng.integers(0, nc, 64)] + 0.3 * rng.standard_normal((64, d))]).astype(np.float32)
    Q = torch.from_numpy(Qn).cuda()
    two = 0
    for k, mx in [(10, 100000), (1, 100000), (40, 100000), (63, 100000), (64, 100000), (10, 40), (10, 3)]:
        st = _both(ix, Q, k, mx)
        if (k, mx) == (10, 100000):
            two = st["two_level"]
    assert two >= 0.5 * Q.shape[0], two


@pytest.mark.parametrize("nq,spec", [(1, "1"), (8, "1"), (64, "1"), (1, "2"), (8, "2")])
def test_small_calls_stream_lists_equal_dense(gpu, nq, spec):
    """Calls of <= 64 queries take the per-call stream filter for both lists (the categorize
    key min(BF or T2 [parent], lp) in cwq_stream.hip) and replay the two-level lists on the
    chunk itself.  On the clustered device-ifit tree (every query ends in a bottleneck tie)
    and a two-level tree, pop order, n_found and calls equal the DENSE re-run and the batch
    call's rows, k = 10 and k = 64, max_nodes cutting inside the search too.  spec "1": the
    second list goes out speculatively after a call that needed it for every query; "2":
    always (CWQ_CAT_SPEC=2), so queries the first replay resolves are gated off the
    two-level replay (the two-level tree resolves most of them that way)."""
    import random
    rng = np.random.default_rng(7)
    n, d, nc = 20_000, 64, 40
    C = rng.standard_normal((nc, d)).astype(np.float32) * 2.0
    X = (C[rng.integers(0, nc, n)] + 0.3 * rng.standard_normal((n, d))).astype(np.float32)
    random.seed(7)
    w = gpu.CobwebWrapper(corpus=None, corpus_embeddings=X)
    w.build_prediction_index()
    Qn = np.concatenate([X[:96] + 0.05 * rng.standard_normal((96, d)),
                         C[rng.integers(0, nc, 32)] + 0.3 * rng.standard_normal((32, d))]).astype(np.float32)
    Q = torch.from_numpy(Qn).cuda()
    Xt = torch.from_numpy(X).cuda()
    g = torch.Generator(device="cuda:0")
    g.manual_seed(8)
    t = gpu.synth.two_level_synth(Xt, torch.randint(0, 300, (n,), generator=g, device="cuda:0"))
    ix2 = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    for ix in (w._index, ix2):
        for k, mx in [(10, 100000), (64, 100000), (10, 40)]:
            ref, _ = _run(ix, Q, k, mx, CWQ_CAT_COUNT="0", CWQ_CAT_TWO="0")
            for a in range(0, 128, nq):
                got, st = _run(ix, Q[a:a + nq].contiguous(), k, mx, CWQ_CAT_SPEC=spec)
                for name, x, y in zip(("nodes", "n_found", "n_calls"), ref, got):
                    assert torch.equal(x[a:a + nq], y), (name, k, mx, a, st)
    ix2.close()
