"""Tree-adaptive cut (cwq_api.hip plan_groups) on broad-rooted trees.

A Cobweb tree of a clustered corpus at scale has a few broad root children, each spanning
many clusters (the 500k x 768 device-ifit tree: 37 root children over 500 clusters).  The
round-4 cut centred every row at its depth-1 ancestor: there the centred norms shrink ~2x,
below the 4x rule, so the rows stayed root-centred, the bf16 bounds admitted whole clusters
and every query fell back to the exact scan.  The tree-adaptive cut splits a broad root
child down to its cluster-level nodes (group centres below depth 1, the split nodes become
top nodes the pruned query computes exactly).  Results must not change: Fast ids AND
scores bit-identical to the exact scan (batch, 1 / 8 / 64 queries per call, group pruning
on and off) and Basic's pop order, n_found and log_prob calls equal to the exact heap
replay.  Reference semantics: CobwebWrapper.py:210-265 (Fast), CobwebTorchTree.py:235-289
(Basic)."""
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


def broad_tree(gpu, n, d, fan, seed, direct=0.05, nq=256):
    """root -> fan[0] broad nodes -> fan[1] children each -> ... -> clusters -> rows.  Every
    level's centres are spread as widely as the level above (2.0 N(0, I) offsets), so a
    depth-1 node spans clusters as far apart as the whole corpus; rows = cluster centre +
    0.3 N(0, I).  A fraction `direct` of the rows hangs directly below a depth-1 node (rows
    whose parent is a top node once that node is split).  BFS order as CobwebIndex takes it."""
    rng = np.random.default_rng(seed)
    # internal nodes level by level: (parent bfs id, centre)
    levels = [[(-1, np.zeros(d, np.float32))]]
    for f in fan:
        lv = []
        for pi, (_, c) in enumerate(levels[-1]):
            for _ in range(f):
                lv.append((pi, c + 2.0 * rng.standard_normal(d).astype(np.float32)))
        levels.append(lv)
    clusters = levels[-1]
    nc = len(clusters)
    lab = rng.integers(0, nc, n)
    Cc = np.stack([c for _, c in clusters])
    X = (Cc[lab] + 0.3 * rng.standard_normal((n, d))).astype(np.float32)
    is_direct = rng.random(n) < direct
    d1 = len(levels[1])
    per_d1 = nc // d1
    # BFS ids: level offsets; depth-2 nodes of each depth-1 node: its internal children, then
    # its direct rows (by row index); deeper: internal children; the last level's rows by cluster
    parent, nos = [-1], np.full(n, -1, np.int64)
    bfs_of = [[0]]
    nid = 1
    for L in range(1, len(levels)):
        ids = []
        for j, (pi, _) in enumerate(levels[L]):
            ids.append(nid)
            parent.append(bfs_of[L - 1][pi])
            nid += 1
            if L == 2 and (j + 1) % fan[1] == 0:   # after a depth-1 node's children: its direct rows
                p1 = pi
                for r in np.nonzero(is_direct & (lab // per_d1 == p1))[0]:
                    parent.append(bfs_of[1][p1])
                    nos[r] = nid
                    nid += 1
        bfs_of.append(ids)
    order = np.argsort(lab * n + np.arange(n), kind="stable")
    for r in order:
        if is_direct[r]:
            continue
        parent.append(bfs_of[-1][lab[r]])
        nos[r] = nid
        nid += 1
    assert (nos >= 0).all()
    Xt = torch.from_numpy(X).cuda()
    t = gpu.synth.tree_synth(Xt, np.asarray(parent, np.int64), nos)
    h = nq // 2
    Q = np.concatenate([X[rng.choice(n, h, replace=False)] + 0.05 * rng.standard_normal((h, d)),
                        Cc[rng.integers(0, nc, nq - h)] + 0.3 * rng.standard_normal((nq - h, d))]).astype(np.float32)
    return t, torch.from_numpy(Q).cuda()


def make_index(gpu, t, monkeypatch, **env):
    for k in ("CWQ_GROUP_CUT", "CWQ_GROUP_CENTRE", "CWQ_GROUP_PRUNE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    for k in env:
        monkeypatch.delenv(k, raising=False)
    return ix


def _prune(on):
    if on:
        os.environ.pop("CWQ_GROUP_PRUNE", None)
    else:
        os.environ["CWQ_GROUP_PRUNE"] = "0"


def check_fast(ix, Q, k=10, per_call=(1, 8, 64), n_pc=96):
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, k)
    ix.set_filter(-1)
    try:
        out = {}
        for on in (False, True):
            _prune(on)
            ids, sc = ix.score_topk(Q, k)
            torch.cuda.synchronize()
            st, ps = ix.last_stats(), ix.last_prune_stats()
            bad = (ids != ids0).any(1).nonzero().flatten()[:4].tolist()
            assert torch.equal(ids, ids0) and torch.equal(sc, s0), (on, bad, st, ps)
            out[on] = (st, ps)
            for nq in per_call:
                for a in range(0, min(n_pc, Q.shape[0]), nq):
                    i3, s3 = ix.score_topk(Q[a:a + nq].contiguous(), k)
                    assert torch.equal(i3, ids0[a:a + nq]) and torch.equal(s3, s0[a:a + nq]), (on, nq, a)
    finally:
        _prune(True)
    return out


def check_basic(ix, Q, k=10, max_nodes=100000):
    got = ix.categorize(Q, k, max_nodes)
    ix.set_filter(0)
    os.environ["CWQ_CAT_COUNT"] = "0"
    try:
        ref = ix.categorize(Q, k, max_nodes)
    finally:
        del os.environ["CWQ_CAT_COUNT"]
        ix.set_filter(-1)
    for name, a, b in zip(("nodes", "n_found", "n_calls"), ref, got):
        assert torch.equal(a, b), name


def test_cut_broad_root_children(gpu, monkeypatch):
    """32 broad root children x 8 clusters (60k x 128): the cut centres the clusters
    (depth 2), the filter engages with no fallback query, pruning keeps the result."""
    t, Q = broad_tree(gpu, 60_000, 128, (32, 8), 61)
    ix = make_index(gpu, t, monkeypatch)
    cut, fi = ix.cut_info(), ix.filter_info()
    print("cut", cut, "filter", fi)
    assert fi["group_centred"], (cut, fi)
    assert cut["max_centre_depth"] == 2 and cut["groups"] >= 200 and cut["top_nodes"] <= 1 + 32, cut
    out = check_fast(ix, Q)
    st, ps = out[True]
    print("pruned", st, ps)
    assert st["filter_used"] and st["fallback_queries"] == 0, st
    assert ps["available"] and ps["queries"] == Q.shape[0], ps
    # beyond each query's best group little is computed
    assert ps["extra_pairs"] <= 0.05 * Q.shape[0] * ps["groups"], ps
    check_basic(ix, Q)
    check_basic(ix, Q[:64], k=5, max_nodes=50)
    # the round-4 depth-1 cut: the centred norms shrink ~2x, the mode stays off
    ix1 = make_index(gpu, t, monkeypatch, CWQ_GROUP_CUT="1")
    print("depth-1 cut", ix1.cut_info(), ix1.filter_info())
    assert not ix1.filter_info()["group_centred"] and ix1.cut_info()["max_centre_depth"] == 1
    ix1.close()
    ix.close()


def test_cut_three_levels_k1_k64(gpu, monkeypatch):
    """A deeper hierarchy (8 x 4 x 6, 48k x 96): centres at depth 3, two levels of top nodes;
    k = 1 and k = 64 (the seed threshold needs K rows of the best group)."""
    t, Q = broad_tree(gpu, 48_000, 96, (8, 4, 6), 62, direct=0.03)
    ix = make_index(gpu, t, monkeypatch)
    cut = ix.cut_info()
    print("cut", cut, ix.filter_info())
    assert ix.filter_info()["group_centred"] and cut["max_centre_depth"] == 3, cut
    for k in (1, 64):
        out = check_fast(ix, Q, k, per_call=(1, 64), n_pc=64)
        print(k, out[True])
        assert out[True][0]["fallback_queries"] == 0, out
    ix.close()


def test_cut_forced_depth1_matches(gpu, monkeypatch):
    """The same tree under the depth-1 cut forced on (CWQ_GROUP_CENTRE=1, CWQ_GROUP_CUT=1)
    and under the adaptive cut: the same ids and scores (each equal to the exact scan)."""
    t, Q = broad_tree(gpu, 30_000, 64, (16, 6), 63)
    ixa = make_index(gpu, t, monkeypatch)
    ixd = make_index(gpu, t, monkeypatch, CWQ_GROUP_CENTRE="1", CWQ_GROUP_CUT="1")
    assert ixd.filter_info()["group_centred"] and ixd.cut_info()["max_centre_depth"] == 1
    a = check_fast(ixa, Q, per_call=(1, 64), n_pc=64)
    d = check_fast(ixd, Q, per_call=(1, 64), n_pc=64)
    print("adaptive", a[True], "depth-1", d[True])
    ida, sa = ixa.score_topk(Q, 10)
    idd, sd = ixd.score_topk(Q, 10)
    assert torch.equal(ida, idd) and torch.equal(sa, sd)
    ixa.close()
    ixd.close()


@pytest.mark.parametrize("pre", ["0", "1"])
def test_lazy_dense_replay_equals_materialised(gpu, monkeypatch, pre):
    """Basic on a tree whose ties nest two levels deep (4 broad root children x 40 clusters:
    the root's lp is the lowest on every path, each broad child's the next lowest for all of
    its rows, so the two-level replay cannot certify and every query takes the DENSE re-run).
    The lazy DENSE replay (leaf rows scored when their parent is popped, CWQ_CAT_LAZY default)
    must give the materialised one's nodes, n_found and log_prob calls (CWQ_CAT_LAZY=0), for
    the batch and one query per call, k = 10 and k = 3 with a small max_nodes.  Both run-merge
    kernels: the packed one (CWQ_LAZY_PRE=0) and the one-round-trip one (1)."""
    t, Q = broad_tree(gpu, 40_000, 128, (4, 40), 64, direct=0.02, nq=128)
    ix = make_index(gpu, t, monkeypatch)
    monkeypatch.setenv("CWQ_LAZY_PRE", pre)
    for k, mx in ((10, 100000), (3, 40)):
        monkeypatch.setenv("CWQ_CAT_LAZY", "0")
        ref = ix.categorize(Q, k, mx)
        st_ref = ix.last_categorize_stats()
        monkeypatch.delenv("CWQ_CAT_LAZY")
        monkeypatch.setenv("CWQ_CAT_LAZY_RUNS", "0")   # the global-heap form alone
        heap = ix.categorize(Q, k, mx)
        monkeypatch.delenv("CWQ_CAT_LAZY_RUNS")
        got = ix.categorize(Q, k, mx)                  # the LDS run-merge form (default)
        st = ix.last_categorize_stats()
        print(k, mx, "materialised", st_ref, "lazy", st)
        for name, a, b, c in zip(("nodes", "n_found", "n_calls"), ref, got, heap):
            assert torch.equal(a, b) and torch.equal(a, c), (k, mx, name)
        if k == 10:
            assert st["dense_reruns"] >= Q.shape[0] // 2, st
        for i in range(0, 16):
            one = ix.categorize(Q[i:i + 1].contiguous(), k, mx)
            for name, a, b in zip(("nodes", "n_found", "n_calls"), ref, one):
                assert torch.equal(a[i:i + 1], b), (k, mx, i, name)
    check_basic(ix, Q[:64])
    ix.close()


@pytest.mark.parametrize("shape", ["nested ties", "ifit"])
def test_direct_lazy_replay(gpu, monkeypatch, shape):
    """Basic straight through the exact lazy replay (CWQ_CAT_DIRECT=1: the list paths
    skipped) against the list paths (CWQ_CAT_DIRECT=0), one and eight queries per call and a
    160-query batch, on
    the nested-tie tree and on a device-ifit clustered tree; the automatic choice tries the
    lazy path only after the lists left a query to the DENSE re-run, then keeps the faster."""
    import random
    if shape == "nested ties":
        t, Q = broad_tree(gpu, 30_000, 96, (4, 30), 65, direct=0.02, nq=160)
        ix = make_index(gpu, t, monkeypatch)
    else:
        rng = np.random.default_rng(66)
        C = rng.standard_normal((30, 64)).astype(np.float32) * 2.0
        X = (C[rng.integers(0, 30, 6000)] + 0.3 * rng.standard_normal((6000, 64))).astype(np.float32)
        random.seed(66)
        w = gpu.CobwebWrapper(corpus=None, corpus_embeddings=X)
        w.build_prediction_index()
        ix = w._index
        Q = torch.from_numpy((X[:160] + 0.05 * rng.standard_normal((160, 64))).astype(np.float32)).cuda()
    for k, mx in ((10, 100000), (4, 60)):
        for m in (1, 8):
            for a in range(0, 32, m):
                q = Q[a:a + m].contiguous()
                monkeypatch.setenv("CWQ_CAT_DIRECT", "0")
                ref = ix.categorize(q, k, mx)
                monkeypatch.setenv("CWQ_CAT_DIRECT", "1")
                got = ix.categorize(q, k, mx)
                assert ix.last_lazy_stats()["direct"] == m
                for name, x, y in zip(("nodes", "n_found", "n_calls"), ref, got):
                    assert torch.equal(x, y), (shape, k, mx, m, a, name)
        # a batch (> 64 queries): the run-merge replays side by side, arena overflows DENSE
        monkeypatch.setenv("CWQ_CAT_DIRECT", "0")
        ref = ix.categorize(Q, k, mx)
        monkeypatch.setenv("CWQ_CAT_DIRECT", "1")
        for pre in ("0", "1"):   # both run-merge kernels (packed / one round trip per pop)
            monkeypatch.setenv("CWQ_LAZY_PRE", pre)
            got = ix.categorize(Q, k, mx)
            lz, st = ix.last_lazy_stats(), ix.last_categorize_stats()
            assert lz["direct"] + st["dense_reruns"] == Q.shape[0], (lz, st)
            for name, x, y in zip(("nodes", "n_found", "n_calls"), ref, got):
                assert torch.equal(x, y), (shape, k, mx, "batch", pre, name)
        monkeypatch.delenv("CWQ_LAZY_PRE")
    monkeypatch.delenv("CWQ_CAT_DIRECT")
    # a fresh index for the automatic rule (the calls above fed the old one's record)
    if shape == "nested ties":
        ix.close()
        ix = make_index(gpu, t, monkeypatch)
    else:
        w._invalidate_prediction_index()
        w.build_prediction_index()
        ix = w._index
    seen = []
    for i in range(6):
        got = ix.categorize(Q[i:i + 1].contiguous(), 10, 100000)
        seen.append((ix.last_categorize_stats()["dense_reruns"], ix.last_lazy_stats()["direct"]))
        monkeypatch.setenv("CWQ_CAT_DIRECT", "0")
        ref = ix.categorize(Q[i:i + 1].contiguous(), 10, 100000)
        monkeypatch.delenv("CWQ_CAT_DIRECT")
        assert all(torch.equal(x, y) for x, y in zip(ref, got)), (shape, i)
    # batches under the automatic choice: the same results whichever path it takes
    for i in range(4):
        got = ix.categorize(Q, 10, 100000)
        monkeypatch.setenv("CWQ_CAT_DIRECT", "0")
        ref = ix.categorize(Q, 10, 100000)
        monkeypatch.delenv("CWQ_CAT_DIRECT")
        assert all(torch.equal(x, y) for x, y in zip(ref, got)), (shape, "batch", i)
    print(shape, seen)
    # the rule: the lazy path is tried only after a list-path call left a query to DENSE; then
    # the faster of the two (measured) is taken
    first_dense = next((i for i, (r, d) in enumerate(seen) if not d and r >= 1), None)
    for i, (r, d) in enumerate(seen):
        if d:
            assert first_dense is not None and i > first_dense, seen
    if shape == "nested ties":   # the lists leave every query DENSE; the lazy path is ~2.5x faster
        assert seen[0] == (1, 0) and seen[1][1] == 1 and sum(d for _, d in seen[2:]) >= 3, seen


def test_cut_500k_scale(gpu, monkeypatch):
    """The scale of the 500k x 768 device-ifit tree: 500k x 768 rows under 37
    broad root children x 14 clusters (518 clusters).  Fast: the filter engages with no
    fallback query and ids AND scores equal the exact scan (batch, 1 and 64 queries per
    call, pruning on and off).  Basic: the list paths, the exact heap replay and the exact
    lazy replay (CWQ_CAT_DIRECT=1, both run-merge kernels) give the same pop order, n_found
    and log_prob calls."""
    t, Q = broad_tree(gpu, 500_000, 768, (37, 14), 67, direct=0.02, nq=256)
    ix = make_index(gpu, t, monkeypatch)
    del t
    cut, fi = ix.cut_info(), ix.filter_info()
    print("cut", cut, "filter", fi)
    assert fi["group_centred"] and cut["max_centre_depth"] == 2 and cut["groups"] >= 500, (cut, fi)
    out = check_fast(ix, Q, per_call=(1, 64), n_pc=64)
    st, ps = out[True]
    print("pruned", st, ps)
    assert st["filter_used"] and st["fallback_queries"] == 0, st
    assert ps["available"] and ps["extra_pairs"] <= 0.05 * Q.shape[0] * ps["groups"], ps
    check_basic(ix, Q[:128])
    ref = ix.categorize(Q[:128], 10, 100000)
    for pre in ("0", "1"):
        monkeypatch.setenv("CWQ_CAT_DIRECT", "1")
        monkeypatch.setenv("CWQ_LAZY_PRE", pre)
        got = ix.categorize(Q[:128], 10, 100000)
        for name, a, b in zip(("nodes", "n_found", "n_calls"), ref, got):
            assert torch.equal(a, b), (pre, name)
        one = ix.categorize(Q[:1].contiguous(), 10, 100000)
        for name, a, b in zip(("nodes", "n_found", "n_calls"), ref, one):
            assert torch.equal(a[:1], b), (pre, "one query", name)
    ix.close()
