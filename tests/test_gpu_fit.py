"""GPU ifit (add path, CU scoring on libcwq) against trees built by the reference's
own ifit (golden G1, G5): identical structure, sentence placement and counts; and the
drop-in CobwebWrapper end to end (construct from embeddings -> query)."""
import random

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def bfs(root):
    out, q, h = [], [root], 0
    while h < len(q):
        n = q[h]
        h += 1
        out.append(n)
        q.extend(n.children)
    return out


@pytest.mark.parametrize("fitter", ["device", "host"])
@pytest.mark.parametrize("name", ["g1_hier_d32", "g5_hier_d384"])
def test_gpu_ifit_reproduces_reference_tree(pkg, name, fitter, monkeypatch):
    """fitter "device": the whole insert loop in one kernel (cwq_fitdev.hip); "host": the
    host-driven fitter (fit.py TreeFitter, one KL launch per level)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("CWQ_FIT_DEVICE", "1" if fitter == "device" else "0")
    g = load_golden(name)
    random.seed(0)   # gen_golden.py seeds the reference the same way
    w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(len(g["X"]))], corpus_embeddings=g["X"])
    nodes = bfs(w.tree.root)
    pos = {id(n): i for i, n in enumerate(nodes)}
    parent = np.array([-1 if n.parent is None else pos[id(n.parent)] for n in nodes])
    np.testing.assert_array_equal(parent, g["parent"])
    np.testing.assert_array_equal([s for n in nodes for s in n.sentence_id], g["sid_list"])
    np.testing.assert_array_equal(np.array([n.count for n in nodes], np.float32), g["count"])
    # the fit kernels use the reference's fp32 op order with contraction off: the node
    # statistics come out bit-identical (measured on MI355X: every mean/meanSq entry)
    np.testing.assert_array_equal(np.stack([n.mean for n in nodes]), g["mean"])
    np.testing.assert_array_equal(np.stack([n.meanSq for n in nodes]), g["meanSq"])
    # the drop-in answers like the reference
    k = int(g["k"])
    for qi in range(6):
        got = w.cobweb_predict_fast(g["Xq"][qi], k, return_ids=True)
        ref = g["fast_ids"][qi]
        rs = g["rank_scores"][qi]
        for a, b in zip(got, ref):
            if a != b:
                assert abs(rs[a] - rs[b]) <= 1e-5 * abs(rs[b])
        sent = w.cobweb_predict_fast(g["Xq"][qi], k)
        assert sent == [f"s{i}" for i in got]
        basic = w.cobweb_predict(g["Xq"][qi], k, return_ids=True)
        exp = [s for nid in g["cat_nodes"][qi] for s in
               sorted(g["sid_list"][g["sid_ptr"][nid]:g["sid_ptr"][nid + 1]])]
        assert basic == exp
    with pytest.raises(IndexError):
        w.cobweb_predict(g["Xq"][0], int(g["n_leaf_nodes"]) + 1)


def test_wrapper_json_roundtrip_and_add(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = load_golden("g1_hier_d32")
    random.seed(0)
    w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(200)], corpus_embeddings=g["X"][:200])
    w.add_sentences([f"s{i}" for i in range(200, 300)], g["X"][200:])   # incremental add, same stream
    w2 = pkg.CobwebWrapper.load_json(w.dump_json())
    assert len(w2) == 300
    for qi in range(4):
        a = w.cobweb_predict_fast(g["Xq"][qi], 10, return_ids=True)
        b = w2.cobweb_predict_fast(g["Xq"][qi], 10, return_ids=True)
        assert a == b


def _tree_arrays(root):
    nodes = bfs(root)
    pos = {id(n): i for i, n in enumerate(nodes)}
    parent = np.array([-1 if n.parent is None else pos[id(n.parent)] for n in nodes])
    return (parent, np.array([n.count for n in nodes], np.float32), np.stack([n.mean for n in nodes]),
            np.stack([n.meanSq for n in nodes]), [list(n.sentence_id) for n in nodes])


@pytest.mark.parametrize("D,n,clusters,fork_min", [(48, 1500, 12, None), (384, 600, 6, None), (768, 400, 0, None),
                                                   (64, 1200, 10, "2"), (96, 1500, 0, "64"), (768, 700, 0, "2"),
                                                   (5, 600, 4, None), (6, 500, 0, "2")])
def test_device_fit_equals_host_fit(pkg, D, n, clusters, fork_min, monkeypatch):
    """Device-resident ifit == host-driven ifit: structure, sentence placement, statistics
    bit for bit, and the random() stream position afterwards; with a batch split in two
    add_sentences calls (state carried over).  The device loop forks levels of >= 64
    children over every CU (flat N(0,I) rows: the root); fork_min forces forks at smaller
    levels -- every level, split passes included, at "2".  D = 5, 6: torch's scalar sum path
    (fewer than 8 elements) in the per-half sums as well."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if fork_min:
        monkeypatch.setenv("CWQ_FIT_FORK_MIN", fork_min)
    rng = np.random.default_rng(D + n)
    if clusters:
        C = rng.standard_normal((clusters, D)).astype(np.float32) * 2.0
        X = (C[rng.integers(0, clusters, n)] + 0.3 * rng.standard_normal((n, D))).astype(np.float32)
    else:
        X = rng.standard_normal((n, D)).astype(np.float32)
    X[n // 3] = X[n // 5]          # an exact match (leaf increment)
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("CWQ_FIT_DEVICE", mode)
        random.seed(7)
        w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(n // 2)], corpus_embeddings=X[:n // 2])
        w.add_sentences([f"s{i}" for i in range(n // 2, n)], X[n // 2:])
        res[mode] = (_tree_arrays(w.tree.root), random.random())
    (pa, ca, ma, sa, ia), ra = res["0"]
    (pb, cb, mb, sb, ib), rb = res["1"]
    np.testing.assert_array_equal(pa, pb)
    np.testing.assert_array_equal(ca, cb)
    np.testing.assert_array_equal(ma, mb)
    np.testing.assert_array_equal(sa, sb)
    assert ia == ib and ra == rb


def test_device_fit_matches_oracle_2k_clustered_768(pkg, monkeypatch):
    """The device-resident ifit on a 2,000-insert prefix of clustered 768-d data builds the
    oracle's tree (oracle/cobweb_oracle.py OTree.ifit -- the restatement pinned to the
    reference's own ifit trees G1/G5): same BFS structure, counts, sentence placement, and
    statistics bit for bit (CobwebTorchTree.py:143-233)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import cobweb_oracle as O
    monkeypatch.setenv("CWQ_FIT_DEVICE", "1")
    rng = np.random.default_rng(2024)
    n, D, k = 2000, 768, 20
    C = rng.standard_normal((k, D)).astype(np.float32) * 2.0
    X = (C[rng.integers(0, k, n)] + 0.3 * rng.standard_normal((n, D))).astype(np.float32)
    ot = O.OTree(D, rng=random.Random(5))
    for i in range(n):
        ot.ifit(X[i]).sentence_id.append(i)
    random.seed(5)
    w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(n)], corpus_embeddings=X)
    onodes = O.bfs_nodes(ot.root)
    opos = {id(x): i for i, x in enumerate(onodes)}
    oparent = np.array([-1 if x.parent is None else opos[id(x.parent)] for x in onodes])
    p, cnt, mean, m2, sids = _tree_arrays(w.tree.root)
    np.testing.assert_array_equal(p, oparent)
    np.testing.assert_array_equal(cnt, np.array([x.count for x in onodes], np.float32))
    assert sids == [list(x.sentence_id) for x in onodes]
    np.testing.assert_array_equal(mean, np.stack([x.mean for x in onodes]))
    np.testing.assert_array_equal(m2, np.stack([x.meanSq for x in onodes]))
    assert len(onodes) > 2 * k and max(len(x.children) for x in onodes) > 1


@pytest.mark.parametrize("fitter", ["device", "host"])
def test_interleaved_add_query_add_matches_reference(pkg, fitter, monkeypatch):
    """Golden G9 from the real reference: add -> Basic query (cobweb_predict) -> add ->
    query -> add on one global random() stream.  The drop-in's cobweb_predict advances
    the stream by the reference's categorize draws (CobwebTorchTree.py:243,268,285) and
    shuffles the retrieved leaves' lists with it (CobwebWrapper.py:456), so the returned
    ids, the tree the later inserts build and the final stream position all equal the
    reference's -- including a query that raises IndexError (max_init_search = 3)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("CWQ_FIT_DEVICE", "1" if fitter == "device" else "0")
    g = load_golden("g9_interleaved_d16")

    def ragged(ptr, ids):
        return [list(ids[ptr[i]:ptr[i + 1]]) for i in range(len(ptr) - 1)]

    random.seed(int(g["seed"]))
    w = pkg.CobwebWrapper(corpus=[f"a{i}" for i in range(len(g["XA"]))], corpus_embeddings=g["XA"])
    assert [w.cobweb_predict(q, 4, return_ids=True) for q in g["Q1"]] == ragged(g["out1_ptr"], g["out1_ids"])
    w.max_init_search = 3
    with pytest.raises(IndexError):
        w.cobweb_predict(g["Q1"][0], 4, return_ids=True)
    w.max_init_search = 100000
    w.add_sentences([f"b{i}" for i in range(len(g["XB"]))], g["XB"])
    assert [w.cobweb_predict(q, 5, return_ids=True) for q in g["Q2"]] == ragged(g["out2_ptr"], g["out2_ids"])
    w.add_sentences([f"c{i}" for i in range(len(g["XC"]))], g["XC"])
    assert random.random() == float(g["random_after"])
    p, cnt, mean, m2, sids = _tree_arrays(w.tree.root)
    np.testing.assert_array_equal(p, g["parent"])
    np.testing.assert_array_equal([s for x in sids for s in x], g["sid_list"])
    np.testing.assert_array_equal(cnt, g["count"])
    np.testing.assert_array_equal(mean, g["mean"])
    np.testing.assert_array_equal(m2, g["meanSq"])


@pytest.mark.parametrize("fail_at", [0, 3])
def test_device_fit_small_pool_reloads_and_fallback(pkg, fail_at, monkeypatch):
    """A node pool capped far below the batch (CWQ_FIT_POOL_SLOTS) makes the device fit
    stop for room many times; every reload exports the tree and the random() state and
    loads them into a fresh pool, with leaf identity kept across reloads.  fail_at > 0:
    the pool allocation of the fail_at-th load fails, and the remaining rows go through
    the host-driven fitter from the last export.  Either way the tree, its statistics,
    the sentence placement and the random() position equal the host fitter's."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(77)
    n, D, ncl = 600, 64, 8
    C = rng.standard_normal((ncl, D)).astype(np.float32) * 2.0
    X = (C[rng.integers(0, ncl, n)] + 0.4 * rng.standard_normal((n, D))).astype(np.float32)
    X[n // 2] = X[n // 7]
    res = {}
    monkeypatch.setenv("CWQ_FIT_DEVICE", "0")
    random.seed(11)
    w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(n)], corpus_embeddings=X)
    res["host"] = (_tree_arrays(w.tree.root), random.random())
    monkeypatch.setenv("CWQ_FIT_DEVICE", "1")
    monkeypatch.setenv("CWQ_FIT_POOL_SLOTS", "100")
    fitmod = __import__(type(w).__module__.rsplit(".", 1)[0] + ".fit", fromlist=["DeviceTreeFitter"])
    L = fitmod.lib()
    calls = {"n": 0}
    real_create = L.cwq_fit_create
    if fail_at:
        def create(*a):
            calls["n"] += 1
            return -3 if calls["n"] == fail_at else real_create(*a)
        monkeypatch.setattr(L, "cwq_fit_create", create)
    seen = []
    real_fit = fitmod.DeviceTreeFitter.fit_batch

    def fit_batch(self, Xb):
        r = real_fit(self, Xb)
        seen.append(dict(self.stats))
        return r
    monkeypatch.setattr(fitmod.DeviceTreeFitter, "fit_batch", fit_batch)
    random.seed(11)
    w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(n // 3)], corpus_embeddings=X[:n // 3])
    w.add_sentences([f"s{i}" for i in range(n // 3, n)], X[n // 3:])
    res["dev"] = (_tree_arrays(w.tree.root), random.random())
    (pa, ca, ma, sa, ia), ra = res["host"]
    (pb, cb, mb, sb, ib), rb = res["dev"]
    np.testing.assert_array_equal(pa, pb)
    np.testing.assert_array_equal(ca, cb)
    np.testing.assert_array_equal(ma, mb)
    np.testing.assert_array_equal(sa, sb)
    assert ia == ib and ra == rb
    loads = sum(st["loads"] for st in seen)
    if fail_at:
        assert sum(st["fallback"] is not None for st in seen) == 1
        assert sum(st["host_rows"] for st in seen) > 0 and calls["n"] == loads + 1
    else:
        assert all(st["fallback"] is None for st in seen) and loads > 3


def test_chip_wide_fit_flat_768_matches_oracle_1k_prefix(pkg, monkeypatch):
    """The chip-wide device ifit on flat N(0,I) 768-d rows -- the reference's high fan-out
    regime (every insert scores every root child, CobwebTorchNode.py:374-420) -- builds the
    oracle's tree over a 1,000-insert prefix of a 20k-row set (oracle/cobweb_oracle.py
    OTree.ifit, pinned to the reference's own trees G1/G5/G8): same structure, counts,
    sentence placement and statistics bit for bit, and the same random() position; and the
    one-workgroup loop (CWQ_FIT_HELPERS=0) builds the same tree."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import cobweb_oracle as O
    monkeypatch.setenv("CWQ_FIT_DEVICE", "1")
    X = np.random.default_rng(20_000).standard_normal((20_000, 768)).astype(np.float32)[:1000]
    ot = O.OTree(768, rng=random.Random(8))
    for i in range(len(X)):
        ot.ifit(X[i]).sentence_id.append(i)
    onodes = O.bfs_nodes(ot.root)
    opos = {id(x): i for i, x in enumerate(onodes)}
    want_r = ot.rng.random()
    for helpers in (None, "0"):
        if helpers is None:
            monkeypatch.delenv("CWQ_FIT_HELPERS", raising=False)
        else:
            monkeypatch.setenv("CWQ_FIT_HELPERS", helpers)
        random.seed(8)
        w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(len(X))], corpus_embeddings=X)
        p, cnt, mean, m2, sids = _tree_arrays(w.tree.root)
        np.testing.assert_array_equal(p, [-1 if x.parent is None else opos[id(x.parent)] for x in onodes])
        np.testing.assert_array_equal(cnt, np.array([x.count for x in onodes], np.float32))
        assert sids == [list(x.sentence_id) for x in onodes]
        np.testing.assert_array_equal(mean, np.stack([x.mean for x in onodes]))
        np.testing.assert_array_equal(m2, np.stack([x.meanSq for x in onodes]))
        assert random.random() == want_r
    assert len(ot.root.children) > 900

@pytest.mark.parametrize("call,rc", [("cwq_fit_insert", -2), ("cwq_fit_load", -2), ("cwq_fit_create", -1)])
def test_device_fit_non_oom_failure_raises(pkg, call, rc, monkeypatch):
    """Only a full pool (CWQ_ERR_OOM) sends the rest of a batch to the host fitter.  A HIP
    error -- which is how cwq_fit_insert reports a chip-wide KL pass that did not complete
    (FD_HANG) -- or bad arguments raise: a protocol fault must not hide behind a slower fit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(3)
    X = rng.standard_normal((40, 32)).astype(np.float32)
    monkeypatch.setenv("CWQ_FIT_DEVICE", "1")
    random.seed(3)
    w = pkg.CobwebWrapper(corpus=[f"s{i}" for i in range(20)], corpus_embeddings=X[:20])
    fitmod = __import__(type(w).__module__.rsplit(".", 1)[0] + ".fit", fromlist=["DeviceTreeFitter"])
    L = fitmod.lib()
    monkeypatch.setattr(L, call, lambda *a: rc)
    with pytest.raises(RuntimeError, match=f"{call} failed \\(status {rc}\\)"):
        w.add_sentences([f"s{i}" for i in range(20, 40)], X[20:])
