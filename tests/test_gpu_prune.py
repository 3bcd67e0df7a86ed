"""Group pruning of the Fast query (cwq_prune.hip) against the exact fp32 scan.

On a group-centred (clustered) tree the Fast path computes the exact internal pass only
for each query's best depth-1 group and for the groups whose certified key bound reaches
the filter's first threshold; every other group's rows get a sentinel prefix and can never
be candidates.  Results must not change: ids AND scores bit-identical to the exact scan and
to the same filter with pruning off (CWQ_GROUP_PRUNE=0 per call), for the batch filter and
for one / 8 / 64 queries per call (the stream filter), including queries between clusters
(several groups relevant: stage B must add them), anisotropic leaf rows inside groups (their
exact scan reads the sentinel prefixes), and k = 1 / 64.  A negative level weight makes the
key bound invalid: the index must not prune.  Reference semantics: CobwebWrapper.py:210-265."""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg


def clustered(n, d, nc, seed, nq=256):
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    C = 2.0 * torch.randn((nc, d), generator=g, device="cuda:0")
    lab = torch.randint(0, nc, (n,), generator=g, device="cuda:0")
    X = (C[lab] + 0.3 * torch.randn((n, d), generator=g, device="cuda:0")).contiguous()
    h = nq // 2
    Q = torch.cat([X[:h] + 0.05 * torch.randn((h, d), generator=g, device="cuda:0"),
                   C[torch.randint(0, nc, (nq - h,), generator=g, device="cuda:0")] +
                   0.3 * torch.randn((nq - h, d), generator=g, device="cuda:0")]).contiguous()
    return X, lab, Q, C


def _call(ix, Q, k, prune):
    old = os.environ.get("CWQ_GROUP_PRUNE")
    if prune:
        os.environ.pop("CWQ_GROUP_PRUNE", None)
    else:
        os.environ["CWQ_GROUP_PRUNE"] = "0"
    try:
        out = ix.score_topk(Q, k)
        torch.cuda.synchronize()
        return out, ix.last_prune_stats(), ix.last_stats()
    finally:
        if old is None:
            os.environ.pop("CWQ_GROUP_PRUNE", None)
        else:
            os.environ["CWQ_GROUP_PRUNE"] = old


def check_pruned(ix, Q, k=10, per_call=(1, 8, 64), n_pc=128):
    """Exact scan == filter without pruning == filter with pruning, batch and per call.
    Returns the pruned batch call's prune stats."""
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, k)
    ix.set_filter(-1)
    (i1, s1), p1, st1 = _call(ix, Q, k, False)
    assert p1["queries"] == 0, p1
    assert torch.equal(i1, ids0) and torch.equal(s1, s0)
    (i2, s2), p2, st2 = _call(ix, Q, k, True)
    assert st2["filter_used"], st2
    assert p2["available"] and p2["queries"] == Q.shape[0], p2
    bad = (i2 != ids0).any(1).nonzero().flatten()[:4].tolist()
    assert torch.equal(i2, ids0) and torch.equal(s2, s0), (bad, p2)
    for nq in per_call:
        for a in range(0, min(n_pc, Q.shape[0]), nq):
            (i3, s3), p3, st3 = _call(ix, Q[a:a + nq].contiguous(), k, True)
            assert p3["queries"] == nq and st3["path"] == "stream", (nq, p3, st3)
            assert torch.equal(i3, ids0[a:a + nq]) and torch.equal(s3, s0[a:a + nq]), (nq, a, p3)
    return p2


def test_prune_clustered_two_level(gpu):
    X, lab, Q, _ = clustered(60_000, 128, 150, 51)
    t = gpu.synth.two_level_synth(X, lab)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    assert ix.filter_info()["group_centred"]
    for k in (10, 1, 64):
        p = check_pruned(ix, Q, k, per_call=(1, 64) if k != 10 else (1, 8, 64))
        print(k, p)
        # separated clusters: beyond each query's best group little is computed
        assert p["extra_pairs"] <= 0.05 * Q.shape[0] * p["groups"], (k, p)
    ix.close()


def test_prune_queries_between_clusters(gpu):
    """Queries at the midpoint of two cluster centres: both clusters are relevant, so stage B
    must compute the second one (and possibly more)."""
    X, lab, _, C = clustered(40_000, 64, 60, 52)
    t = gpu.synth.two_level_synth(X, lab)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(53)
    a = torch.randint(0, 60, (256,), generator=g, device="cuda:0")
    b = (a + 1 + torch.randint(0, 59, (256,), generator=g, device="cuda:0")) % 60
    w = torch.rand((256, 1), generator=g, device="cuda:0") * 0.2 + 0.4
    Q = (w * C[a] + (1 - w) * C[b] + 0.05 * torch.randn((256, 64), generator=g, device="cuda:0")).contiguous()
    p = check_pruned(ix, Q)
    print(p)
    assert p["extra_pairs"] > 0, p
    ix.close()


def test_prune_device_ifit_tree(gpu, monkeypatch):
    """A device-ifit tree of 40 Gaussian clusters (C2's generator at 64 dims): deep groups.
    At 64 dims the automatic rule leaves the rows root-centred; the group mode is forced."""
    monkeypatch.setenv("CWQ_GROUP_CENTRE", "1")
    rng = np.random.default_rng(54)
    n, d, nc = 20_000, 64, 40
    C = rng.standard_normal((nc, d)).astype(np.float32) * 2.0
    X = (C[rng.integers(0, nc, n)] + 0.3 * rng.standard_normal((n, d))).astype(np.float32)
    random.seed(54)
    w = gpu.CobwebWrapper(corpus=None, corpus_embeddings=X)
    w.build_prediction_index()
    ix = w._index
    assert ix.filter_info()["group_centred"] and ix.info["max_depth"] >= 4, ix.info
    Qn = np.concatenate([X[:192] + 0.05 * rng.standard_normal((192, d)),
                         C[rng.integers(0, nc, 64)] + 0.3 * rng.standard_normal((64, d))]).astype(np.float32)
    p = check_pruned(ix, torch.from_numpy(Qn).cuda())
    # (at 64 dims ifit's depth-1 nodes each hold several of the 40 clusters -- 11 groups --
    # so a group's radius spans clusters and little is pruned: exactness is the point here)
    print(p)


def test_prune_with_anisotropic_rows(gpu):
    """Every 7th leaf row made anisotropic (count > 1 variances): those rows go through the
    exact scan, which reads the pruned groups' sentinel prefixes."""
    X, lab, Q, _ = clustered(30_000, 96, 80, 55)
    t = gpu.synth.two_level_synth(X, lab)
    var = t["var"].clone()
    n_int = 1 + t["n_clusters"]
    g = torch.Generator(device="cuda:0")
    g.manual_seed(56)
    rows = torch.arange(n_int, var.shape[0], 7, device="cuda:0")
    var[rows] = var[rows] * (1.0 + 0.5 * torch.rand((rows.numel(), var.shape[1]), generator=g, device="cuda:0"))
    ix = gpu.index.CobwebIndex(t["mean"], var, t["parent"], t["node_of_sentence"], device="cuda:0")
    assert ix.info["leaf_rows"] > ix.info["isotropic_rows"] and ix.filter_info()["group_centred"], ix.info
    check_pruned(ix, Q)
    ix.close()


def test_no_prune_with_negative_level_weight(gpu):
    X, lab, Q, _ = clustered(20_000, 64, 40, 57, nq=128)
    t = gpu.synth.two_level_synth(X, lab)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], [1.0, -0.5, 1.0],
                               device="cuda:0")
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, 10)
    ix.set_filter(-1)
    ids1, s1 = ix.score_topk(Q, 10)
    assert not ix.last_prune_stats()["available"]
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    ix.close()


def test_live_block_list_equals_full_pass(gpu, monkeypatch):
    """The per-call filter passes over the live 16-row blocks only (blocks whose rows all lie
    in groups pruned for every query of the call are left out, prune_stage_b_kernel): same
    ids and scores as the pass over every block (CWQ_PRUNE_LIVE=0) and as the exact scan,
    for 1 / 8 / 64 queries per call, queries inside and between clusters."""
    X, lab, Q, C = clustered(50_000, 96, 120, 58, nq=128)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(59)
    a = torch.randint(0, 120, (64,), generator=g, device="cuda:0")
    mid = (0.5 * C[a] + 0.5 * C[(a + 7) % 120]).contiguous()
    Q = torch.cat([Q, mid]).contiguous()
    t = gpu.synth.two_level_synth(X, lab)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, 10)
    ix.set_filter(-1)
    for nq in (1, 8, 64):
        for a0 in range(0, Q.shape[0], max(nq, 16)):
            q = Q[a0:a0 + nq].contiguous()
            out = {}
            for v in ("0", "1"):
                monkeypatch.setenv("CWQ_PRUNE_LIVE", v)
                ids, sc = ix.score_topk(q, 10)
                assert ix.last_stats()["path"] == "stream" and ix.last_prune_stats()["queries"] == q.shape[0]
                out[v] = (ids, sc)
            m = q.shape[0]
            assert torch.equal(out["0"][0], ids0[a0:a0 + m]) and torch.equal(out["0"][1], s0[a0:a0 + m]), (nq, a0)
            assert torch.equal(out["1"][0], ids0[a0:a0 + m]) and torch.equal(out["1"][1], s0[a0:a0 + m]), (nq, a0)
    ix.close()
