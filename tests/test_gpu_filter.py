"""bf16-MFMA candidate filter + exact rerank (cwq_mfma.hip): the filter changes how
the isotropic rows are searched, never the answer.  Every case compares the filter
(cwq_set_filter 1) with the exact fp32 scan (mode 0): ids AND scores bit-identical,
plus the reference goldens through the filter, mixed isotropic/anisotropic rows,
wide boundary ties, candidate-list overflow (exact fallback), and data with a large
common offset or scale."""
import numpy as np
import pytest

from conftest import load_golden
from test_gpu_parity import HIER, index_from_golden, rel_err, topk_equiv, RTOL

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


def both(ix, Q, k):
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, k)
    assert not ix.last_stats()["filter_used"]
    ix.set_filter(1)
    ids1, s1 = ix.score_topk(Q, k)
    st = ix.last_stats()
    ix.set_filter(-1)
    return ids0.cpu(), s0.cpu(), ids1.cpu(), s1.cpu(), st


@pytest.mark.parametrize("N,D,k", [(20000, 96, 10), (30000, 768, 10), (5000, 64, 1), (5000, 64, 32),
                                   (1000, 32, 16), (100, 32, 10), (40, 32, 32), (3000, 200, 7),
                                   (5000, 64, 64)])
def test_filter_equals_exact_scan(gpu, N, D, k):
    X = gpu.synth.synthetic_corpus(N, D, seed=N + D)
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=k)
    ids0, s0, ids1, s1, st = both(ix, Q, k)
    assert st["filter_used"] and st["filter_queries"] == 300
    assert torch.equal(ids0, ids1)
    assert torch.equal(s0, s1)
    assert st["fallback_queries"] <= 15, st


@pytest.mark.parametrize("name", HIER)
def test_goldens_through_filter(gpu, name):
    g = load_golden(name)
    ix = index_from_golden(gpu, g)
    ix.set_filter(1)
    k = int(g["k"])
    ids, scores = ix.score_topk(g["Xq"], k)
    assert ix.last_stats()["filter_used"]
    ids, scores = ids.cpu().numpy(), scores.cpu().numpy()
    for qi in range(len(g["Xq"])):
        ref = g["rank_scores"][qi].astype(np.float64)
        topk_equiv(ids[qi], g["fast_ids"][qi], ref)
        assert rel_err(scores[qi], ref[ids[qi]]) < RTOL


def test_mixed_iso_aniso_rows(gpu):
    """Leaves with per-dimension variances (count >= 2 leaves) go through the exact
    scan and are merged with the filtered isotropic rows."""
    X = gpu.synth.synthetic_corpus(6000, 64, seed=3)
    fs = gpu.synth.flat_synth(X)
    var = fs["var"].clone()
    g = torch.Generator(device=X.device)
    g.manual_seed(5)
    an = torch.randperm(6000, generator=g, device=X.device)[:700] + 1
    var[an] = var[an] * (0.5 + torch.rand((700, 64), generator=g, device=X.device))
    ix = gpu.index.CobwebIndex(fs["mean"], var, fs["parent"], fs["node_of_sentence"], device="cuda:0")
    assert ix.info["isotropic_rows"] == 5300
    Q, _ = gpu.synth.synthetic_queries(X, 200, seed=9)
    for k in (5, 20):
        ids0, s0, ids1, s1, st = both(ix, Q, k)
        assert st["filter_used"]
        assert torch.equal(ids0, ids1) and torch.equal(s0, s1)


def test_boundary_ties(gpu):
    """200 identical leaves around every query: the top-k boundary is a 200-way tie;
    every tied row is a candidate and is reranked exactly (ties -> lower row id)."""
    X = gpu.synth.synthetic_corpus(5000, 48, seed=11)
    X[1000:1200] = X[1000]
    ix = flat_index(gpu, X)
    Q = X[1000].repeat(50, 1) + 0.01 * gpu.synth.synthetic_corpus(50, 48, seed=12)
    ids0, s0, ids1, s1, st = both(ix, Q, 10)
    assert st["fallback_queries"] == 0, st
    assert st["exact_reranks"] >= 200, st
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)


def test_candidate_overflow_falls_back(gpu):
    """6000 identical leaves next to every query overflow the per-tile record lists and
    the per-query candidate lists: those queries are re-run by the exact scan."""
    X = gpu.synth.synthetic_corpus(20000, 64, seed=13)
    X[2000:8000] = X[2000]
    ix = flat_index(gpu, X)
    Q = torch.cat([X[2000].repeat(40, 1) + 0.01 * gpu.synth.synthetic_corpus(40, 64, seed=14),
                   gpu.synth.synthetic_queries(X, 60, seed=15)[0]])
    ids0, s0, ids1, s1, st = both(ix, Q, 10)
    assert st["fallback_queries"] >= 40, st
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)


def test_auto_mode_drops_a_failing_filter(gpu):
    """Auto mode: an index on which >= 9 in 10 of >= 256 filtered queries overflow their
    candidate lists (every query next to 6,000 identical leaves) takes the exact scan from then
    on -- same answers, the filter's pass no longer paid for nothing; mode 1 still forces it."""
    X = gpu.synth.synthetic_corpus(20000, 64, seed=17)
    X[2000:8000] = X[2000]
    ix = flat_index(gpu, X)
    Q = X[2000].repeat(300, 1) + 0.01 * gpu.synth.synthetic_corpus(300, 64, seed=18)
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, 10)
    ix.set_filter(-1)
    ids1, s1 = ix.score_topk(Q, 10)
    st = ix.last_stats()
    assert st["filter_used"] and st["fallback_queries"] >= 270, st
    ids2, s2 = ix.score_topk(Q, 10)
    assert not ix.last_stats()["filter_used"]
    ix.set_filter(1)
    ids3, s3 = ix.score_topk(Q, 10)
    assert ix.last_stats()["filter_used"]
    ix.set_filter(-1)
    for i, s_ in ((ids1, s1), (ids2, s2), (ids3, s3)):
        assert torch.equal(ids0, i) and torch.equal(s0, s_)


@pytest.mark.parametrize("shift,scale", [(50.0, 1.0), (0.0, 100.0), (0.0, 0.01), (-3.0, 7.0)])
def test_offset_and_scale(gpu, shift, scale):
    X = gpu.synth.synthetic_corpus(8000, 128, seed=21) * scale + shift
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, 200, seed=22, sigma=0.1 * scale)
    ids0, s0, ids1, s1, st = both(ix, Q, 10)
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    assert st["fallback_queries"] <= 10, st


def test_hierarchical_two_level(gpu):
    X = gpu.synth.synthetic_corpus(12000, 96, seed=31)
    g = torch.Generator(device=X.device)
    g.manual_seed(32)
    labels = torch.randint(0, 40, (12000,), generator=g, device=X.device)
    ts = gpu.synth.two_level_synth(X, labels)
    ix = gpu.index.CobwebIndex(ts["mean"], ts["var"], ts["parent"], ts["node_of_sentence"], device="cuda:0")
    Q, _ = gpu.synth.synthetic_queries(X, 256, seed=33)
    ids0, s0, ids1, s1, st = both(ix, Q, 10)
    assert st["filter_used"]
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)


@pytest.mark.parametrize("G", [1500, 6000])
def test_multi_parent_tiles(gpu, G, monkeypatch):
    """Small clusters put several parents in one 256-row tile (TileF uniform 2: pretest
    with the most permissive parent, per-row parent prefix for survivors).  Same answer
    as the exact scan, and as the generic per-element path (CWQ_FG_NO_MULTI)."""
    X = gpu.synth.synthetic_corpus(24000, 64, seed=G)
    g = torch.Generator(device=X.device)
    g.manual_seed(G + 1)
    labels = torch.randint(0, G, (24000,), generator=g, device=X.device)
    ts = gpu.synth.two_level_synth(X, labels)
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=G + 2)
    ix = gpu.index.CobwebIndex(ts["mean"], ts["var"], ts["parent"], ts["node_of_sentence"], device="cuda:0")
    ids0, s0, ids1, s1, st = both(ix, Q, 10)
    assert st["filter_used"] and st["fallback_queries"] <= 15, st
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    monkeypatch.setenv("CWQ_FG_NO_MULTI", "1")
    ix2 = gpu.index.CobwebIndex(ts["mean"], ts["var"], ts["parent"], ts["node_of_sentence"], device="cuda:0")
    ix2.set_filter(1)
    ids2, s2 = ix2.score_topk(Q, 10)
    assert torch.equal(ids0, ids2.cpu()) and torch.equal(s0, s2.cpu())


def test_multi_parent_tiles_clustered(gpu):
    """Well-separated small clusters: the parents inside one tile have very different path
    prefixes for a query, so the per-tile pretest bound spans a wide range -- the answer
    must still equal the exact scan bit for bit."""
    g = torch.Generator(device="cuda:0")
    g.manual_seed(5)
    G, per, D = 2400, 10, 48
    centers = torch.randn(G, D, generator=g, device="cuda:0") * 4.0
    labels = torch.arange(G, device="cuda:0").repeat_interleave(per)
    X = centers[labels] + 0.3 * torch.randn(G * per, D, generator=g, device="cuda:0")
    ts = gpu.synth.two_level_synth(X, labels)
    Q = X[torch.randperm(G * per, generator=g, device="cuda:0")[:300]] + \
        0.2 * torch.randn(300, D, generator=g, device="cuda:0")
    ix = gpu.index.CobwebIndex(ts["mean"], ts["var"], ts["parent"], ts["node_of_sentence"], device="cuda:0")
    ids0, s0, ids1, s1, st = both(ix, Q, 10)
    assert st["filter_used"]
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)


def test_auto_mode_threshold(gpu):
    X = gpu.synth.synthetic_corpus(20000, 32, seed=41)
    ix = flat_index(gpu, X)
    Q = X[:8].contiguous()
    ix.score_topk(Q, 10)
    assert ix.last_stats()["filter_used"]          # >= 16384 iso rows, k <= 64
    ix.score_topk(Q, 70)
    assert not ix.last_stats()["filter_used"]      # k > 64: exact scan (full ranking path)


def test_auto_mode_small_tree(gpu):
    """Automatic mode on a C1-sized tree (1.5k rows): per-call batches take the stream
    filter, larger batches the exact scan; the same answers either way."""
    X = gpu.synth.synthetic_corpus(1500, 384, seed=42)
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, 100, seed=43)
    ids1, s1 = ix.score_topk(Q[:5], 10)
    assert ix.last_stats()["path"] == "stream"
    ids2, s2 = ix.score_topk(Q, 10)
    assert ix.last_stats()["path"] == "scan"
    assert torch.equal(ids1, ids2[:5]) and torch.equal(s1, s2[:5])


@pytest.mark.parametrize("cuts,phases", [("64,256", None), ("8,16,32,64", None), ("1000", None), ("", None),
                                         ("", "0")])
def test_filter_phase_cuts(gpu, cuts, phases, monkeypatch):
    """Any split of the row tiles into filter launches (CWQ_FG_CUTS, read per call; the
    incremental tighten/final list carried across them, or no tighten at all with one
    launch) returns the exact scan's answer.  A first launch over most of the rows runs
    on the loose sample threshold alone and may overflow the record buffers: those
    queries fall back to the exact scan, which is the designed outcome, so the fallback
    count is bounded only for small first launches."""
    N, D, k = 24000, 128, 10
    X = gpu.synth.synthetic_corpus(N, D, seed=11)
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, 512, seed=5)
    monkeypatch.setenv("CWQ_FG_CUTS", cuts)
    if phases is not None:
        monkeypatch.setenv("CWQ_FG_PHASES", phases)
    ids0, s0, ids1, s1, st = both(ix, Q, k)
    assert st["filter_used"]
    assert torch.equal(ids0, ids1)
    assert torch.equal(s0, s1)
    if cuts in ("64,256", "8,16,32,64"):
        assert st["fallback_queries"] <= 20, st


@pytest.mark.parametrize("filt", [0, 1])
def test_query_chunking(gpu, filt, monkeypatch):
    """A batch larger than one workspace chunk (CWQ_WS_BUDGET_MB shrinks the 8 GiB budget,
    so the call splits into several query chunks — whole 256-query tiles on the filter
    path) returns what one chunk returns, ids and scores bit-identical."""
    N, D, k = 20000, 96, 10
    X = gpu.synth.synthetic_corpus(N, D, seed=21)
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, 1500, seed=22)
    ix.set_filter(filt)
    ids0, s0 = ix.score_topk(Q, k)
    monkeypatch.setenv("CWQ_WS_BUDGET_MB", "1")
    ids1, s1 = ix.score_topk(Q, k)
    ix.set_filter(-1)
    assert torch.equal(ids0.cpu(), ids1.cpu())
    assert torch.equal(s0.cpu(), s1.cpu())


@pytest.mark.parametrize("N,D,k,nq", [(60000, 768, 10, 1), (60000, 768, 10, 7), (60000, 768, 10, 64),
                                      (40000, 96, 1, 16), (40000, 96, 64, 17), (30000, 1024, 10, 33),
                                      (30000, 200, 5, 48), (20000, 256, 32, 64),
                                      (600, 384, 10, 1), (1500, 384, 10, 64)])   # small trees (auto: >= 512 rows)
def test_stream_path_equals_exact_scan(gpu, N, D, k, nq):
    """Small batches (nq <= 64) take the stream filter (cwq_stream.hip): bit-identical to
    the exact scan, with and without the filter's threshold probe finding the targets."""
    X = gpu.synth.synthetic_corpus(N, D, seed=N + D + k)
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, nq, seed=nq)
    ids0, s0, ids1, s1, st = both(ix, Q, k)
    assert st["path"] == "stream" and st["filter_queries"] == nq, st
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    assert st["fallback_queries"] == 0, st


@pytest.mark.parametrize("N,D,nq", [(60000, 768, 1), (60000, 768, 16), (40000, 1536, 3), (30000, 200, 64),
                                    (2000, 64, 5)])
def test_stream_int8_pass_equals_bf16_pass(gpu, N, D, nq, monkeypatch):
    """The stream filter's int8 pass (cwq_stream.hip I8: int8 rows and queries, exact int32
    products, per-row / per-query scales; on by default) and its bf16 pass select different
    candidate sets, never different answers: both bit-identical to the exact scan.  D = 200
    and 64 leave a partial 8-fragment load chunk, D = 768 / 1536 take 12-fragment chunks."""
    X = gpu.synth.synthetic_corpus(N, D, seed=N + D + 5)
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, nq, seed=nq + 2)
    st = {}
    for v in ("0", "1"):
        monkeypatch.setenv("CWQ_STREAM_I8", v)
        ids0, s0, ids1, s1, st[v] = both(ix, Q, 10)
        assert st[v]["path"] == "stream" and st[v]["fallback_queries"] == 0, st[v]
        assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    assert st["1"]["int8_pass"] and not st["0"]["int8_pass"], st
    if N >= 30000:   # the int8 bounds are wider: more candidates
        assert st["1"]["candidates"] > st["0"]["candidates"], st


@pytest.mark.parametrize("N", [4000, 20000])
def test_stream_near_duplicate_rows(gpu, N, monkeypatch):
    """Rows that nearly coincide: every row is a candidate.  N = 4000: the workgroups' LDS
    candidate buffers (kStreamSlots per query) overflow into the global lists; N = 20000:
    the query's list itself overflows and the exact fallback answers.  Still exact."""
    D = 64
    g = torch.Generator(device="cuda:0").manual_seed(N)
    base = torch.randn(D, device="cuda:0", generator=g)
    X = base + 1e-3 * torch.randn(N, D, device="cuda:0", generator=g)
    ix = flat_index(gpu, X)
    Q = X[:5] + 1e-4 * torch.randn(5, D, device="cuda:0", generator=g)
    for v in ("0", "1"):
        monkeypatch.setenv("CWQ_STREAM_I8", v)
        ids0, s0, ids1, s1, st = both(ix, Q, 10)
        assert st["path"] == "stream", st
        assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
        if N == 20000:
            assert st["fallback_queries"] == 5, st
        else:
            assert st["fallback_queries"] == 0 and st["candidates"] > 1000, st


@pytest.mark.parametrize("N,D,nq,k", [(60000, 768, 1, 10), (60000, 768, 3, 64), (4000, 64, 2, 10),
                                      (600, 384, 1, 10), (30000, 200, 64, 5)])
def test_stream_tail_split_equals_one_workgroup(gpu, N, D, nq, k, monkeypatch):
    """The per-call rerank tail split over several workgroups per query (FwExpand::split, the
    int8 pass: each reranks a slice of the candidate list, the last merges) returns what one
    workgroup per query returns, and both equal the exact scan: many candidates
    (near-duplicate rows at N = 4000), fewer candidates than workgroups (N = 600), k = 64."""
    if N == 4000:
        g = torch.Generator(device="cuda:0").manual_seed(N)
        base = torch.randn(D, device="cuda:0", generator=g)
        X = base + 1e-3 * torch.randn(N, D, device="cuda:0", generator=g)
    else:
        X = gpu.synth.synthetic_corpus(N, D, seed=N + D + 9)
    ix = flat_index(gpu, X)
    Q, _ = gpu.synth.synthetic_queries(X, nq, seed=nq + 9)
    monkeypatch.setenv("CWQ_STREAM_I8", "1")   # the split serves the int8 pass's long lists
    out = {}
    for v in ("1", "32"):
        monkeypatch.setenv("CWQ_FW_SPLIT", v)
        ids0, s0, ids1, s1, st = both(ix, Q, k)
        assert st["path"] == "stream" and st["int8_pass"] and st["fallback_queries"] == 0, st
        assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
        out[v] = (ids1, s1, st["exact_reranks"])
    assert torch.equal(out["1"][0], out["32"][0]) and torch.equal(out["1"][1], out["32"][1])
    assert out["1"][2] == out["32"][2]   # the split workgroups' exact reranks add up


@pytest.mark.parametrize("i8", ["0", "1"])
def test_stream_path_two_level_tree(gpu, i8, monkeypatch):
    """Stream filter on a hierarchical tree (per-row parent prefixes) and on a tree with
    anisotropic leaves (exact scan for those rows, merged with the stream candidates);
    bf16 and int8 filter passes."""
    monkeypatch.setenv("CWQ_STREAM_I8", i8)
    N, D = 50000, 128
    X = gpu.synth.synthetic_corpus(N, D, seed=77)
    labels = torch.randint(0, 500, (N,), device="cuda:0", generator=torch.Generator(device="cuda:0").manual_seed(1))
    ts = gpu.synth.two_level_synth(X, labels)
    var = ts["var"].clone()
    var[-100:, :7] *= 1.25          # 100 anisotropic leaves
    ix = gpu.index.CobwebIndex(ts["mean"], var, ts["parent"], ts["node_of_sentence"], device="cuda:0")
    Q, _ = gpu.synth.synthetic_queries(X, 40, seed=3)
    for k in (1, 10, 40):
        ids0, s0, ids1, s1, st = both(ix, Q, k)
        assert st["path"] == "stream", st
        assert torch.equal(ids0, ids1) and torch.equal(s0, s1)


def three_level(pkg, X, G1, S, seed=0):
    """root -> G1 clusters -> S sub-clusters each -> leaves (BFS order), node statistics
    by the GPU Welford builder (the reference's increment_counts order)."""
    N, D = X.shape
    g = torch.Generator(device=X.device)
    g.manual_seed(seed)
    l1 = torch.randint(0, G1, (N,), generator=g, device=X.device)
    l2 = l1 * S + torch.randint(0, S, (N,), generator=g, device=X.device)
    u1, inv1, c1 = torch.unique(l1, return_inverse=True, return_counts=True)
    u2, inv2, c2 = torch.unique(l2, return_inverse=True, return_counts=True)
    ar = torch.arange(N, device=X.device)
    o1 = torch.argsort(inv1 * N + ar)
    o2 = torch.argsort(inv2 * N + ar)
    p1 = torch.cat([torch.zeros(1, dtype=torch.int64, device=X.device), torch.cumsum(c1, 0)])
    p2 = torch.cat([torch.zeros(1, dtype=torch.int64, device=X.device), torch.cumsum(c2, 0)])
    n1, m1, q1 = pkg.index.welford_groups(X, o1, p1)
    n2, m2, q2 = pkg.index.welford_groups(X, o2, p2)
    n0, m0, q0 = pkg.index.welford_groups(X, ar, torch.tensor([0, N], device=X.device))
    var = lambda n, q: q / n[:, None] + float(pkg.PRIOR_VAR)   # noqa: E731
    G1n, G2n = u1.numel(), u2.numel()
    mean = torch.cat([m0, m1, m2, X[o2]])
    vv = torch.cat([var(n0, q0), var(n1, q1), var(n2, q2), torch.full((N, D), float(pkg.PRIOR_VAR), device=X.device)])
    par2 = 1 + torch.searchsorted(u1, u2 // S)                          # level-2 node -> its level-1 node
    parent = torch.cat([torch.tensor([-1]), torch.zeros(G1n, dtype=torch.int64), par2.cpu(),
                        1 + G1n + torch.repeat_interleave(torch.arange(G2n), c2.cpu())])
    nos = torch.empty(N, dtype=torch.int64)
    nos[o2.cpu()] = torch.arange(1 + G1n + G2n, 1 + G1n + G2n + N)
    return mean, vv, parent.numpy(), nos.numpy()


@pytest.mark.parametrize("N,D,G1,S,weights", [(60000, 128, 64, 8, None), (40000, 96, 200, 4, (1.0, 0.5, 2.0, 1.0)),
                                              (30000, 256, 16, 32, (0.3, 1.0, 1.0, 1.5))])
def test_internal_bounds_three_level(gpu, N, D, G1, S, weights):
    """Hierarchical trees through the filter with BOUNDED internal prefixes (bf16-MFMA
    internal-node bounds + exact parent chains in the rerank): ids and scores identical to
    the exact scan, for the batch filter (300 queries) and the stream filter (40)."""
    import os
    X = gpu.synth.synthetic_corpus(N, D, seed=N + G1)
    mean, var, parent, nos = three_level(gpu, X, G1, S)
    ix = gpu.index.CobwebIndex(mean, var, parent, nos, weights, device="cuda:0")
    assert ix.info["max_depth"] == 3
    for nq in (300, 40):
        Q, _ = gpu.synth.synthetic_queries(X, nq, seed=nq)
        for k in (1, 10):
            ids0, s0, ids1, s1, st = both(ix, Q, k)
            assert st["path"] == ("fgemm" if nq > 64 else "stream"), st
            assert torch.equal(ids0, ids1) and torch.equal(s0, s1), (nq, k, st)
    # the exact internal pass (bounds off) gives the same
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=300)
    ids1, s1 = ix.score_topk(Q, 10)
    os.environ["CWQ_INT_BOUND"] = "0"
    try:
        ids2, s2 = ix.score_topk(Q, 10)
    finally:
        del os.environ["CWQ_INT_BOUND"]
    assert torch.equal(ids1, ids2) and torch.equal(s1, s2)


@pytest.mark.parametrize("N,D,G,k", [(60000, 128, 0, 10), (60000, 768, 0, 1), (50000, 96, 300, 10),
                                     (40000, 64, 2000, 25), (30000, 256, 0, 64)])
def test_categorize_filter_equals_exact(gpu, N, D, G, k):
    """Basic query (categorize, A4) with the isotropic leaf rows through the bf16-MFMA
    filter on the categorize key min(BF[parent], lp): retrieved nodes in pop order, found
    counts and log_prob call counts identical to the exact scan of every leaf row."""
    X = gpu.synth.synthetic_corpus(N, D, seed=N + G + k)
    if G:
        labels = torch.randint(0, G, (N,), device="cuda:0", generator=torch.Generator(device="cuda:0").manual_seed(5))
        t = gpu.synth.two_level_synth(X, labels)
    else:
        t = gpu.synth.flat_synth(X)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=k)
    ix.set_filter(0)
    ref = ix.categorize(Q, k)
    ix.set_filter(1)
    got = ix.categorize(Q, k)
    ix.set_filter(-1)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("branching,depth", [(4, 6), (3, 8), (10, 3)])
@pytest.mark.parametrize("path", ["1", "0"])
def test_deep_balanced_tree(gpu, branching, depth, path, monkeypatch):
    """Deep trees shaped like Cobweb hierarchies (synth.balanced_synth): internal-node
    bounds as path sums over the leaf parents (CWQ_INT_PATH=1, default) or per node plus
    per-level prefix passes (0); multi-parent leaf tiles with up to ~90 parents; ids and
    scores identical to the exact scan, batch and per-call paths."""
    monkeypatch.setenv("CWQ_INT_PATH", path)
    X = gpu.synth.synthetic_corpus(30000, 64, seed=61)
    t = gpu.synth.balanced_synth(X, branching, depth, seed=62)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=63)
    for q in (Q, Q[:3]):
        ids0, s0, ids1, s1, st = both(ix, q, 10)
        assert st["filter_used"], st
        assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    ix.close()


def _bounds_tree(pkg, name):
    if name.startswith("three_level"):
        X = pkg.synth.synthetic_corpus(40000, 96, seed=71)
        mean, var, parent, nos = three_level(pkg, X, 200, 4)
        w = (1.0, -0.5, 2.0, 1.0) if name.endswith("negw") else (0.3, 1.0, 1.0, 1.5)
        return X, mean, var, np.asarray(parent), nos, w
    if name.startswith("balanced"):
        b, d = (int(v) for v in name.split("_")[1:])
        X = pkg.synth.synthetic_corpus(30000, 64, seed=72)
        t = pkg.synth.balanced_synth(X, b, d, seed=73)
    else:
        X = pkg.synth.synthetic_corpus(50000, 256, seed=74)
        lab = torch.randint(0, 3000, (X.shape[0],), device="cuda:0",
                            generator=torch.Generator(device="cuda:0").manual_seed(75))
        t = pkg.synth.two_level_synth(X, lab)
    return X, t["mean"], t["var"], np.asarray(t["parent"]), t["node_of_sentence"], None


@pytest.mark.parametrize("tree", ["three_level", "three_level_negw", "balanced_4_6", "balanced_3_8", "two_level"])
@pytest.mark.parametrize("path", ["1", "0"])
def test_prefix_bounds_enclose_exact(gpu, tree, path, monkeypatch):
    """The bf16-MFMA internal bounds the Fast filter reads enclose the exact pass's fp32
    path prefixes (cwq_prefix_bounds): path sums over the leaf parents (CWQ_INT_PATH=1)
    and per-node bounds + prefix passes (0), level weights incl. a negative one, queries
    near the data and far from it.  Every leaf parent has finite bounds; the widths stay
    far below the prefixes' magnitude (the pretest keeps its pruning power)."""
    monkeypatch.setenv("CWQ_INT_PATH", path)
    X, mean, var, parent, nos, w = _bounds_tree(gpu, tree)
    ix = gpu.index.CobwebIndex(mean, var, parent, nos, w, device="cuda:0")
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=76)
    g = torch.Generator(device="cuda:0").manual_seed(77)
    Q = torch.cat([Q, 3.0 * torch.randn(40, X.shape[1], device="cuda:0", generator=g)])
    lo, hi, ex = ix.prefix_bounds(Q)
    n = parent.shape[0]
    nch = np.bincount(parent[1:], minlength=n)
    internal = np.nonzero(nch > 0)[0]
    leafpar = np.zeros(n, dtype=bool)
    kids = np.arange(1, n)
    leafpar[parent[1:][nch[kids] == 0]] = True
    need = torch.from_numpy(leafpar[internal]).to("cuda:0")
    fin = torch.isfinite(lo) & torch.isfinite(hi)
    assert bool(fin[:, need].all()), "a leaf parent without bounds"
    if path == "0":
        assert bool(fin.all())
    assert bool(torch.isfinite(ex).all())
    ok = (lo <= ex) & (ex <= hi)
    bad = (~ok & fin).nonzero()
    assert bad.shape[0] == 0, [(int(q), int(i), float(lo[q, i]), float(ex[q, i]), float(hi[q, i]))
                               for q, i in bad[:5].tolist()]
    rel = ((hi - lo) / ex.abs().clamp_min(1.0))[fin]
    print(f"{tree} path={path}: rel width median {float(rel.median()):.2e} max {float(rel.max()):.2e}")
    assert float(rel.median()) < 5e-2
    ix.close()


def ragged_tree(pkg, X, G1, S, seed=0):
    """root -> G1 clusters; even clusters hold their leaves directly (depth 2), odd ones
    through S sub-clusters (depth 3).  In BFS order the depth-2 leaf parents (the even
    clusters) alternate with internal nodes that have no leaf directly below them, so a
    leaf tile's parent range [par, par_hi] spans internal ids with no path-sum operand row.
    Node statistics by the GPU Welford builder."""
    N, D = X.shape
    g = torch.Generator(device=X.device)
    g.manual_seed(seed)
    l1 = torch.randint(0, G1, (N,), generator=g, device=X.device).cpu().numpy()
    sub = torch.randint(0, S, (N,), generator=g, device=X.device).cpu().numpy()
    u1 = np.unique(l1)
    rows_of = {c: np.nonzero(l1 == c)[0] for c in u1}
    depth2, depth3, l2groups = [], [], []   # depth-2 entries: ("leaf", row) | ("int", group rows)
    for c in u1:
        if c % 2 == 0:
            depth2 += [("leaf", int(r)) for r in rows_of[c]]
        else:
            for sg in np.unique(sub[rows_of[c]]):
                gr = rows_of[c][sub[rows_of[c]] == sg]
                depth2.append(("int", len(l2groups)))
                l2groups.append(gr)
    for gr in l2groups:
        depth3 += [int(r) for r in gr]

    def stats(groups):
        order = torch.from_numpy(np.concatenate(groups)).to(X.device)
        ptr = torch.from_numpy(np.cumsum([0] + [len(x) for x in groups])).to(X.device)
        n, m, q = pkg.index.welford_groups(X, order, ptr)
        return m, q / n[:, None] + float(pkg.PRIOR_VAR)

    m0, v0 = stats([np.arange(N)])
    m1, v1 = stats([rows_of[c] for c in u1])
    m2, v2 = stats(l2groups)
    G1n = len(u1)
    parent, nos = [-1] + [0] * G1n, np.empty(N, dtype=np.int64)
    mean_parts, var_parts = [m0, m1], [v0, v1]
    int_node = {}
    pos = 1 + G1n
    leaf_rows = []
    ci = {c: 1 + i for i, c in enumerate(u1)}
    for kind, v in depth2:
        if kind == "leaf":
            parent.append(ci[l1[v]])
            nos[v] = pos
            leaf_rows.append(v)
        else:
            parent.append(ci[l1[l2groups[v][0]]])
            int_node[v] = pos
        pos += 1
    d2_leaf = torch.from_numpy(np.asarray(leaf_rows, dtype=np.int64)).to(X.device)
    for gi, gr in enumerate(l2groups):
        for r in gr:
            parent.append(int_node[gi])
            nos[r] = pos
            pos += 1
    # depth-2 node means/vars in BFS order: leaves (X rows, prior var) and level-2 groups
    d2m, d2v = [], []
    for kind, v in depth2:
        if kind == "leaf":
            d2m.append(X[v:v + 1])
            d2v.append(torch.full((1, D), float(pkg.PRIOR_VAR), device=X.device))
        else:
            d2m.append(m2[v:v + 1])
            d2v.append(v2[v:v + 1])
    d3 = torch.from_numpy(np.asarray(depth3, dtype=np.int64)).to(X.device)
    mean = torch.cat(mean_parts + d2m + [X[d3]])
    var = torch.cat(var_parts + d2v + [torch.full((len(depth3), D), float(pkg.PRIOR_VAR), device=X.device)])
    assert mean.shape[0] == len(parent) and int(d2_leaf.numel()) + len(depth3) == N
    return mean, var, np.asarray(parent, dtype=np.int64), nos


def test_ragged_tree_parent_gaps(gpu):
    """Leaves at depths 2 and 3 (ragged_tree): multi-parent leaf tiles whose parent ranges
    include internal nodes with no leaf below them (no path-sum operand row, PathB
    par -2).  The filter's ids and scores equal the exact scan's, batch and per-call; the
    path-sum bounds enclose the exact prefixes of every leaf parent."""
    X = gpu.synth.synthetic_corpus(40000, 96, seed=81)
    mean, var, parent, nos = ragged_tree(gpu, X, 120, 3)
    ix = gpu.index.CobwebIndex(mean, var, parent, nos, device="cuda:0")
    assert ix.info["max_depth"] == 3
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=82)
    for q in (Q, Q[:5]):
        for k in (1, 10):
            ids0, s0, ids1, s1, st = both(ix, q, k)
            assert st["filter_used"], st
            assert torch.equal(ids0, ids1) and torch.equal(s0, s1), (q.shape[0], k, st)
    lo, hi, ex = ix.prefix_bounds(Q[:100])
    fin = torch.isfinite(lo) & torch.isfinite(hi)
    assert bool(((lo <= ex) | ~fin).all()) and bool(((ex <= hi) | ~fin).all())
    ix.close()
