"""Small-batch code paths (the reference harness's one-query-per-call mode and small
serving batches) against their large-batch / exact counterparts, bit for bit:

* the per-call stream path's fused prep (`sb_prep_kernel`: padded queries, bf16 prep,
  exact internal pass, counter clear) vs the unfused launches (CWQ_SB_UNFUSED), on trees
  whose internal pass is exact (anisotropic leaf rows) with few and with many internal
  nodes, vs the exact scan;
* the workgroup-per-query rerank (`final_wide_kernel`) vs the wave-per-query one
  (CWQ_FINAL_WIDE=0), flat and hierarchical (exact parent chains);
* the exact scan's shared-query configuration (calls of <= 256 queries) vs the
  query-per-wave one (larger calls): rank scores, node log-probs, Fast top-k and
  categorize of a query must not depend on the size of the call it arrives in."""
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg


def two_level(pkg, N, D, G, n_aniso, seed):
    X = pkg.synth.synthetic_corpus(N, D, seed=seed)
    lab = torch.randint(0, G, (N,), device="cuda:0", generator=torch.Generator(device="cuda:0").manual_seed(seed + 1))
    t = pkg.synth.two_level_synth(X, lab)
    var = t["var"].clone()
    if n_aniso:
        g = torch.Generator(device="cuda:0")
        g.manual_seed(seed + 2)
        leaf0 = var.shape[0] - N   # BFS: root, clusters, then the leaves
        an = torch.randperm(N, generator=g, device="cuda:0")[:n_aniso] + leaf0
        var[an] = var[an] * (0.5 + torch.rand((n_aniso, D), generator=g, device="cuda:0"))
    ix = pkg.index.CobwebIndex(t["mean"], var, t["parent"], t["node_of_sentence"], device="cuda:0")
    return X, ix


def run(ix, Q, k, mode):
    ix.set_filter(mode)
    ids, s = ix.score_topk(Q, k)
    st = ix.last_stats()
    ix.set_filter(-1)
    return ids.cpu(), s.cpu(), st


@pytest.mark.parametrize("G", [20, 150])
def test_stream_prep_fused_vs_unfused_vs_exact(gpu, G, monkeypatch):
    X, ix = two_level(gpu, 24000, 96, G, 300, seed=31)
    Q, _ = gpu.synth.synthetic_queries(X, 64, seed=32)
    for nq in (1, 7, 64):
        ref = run(ix, Q[:nq], 10, 0)
        fused = run(ix, Q[:nq], 10, 1)
        assert fused[2]["path"] == "stream", fused[2]
        monkeypatch.setenv("CWQ_SB_UNFUSED", "1")
        unf = run(ix, Q[:nq], 10, 1)
        monkeypatch.delenv("CWQ_SB_UNFUSED")
        for got in (fused, unf):
            assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    ix.close()


@pytest.mark.parametrize("tree", ["flat", "two_level"])
def test_final_wide_vs_wave(gpu, tree, monkeypatch):
    if tree == "flat":
        X = gpu.synth.synthetic_corpus(30000, 128, seed=41)
        fs = gpu.synth.flat_synth(X)
        ix = gpu.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device="cuda:0")
    else:   # isotropic leaves: internal-node bounds + exact parent chains in the rerank
        X, ix = two_level(gpu, 30000, 128, 300, 0, seed=42)
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=43)
    for nq in (1, 100, 300):   # stream path, batch path (wide), batch path (wave)
        wide = run(ix, Q[:nq], 10, 1)
        monkeypatch.setenv("CWQ_FINAL_WIDE", "0")
        wave = run(ix, Q[:nq], 10, 1)
        monkeypatch.delenv("CWQ_FINAL_WIDE")
        ref = run(ix, Q[:nq], 10, 0)
        assert wide[2]["filter_used"] and wide[2]["fallback_queries"] == 0, wide[2]
        for got in (wide, wave):
            assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    ix.close()


def test_scan_config_independent_of_call_size(gpu):
    """300 queries in one call (query-per-wave scan) vs the same queries in calls of 100
    and 1 (shared-query scan): identical outputs."""
    X, ix = two_level(gpu, 20000, 64, 40, 500, seed=51)
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=52)
    ix.set_filter(0)
    big = [ix.rank_scores(Q), ix.node_logprob(Q, full=True), *ix.score_topk(Q, 10), *ix.categorize(Q, 10)]
    parts = [[ix.rank_scores(q), ix.node_logprob(q, full=True), *ix.score_topk(q, 10), *ix.categorize(q, 10)]
             for q in Q.split(100)]
    for i, b in enumerate(big):
        assert torch.equal(b, torch.cat([p[i] for p in parts])), i
    for j in (0, 57, 299):
        one = [ix.rank_scores(Q[j:j + 1]), ix.node_logprob(Q[j:j + 1], full=True), *ix.score_topk(Q[j:j + 1], 10),
               *ix.categorize(Q[j:j + 1], 10)]
        for i, b in enumerate(big):
            assert torch.equal(b[j:j + 1], one[i]), (j, i)
    ix.set_filter(-1)
    ix.close()


@pytest.mark.parametrize("tree", ["balanced", "two_level"])
def test_categorize_replay_wave_vs_binary_heap(gpu, tree, monkeypatch):
    """The heap replay of the best-first categorize: the wave-per-query 64-ary heap
    (default) and the thread-per-query binary heap (CWQ_SIM_BINARY=1) pop the same
    sequence -- retrieved nodes, n_found and log_prob call counts identical, with and
    without max_nodes cutting the search short, through the filter and the exact scan."""
    X = gpu.synth.synthetic_corpus(20000, 48, seed=71)
    if tree == "balanced":
        t = gpu.synth.balanced_synth(X, 5, 4, seed=72)
        ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    else:
        X, ix = two_level(gpu, 20000, 48, 300, 200, seed=73)
    Q, _ = gpu.synth.synthetic_queries(X, 200, seed=74)
    for mode in (0, 1):
        ix.set_filter(mode)
        for k, mx in ((10, 100000), (3, 50), (20, 1000)):
            wave = ix.categorize(Q, k, max_nodes=mx)
            monkeypatch.setenv("CWQ_SIM_BINARY", "1")
            binary = ix.categorize(Q, k, max_nodes=mx)
            monkeypatch.delenv("CWQ_SIM_BINARY")
            for a, b in zip(wave, binary):
                assert torch.equal(a, b), (mode, k, mx)
    ix.set_filter(-1)
    ix.close()


def _dup_rows(X, n_dup, seed):
    """Copies of random corpus rows (exact key ties between distinct rows)."""
    g = torch.Generator(device=X.device).manual_seed(seed)
    src = torch.randint(0, X.shape[0], (n_dup,), device=X.device, generator=g)
    return torch.cat([X, X[src]], 0)


@pytest.mark.parametrize("shape", [(1500, 384, "flat"), (5000, 128, "two_level"), (16000, 96, "flat"),
                                   (3000, 64, "aniso")])
def test_small_scan_vs_row_sliced_scan(gpu, shape, monkeypatch):
    """The lane-per-query scan of small isotropic segments (scan_small_kernel) against the
    row-sliced scan (CWQ_SCAN_SMALL=0): ids and scores bit for bit, k = 1 / 10 / 16 and the
    list-64 form (k = 20, which keeps the row-sliced scan), 64 ... 1000 queries."""
    N, D, kind = shape
    X = gpu.synth.synthetic_corpus(N, D, seed=61)
    if kind == "flat":
        X = _dup_rows(X, 64, seed=62)
        fs = gpu.synth.flat_synth(X)
        ix = gpu.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device="cuda:0")
    else:   # hierarchical (parent prefixes in the keys); "aniso": both leaf segments
        X, ix = two_level(gpu, N, D, 40, 200 if kind == "aniso" else 0, seed=63)
    Q, _ = gpu.synth.synthetic_queries(X, 1000, seed=64)
    for nq in (64, 100, 300, 1000):
        for k in (1, 10, 16, 20):
            got = run(ix, Q[:nq], k, 0)
            monkeypatch.setenv("CWQ_SCAN_SMALL", "0")
            ref = run(ix, Q[:nq], k, 0)
            monkeypatch.delenv("CWQ_SCAN_SMALL")
            assert torch.equal(got[0], ref[0]), (nq, k)
            assert torch.equal(got[1], ref[1]), (nq, k)
    ix.close()


# the stream pass loads K in 8-fragment chunks with the LDS query image zero-padded to
# whole chunks: dims whose fragment count is not a multiple of 8, and an LDS image at the
# 160 KiB limit (D = 1100: 35 fragments -> 40, 4 query blocks = 160 KiB; D = 1300: 41 -> 48,
# stream up to 3 query blocks, the batch filter above)
@pytest.mark.parametrize("N,D,nqs", [(20000, 300, (1, 17, 64)), (20000, 1100, (1, 64)),
                                     (20000, 1300, (33, 48, 64))])
def test_stream_chunk_padding_vs_exact(gpu, N, D, nqs):
    X = gpu.synth.synthetic_corpus(N, D, seed=41)
    fs = gpu.synth.flat_synth(X)
    ix = gpu.index.CobwebIndex(fs["mean"], fs["var"], fs["parent"], fs["node_of_sentence"], device="cuda:0")
    Q, _ = gpu.synth.synthetic_queries(X, max(nqs), seed=42)
    dpb = max(96, (D + 31) // 32 * 32)
    nkp = (dpb // 32 + 7) // 8 * 8
    for nq in nqs:
        ref = run(ix, Q[:nq], 10, 0)
        got = run(ix, Q[:nq], 10, 1)
        if ((nq + 15) // 16) * nkp * 1024 <= 160 * 1024:
            assert got[2]["path"] == "stream", (nq, got[2])
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]), (D, nq)
    ix.close()
