"""Config C2 (BASELINE configs[1]: MS-MARCO 100k passages, 768-d, 1k queries on one
MI355X) at its shape, on a tree the drop-in builds itself -- the reference's workflow
(CobwebWrapper.py:13-80 via benchmark_utils.load_cobweb_model :438-467, then
retrieve_cobweb_basic :576-581):

  100k x 768 clustered embeddings -> CobwebWrapper(corpus, embeddings) (device ifit,
  CU scoring on libcwq) -> build_prediction_index -> 1,000 queries.

The ifit tree is a real Cobweb hierarchy (depth ~9, uneven fan-out, ~35k internal nodes),
so the query kernels run on the shape the reference produces rather than on a synthetic
flat / balanced tree.  Checks:
  * Fast, batch of 1,000: the bf16-MFMA filter's ids AND scores bit-identical to the
    exact fp32 scan; per call (nq = 1 / 8 / 64, the stream filter) the same rows;
  * Fast top-10 against the oracle (oracle/cobweb_oracle.py: its own flatten of the node
    statistics, CobwebWrapper.py:91-208, and its rank scores, :210-294) on 8 queries;
  * Basic: pop order, n_found and log_prob calls of the counting path equal the exact heap
    replay on the exact scan's keys for all 1,000 queries, and OTree.categorize
    (CobwebTorchTree.py:235-289) on 4; the drop-in cobweb_predict returns those leaves.
Real MS-MARCO embeddings need the network; the corpus is 100 Gaussian
clusters (centres N(0, 4I), spread 0.3), the queries half perturbed passages (+0.1 N(0,I)),
half fresh draws around the cluster centres."""
import os
import random

import numpy as np
import pytest

from oracle import cobweb_oracle as O
from test_gpu_configs import check_against_oracle

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

N, D, NC, NQ, K = 100_000, 768, 100, 1000, 10


def c2_corpus(seed=2):
    rng = np.random.default_rng(seed)
    C = rng.standard_normal((NC, D)).astype(np.float32) * 2.0
    X = (C[rng.integers(0, NC, N)] + 0.3 * rng.standard_normal((N, D))).astype(np.float32)
    pick = rng.choice(N, NQ // 2, replace=False)
    Qp = X[pick] + 0.1 * rng.standard_normal((NQ // 2, D))
    Qf = C[rng.integers(0, NC, NQ - NQ // 2)] + 0.3 * rng.standard_normal((NQ - NQ // 2, D))
    return X, np.concatenate([Qp, Qf]).astype(np.float32), pick


@pytest.fixture(scope="module")
def c2(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    X, Qn, pick = c2_corpus()
    random.seed(2)
    w = pkg.CobwebWrapper(corpus=[f"p{i}" for i in range(N)], corpus_embeddings=X)
    w.build_prediction_index()
    Q = torch.from_numpy(Qn).cuda()
    yield w, X, Q, Qn, pick
    w._invalidate_prediction_index()


def test_c2_tree_is_hierarchical(c2):
    w, *_ = c2
    info = w._index.info
    assert info["n_sent"] == N and info["internal_nodes"] > 10_000 and info["max_depth"] >= 5, info
    assert info["isotropic_rows"] == info["leaf_rows"]    # count-1 leaves (and exact duplicates)


def test_c2_fast_batch_and_per_call_equal_exact_scan(c2):
    w, X, Q, Qn, pick = c2
    ix = w._index
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, K)
    assert not ix.last_stats()["filter_used"]
    ix.set_filter(-1)
    ids1, s1 = ix.score_topk(Q, K)
    st = ix.last_stats()
    assert st["filter_used"] and st["path"] == "fgemm", st
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    assert np.all(np.diff(s1.cpu().numpy(), axis=1) <= 0)
    for nq in (1, 8, 64):
        for a in range(0, 192 if nq < 64 else NQ, nq):
            i2, s2 = ix.score_topk(Q[a:a + nq].contiguous(), K)
            assert torch.equal(i2, ids0[a:a + nq]) and torch.equal(s2, s0[a:a + nq]), (nq, a)
        assert ix.last_stats()["path"] == "stream"
    # the harness's call (benchmark_utils.py:576-579): numpy in, sentences out
    for qi in (0, 499, 500, 999):
        assert w.cobweb_predict_fast(Qn[qi], K) == [f"p{i}" for i in ids0[qi].tolist()]


def test_c2_fast_against_oracle(c2):
    w, X, Q, Qn, pick = c2
    nodes = w._nodes
    parent = w.tree.flatten(N)[1]
    sid_ptr = np.concatenate([[0], np.cumsum([len(n.sentence_id or []) for n in nodes])]).astype(np.int64)
    sid_list = np.array([s for n in nodes for s in (n.sentence_id or [])], np.int64)
    root = O.tree_from_arrays(parent, np.array([n.count for n in nodes], np.float32),
                              np.stack([n.mean for n in nodes]), np.stack([n.meanSq for n in nodes]), sid_ptr, sid_list)
    idx = O.flatten_tree(root, N)
    pa = O.path_arrays(idx)
    qs = [0, 1, 250, 499, 500, 501, 777, 999]
    ids, s = w._index.score_topk(Q[qs], K)
    for j, qi in enumerate(qs):
        check_against_oracle(ids[j].cpu().numpy(), s[j].cpu().numpy(), O.rank_scores_vec(Qn[qi], idx, pa))


def test_c2_basic_count_equals_replay_and_oracle(c2):
    w, X, Q, Qn, pick = c2
    ix = w._index
    got = ix.categorize(Q, K, w.max_init_search)
    st = ix.last_categorize_stats()        # how the queries resolved (reported by scripts/c2_probe.py)
    ix.set_filter(0)
    os.environ["CWQ_CAT_COUNT"] = "0"
    try:
        ref = ix.categorize(Q, K, w.max_init_search)
    finally:
        del os.environ["CWQ_CAT_COUNT"]
        ix.set_filter(-1)
    for name, a, b in zip(("nodes", "n_found", "n_calls"), ref, got):
        assert torch.equal(a, b), (name, st)
    assert bool((got[1] == K).all())          # every query retrieves k leaves (no max_nodes stop)
    # the oracle's heap search on its own node tree
    nodes = w._nodes
    parent = w.tree.flatten(N)[1]
    sid_ptr = np.concatenate([[0], np.cumsum([len(n.sentence_id or []) for n in nodes])]).astype(np.int64)
    sid_list = np.array([s for n in nodes for s in (n.sentence_id or [])], np.int64)
    tree = O.OTree(D)
    tree.root = O.tree_from_arrays(parent, np.array([n.count for n in nodes], np.float32),
                                   np.stack([n.mean for n in nodes]), np.stack([n.meanSq for n in nodes]),
                                   sid_ptr, sid_list)
    bfs = {id(n): i for i, n in enumerate(O.bfs_nodes(tree.root))}
    for qi in (0, 499, 500, 999):
        leaves, calls = tree.categorize(Qn[qi], K, order=bfs)
        assert [bfs[id(n)] for n in leaves] == got[0][qi].cpu().tolist(), qi
        assert calls == int(got[2][qi]), qi
    # the drop-in's Basic call returns the sentences of those leaves
    r = w.cobweb_predict(Qn[0], K, return_ids=True)
    assert sorted(r) == sorted(s for nid in got[0][0].tolist() for s in nodes[nid].sentence_id)
