"""C4 and C5 at their FULL per-GPU index sizes: both indexes are past 2^31 fp32 elements,
where a 32-bit element offset anywhere in the build, the exact scan, the bf16 filter or
the rerank would break.

* C4 (BASELINE configs[3]): 10,000,000 x 1024 flat-synth = 1.02e10 elements per replica
  (every rank of the 8-GPU run holds the whole tree).
* C5 (BASELINE configs[4]): 8,800,000 x 256 = 2.25e9 elements (whitened MS-MARCO shape).

On each index (reference path: CobwebWrapper.cobweb_predict_indexed,
CobwebWrapper.py:230-257):
* the automatic strategy (bf16-MFMA certified filter + exact rerank) returns ids AND
  scores bit-identical to the exact fp32 scan on 1024 queries;
* perturbed corpus points find their source row first; scores descend;
* the batch is split-invariant across the 8-rank shard bounds of the C4 run
  (dist.shard_bounds) -- bench.py --preset c4's query split;
* the CPU oracle (oracle/cobweb_oracle.py, node_logprob_prime + the path weights) over
  ALL rows, from chunked host copies of the index's own mean rows, for sampled queries:
  top-10 identical up to reference-indistinguishable swaps, scores within 1e-5.
The variances go in compact form (cwq_index_create_cv): one scalar per leaf, the
root's row in full -- the [Nn, D] variance array alone would be 41 GB at C4."""
import concurrent.futures as cf
import gc

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


def _oracle_topk(mean_dev, root_var, Qn, k, chunk=131072, workers=16):
    """Oracle scores of every leaf for each query in Qn, from host copies of the mean rows
    in chunks (flat tree: score = c*lp'(root) + c*lp'(leaf), c = level weight / path
    length = 1/2, CobwebWrapper.py:160-168, 240-241).  Returns per query the top-(k+16)
    (ids, scores) and a function giving the oracle score of any leaf ids."""
    N = mean_dev.shape[0] - 1
    D = mean_dev.shape[1]
    c = O.path_weight(0, 2, O.DEFAULT_LEVEL_WEIGHTS)
    root_mu = mean_dev[0].cpu().numpy()
    lp_root = [O.node_logprob_prime(x, root_mu[None, :], root_var[None, :])[0] for x in Qn]
    pv = np.full((chunk, D), O.PRIOR_VAR, np.float32)    # every leaf's var row (count 1)
    keep = k + 16

    def one(c0):
        c1 = min(N, c0 + chunk)
        rows = mean_dev[1 + c0:1 + c1].cpu().numpy()
        out = []
        for qi, x in enumerate(Qn):
            s = (c * lp_root[qi] + c * O.node_logprob_prime(x, rows, pv[:c1 - c0])).astype(np.float32)
            part = np.argpartition(-s, keep - 1)[:keep]
            out.append((part + c0, s[part]))
        return out

    with cf.ThreadPoolExecutor(workers) as ex:
        res = list(ex.map(one, range(0, N, chunk)))
    tops = []
    for qi in range(len(Qn)):
        ids = np.concatenate([r[qi][0] for r in res])
        sc = np.concatenate([r[qi][1] for r in res])
        o = np.lexsort((ids, -sc.astype(np.float64)))[:keep]
        tops.append((ids[o], sc[o]))

    def score_of(qi, leaf_ids):
        rows = mean_dev[1 + torch.as_tensor(leaf_ids, device=mean_dev.device)].cpu().numpy()
        return (c * lp_root[qi] + c * O.node_logprob_prime(Qn[qi], rows, pv[:len(leaf_ids)])).astype(np.float32)

    return tops, score_of


def _full_size_case(pkg, N, D, NQ, seed, qseed, oracle_q, k=10):
    gc.collect()
    torch.cuda.empty_cache()
    free, total = torch.cuda.mem_get_info()
    need = N * D * 4 * 3.8 + (8 << 30)        # caller's mean + ~2.6x the means in the index + workspace
    if free < need:
        pytest.skip(f"needs ~{need / 2**30:.0f} GiB of device memory, {free / 2**30:.0f} GiB free")
    X = pkg.synth.synthetic_corpus(N, D, seed=seed)
    t = pkg.synth.flat_synth(X, compact=True)
    del X
    mean = t["mean"]
    root_var = t["var"][0].cpu().numpy()
    ix = pkg.index.CobwebIndex(mean, t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    assert ix.info["isotropic_rows"] == N and N * D > 2 ** 31
    Q, targets = pkg.synth.synthetic_queries(mean[1:], NQ, seed=qseed)
    # exact fp32 scan vs the automatic strategy (the batch bf16-MFMA filter)
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, k)
    assert not ix.last_stats()["filter_used"]
    ix.set_filter(-1)
    ids1, s1 = ix.score_topk(Q, k)
    st = ix.last_stats()
    assert st["path"] == "fgemm" and st["filter_queries"] == NQ and st["fallback_queries"] == 0, st
    assert torch.equal(ids0, ids1) and torch.equal(s0, s1)
    ids, s = ids1.cpu().numpy(), s1.cpu().numpy()
    tg = targets.cpu().numpy()
    assert np.all(ids[:len(tg), 0] == tg)                       # perturbed corpus rows find their source first
    assert np.all(np.diff(s, axis=1) <= 0)
    assert ids.min() >= 0 and ids.max() < N
    # the 8-rank shard split of the C4 run (and the per-call stream path on the shard heads)
    for r in range(8):
        lo, hi = pkg.dist.shard_bounds(NQ, r, 8)
        i2, s2 = ix.score_topk(Q[lo:hi], k)
        assert torch.equal(i2, ids1[lo:hi]) and torch.equal(s2, s1[lo:hi])
        i3, s3 = ix.score_topk(Q[lo:lo + 1], k)
        assert ix.last_stats()["path"] == "stream"
        assert torch.equal(i3, ids1[lo:lo + 1]) and torch.equal(s3, s1[lo:lo + 1])
    # the oracle over every row (host copies of the index's mean rows, in chunks)
    Qn = Q[oracle_q].cpu().numpy()
    tops, score_of = _oracle_topk(mean, root_var, Qn, k)
    for j, qi in enumerate(oracle_q):
        ref_ids, ref_sc = tops[j]
        lookup = dict(zip(ref_ids.tolist(), ref_sc.tolist()))
        for a in ids[qi]:
            if a not in lookup:
                lookup[int(a)] = float(score_of(j, [int(a)])[0])
        topk_equiv(ids[qi], ref_ids[:k], lookup)
        assert rel_err(s[qi], score_of(j, ids[qi])) < RTOL
    ix.close()
    del t, mean, Q
    gc.collect()
    torch.cuda.empty_cache()


def test_c4_full_per_gpu_index_10m_x_1024(gpu):
    # C4: 10M x 1024 = 1.02e10 fp32 elements per replica; 12,500 queries = the bench's
    # per-rank batch of the 8-GPU C4 run (100k queries split over 8 ranks)
    _full_size_case(gpu, 10_000_000, 1024, 12_500, seed=0, qseed=1, oracle_q=[0, 700, 12_499])


def test_c5_full_index_8_8m_x_256(gpu):
    # C5: 8.8M x 256 = 2.25e9 fp32 elements (whitened MS-MARCO shape, N(0, I) stand-in)
    _full_size_case(gpu, 8_800_000, 256, 1024, seed=5, qseed=6, oracle_q=[3, 511, 900])


@pytest.mark.parametrize("name", ["g4_twolevel_d48", "g1_hier_d32"])
def test_compact_var_index_identical(gpu, name):
    """cwq_index_create_cv (compact variances) builds the same index as cwq_index_create:
    every query output bit-identical, on goldens with internal nodes and an anisotropic leaf."""
    from conftest import load_golden
    from test_gpu_parity import index_from_golden
    g = load_golden(name)
    full = index_from_golden(gpu, g)
    var = O.compute_var(g["meanSq"], g["count"][:, None])
    var[g["count"] == 0] = O.PRIOR_VAR
    cv = gpu.index.CompactVar.from_full(torch.from_numpy(np.ascontiguousarray(var)))
    assert cv.an_var.shape[0] < var.shape[0]
    assert torch.equal(cv.full(), torch.from_numpy(np.ascontiguousarray(var)))
    nos = np.full(int(g["n_sent"]), -1, np.int64)
    for i in range(len(g["parent"])):
        for s in g["sid_list"][g["sid_ptr"][i]:g["sid_ptr"][i + 1]]:
            nos[s] = i
    comp = gpu.index.CobwebIndex(g["mean"], cv, g["parent"], nos, device="cuda:0")
    assert comp.info == full.info
    Q = torch.from_numpy(g["Xq"]).cuda()
    for mode in (0, 1, -1):
        full.set_filter(mode)
        comp.set_filter(mode)
        for k in (1, 10):
            a, b = full.score_topk(Q, k), comp.score_topk(Q, k)
            assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert torch.equal(full.rank_scores(Q), comp.rank_scores(Q))
    assert torch.equal(full.node_logprob(Q, full=True), comp.node_logprob(Q, full=True))
    a, b = full.categorize(Q, 3), comp.categorize(Q, 3)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    full.close()
    comp.close()
