"""F3 (harness counterpart) against the REAL reference metric loop: tests/golden/
g7_harness.npz holds canned retrieval lists and what the reference's
`evaluate_retrieval` (src/utils/benchmark_utils.py:710-833) and `retrieve_torch_dot`
(:602-614) returned for them (tests/golden/gen_harness.py).  The lists cover targets
at every rank, absent targets, short and empty lists, duplicate texts and the
reference's single-entry abort (ndcg_score raising inside its try block).

CPU: rag_cobweb_amd.harness on CPU tensors.  GPU (-m gpu): the same metrics computed
on the device, and the GPU brute-force flat-IP / flat-L2 ground truth."""
import numpy as np
import pytest

from conftest import load_golden

torch = pytest.importorskip("torch")
TOPKS = [10, 50, 5]


def expected(g, top_k):
    names = [str(n) for n in g[f"k{top_k}_metric_names"]]
    return dict(zip(names, (float(v) for v in g[f"k{top_k}_metric_values"])))


def keyed(g, top_k, device):
    ids = torch.as_tensor(g[f"k{top_k}_ids"], device=device)
    text_of = torch.as_tensor(g["text_of"], device=device)
    keys = torch.where(ids >= 0, text_of[ids.clamp(min=0)], ids)      # match by text, like the reference
    tgt = text_of[torch.as_tensor(g[f"k{top_k}_targets"], device=device)]
    return keys, tgt, torch.as_tensor(g[f"k{top_k}_lengths"], device=device)


@pytest.mark.parametrize("top_k", TOPKS)
def test_metrics_match_reference_cpu(pkg, top_k):
    g = load_golden("g7_harness")
    keys, tgt, lengths = keyed(g, top_k, "cpu")
    got = pkg.harness.retrieval_metrics(keys, tgt, top_k, lengths)
    assert got == expected(g, top_k)


def test_single_entry_abort_is_exercised():
    g = load_golden("g7_harness")
    n = 0
    for top_k in TOPKS:
        ids, L, t = g[f"k{top_k}_ids"], g[f"k{top_k}_lengths"], g[f"k{top_k}_targets"]
        n += int(np.sum((L == 1) & (g["text_of"][ids[:, 0]] == g["text_of"][t])))
    assert n > 0


@pytest.mark.gpu
@pytest.mark.parametrize("top_k", TOPKS)
def test_metrics_match_reference_gpu(pkg, top_k):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = load_golden("g7_harness")
    keys, tgt, lengths = keyed(g, top_k, "cuda:0")
    got = pkg.harness.retrieval_metrics(keys, tgt, top_k, lengths)
    assert got == expected(g, top_k)
    # the batched evaluate_retrieval wrapper over the same lists (ids -> text keys)
    ids = torch.as_tensor(g[f"k{top_k}_ids"], device="cuda:0")
    rows = {"i": 0}

    def retrieve_batch(qb, k):
        out = ids[rows["i"]:rows["i"] + len(qb), :]
        rows["i"] += len(qb)
        return out

    tg = torch.as_tensor(g["text_of"], device="cuda:0")[torch.as_tensor(g[f"k{top_k}_targets"], device="cuda:0")]
    m = pkg.harness.evaluate_retrieval_batch("canned", list(range(ids.shape[0])), tg, retrieve_batch, top_k=top_k,
                                             batch_size=64, key_of_id=g["text_of"])
    for name, v in expected(g, top_k).items():
        assert m[name] == v, name


@pytest.mark.gpu
def test_brute_force_ground_truth_gpu(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = load_golden("g7_harness")
    X = torch.from_numpy(g["dot_X"]).cuda()
    Q = torch.from_numpy(g["dot_Q"]).cuda()
    for exact in (False, True):
        got = pkg.harness.brute_force_topk(X, Q, 10, "ip", exact=exact).cpu().numpy()
        np.testing.assert_array_equal(got, g["dot_ids"])         # the reference's Torch Dot top-10
    # flat-L2 (the reference's FAISS IndexFlatL2 setting, benchmark_utils.py:541-542) vs float64 numpy
    d = ((g["dot_Q"].astype(np.float64)[:, None, :] - g["dot_X"].astype(np.float64)[None, :, :]) ** 2).sum(-1)
    want = np.argsort(d, axis=1, kind="stable")[:, :10]
    got = pkg.harness.brute_force_topk(X, Q, 10, "l2", exact=True).cpu().numpy()
    np.testing.assert_array_equal(got, want)
