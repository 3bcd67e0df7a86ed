"""cwq_score_topk_host (host query in, results written into mapped host memory) == cwq_score_topk.

The reference harness times cobweb_predict_fast on a numpy embedding (benchmark_utils.py:
801-805); the drop-in's CobwebWrapper sends a host embedding through the host entry point.
Same ids and scores as the device-tensor call: flat and clustered trees, one / 8 / 64 / 300
queries (stream and batch filters), k = 1 / 10 / 64, and near-duplicate rows whose candidate
lists overflow (the exact re-run scatters into the host buffers)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg


def _same(ix, Q, k):
    ids0, s0 = ix.score_topk(Q, k)
    ids1, s1 = ix.score_topk_host(Q.cpu().numpy(), k)
    assert np.array_equal(ids0.cpu().numpy(), ids1) and np.array_equal(s0.cpu().numpy(), s1), k


@pytest.mark.parametrize("shape", ["flat", "clustered"])
def test_host_call_equals_device_call(gpu, shape):
    g = torch.Generator(device="cuda:0")
    g.manual_seed(61)
    if shape == "flat":
        X = gpu.synth.synthetic_corpus(40_000, 96, seed=61)
        X[100:140] = X[7]                                  # near-duplicate rows: list overflow -> exact re-run
        t = gpu.synth.flat_synth(X)
    else:
        C = 2.0 * torch.randn((80, 96), generator=g, device="cuda:0")
        lab = torch.randint(0, 80, (40_000,), generator=g, device="cuda:0")
        X = (C[lab] + 0.3 * torch.randn((40_000, 96), generator=g, device="cuda:0")).contiguous()
        t = gpu.synth.two_level_synth(X, lab)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    Q, _ = gpu.synth.synthetic_queries(X, 300, seed=62)
    Q[3] = X[7]
    for k in (1, 10, 64):
        for nq in (1, 8, 64, 300):
            _same(ix, Q[:nq].contiguous(), k)
    ix.close()


def test_wrapper_numpy_query_uses_host_call(gpu):
    rng = np.random.default_rng(63)
    X = rng.standard_normal((3000, 32)).astype(np.float32)
    w = gpu.CobwebWrapper(corpus=[f"s{i}" for i in range(3000)], corpus_embeddings=X)
    q = X[11] + 0.01 * rng.standard_normal(32).astype(np.float32)
    got = w.cobweb_predict_fast(q, 5, is_embedding=True)
    via_encode = w.cobweb_predict_fast(q, 5)            # the default encode_func passes it through
    via_tensor = w.cobweb_predict_fast(torch.from_numpy(q).cuda(), 5, is_embedding=True)
    assert got == via_encode
    assert got == via_tensor and got[0] == "s11", (got, via_tensor)
