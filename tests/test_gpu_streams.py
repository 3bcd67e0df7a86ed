"""One index handle used from two torch streams back to back: every query entry point
carves the handle's single workspace, so the second call must wait for the first call's
kernels (cwq_index::ws_begin / ws_end).  Results must equal the serial ones."""
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(pkg):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return pkg


def test_two_streams_equal_serial(gpu):
    X = gpu.synth.synthetic_corpus(60_000, 256, seed=21)
    lab = torch.randint(0, 64, (60_000,), device="cuda:0", generator=torch.Generator(device="cuda:0").manual_seed(3))
    t = gpu.synth.two_level_synth(X, lab)
    ix = gpu.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], device="cuda:0")
    Q1, _ = gpu.synth.synthetic_queries(X, 4096, seed=22)   # a long first call (exact scan below)
    Q2, _ = gpu.synth.synthetic_queries(X, 300, seed=23)
    ix.set_filter(0)
    ref1 = ix.score_topk(Q1, 10)
    ref2 = ix.score_topk(Q2, 10)
    refr = ix.rank_scores(Q2[:8])
    refc = ix.categorize(Q2[:16], 10)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        s1.wait_stream(torch.cuda.current_stream())
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s1):
            a = ix.score_topk(Q1, 10)
        with torch.cuda.stream(s2):
            b = ix.score_topk(Q2, 10)
            r = ix.rank_scores(Q2[:8])
        with torch.cuda.stream(s1):
            c = ix.categorize(Q2[:16], 10)
        torch.cuda.synchronize()
        assert torch.equal(a[0], ref1[0]) and torch.equal(a[1], ref1[1])
        assert torch.equal(b[0], ref2[0]) and torch.equal(b[1], ref2[1])
        assert torch.equal(r, refr)
        assert all(torch.equal(x, y) for x, y in zip(c, refc))
    ix.set_filter(-1)
    ix.close()
