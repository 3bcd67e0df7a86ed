"""F4: PCA + ICA whitening.  CPU: the oracle restatement against the reference's own
outputs (tests/golden/g6_pcaica.npz, made by tests/golden/gen_whiten.py), and the
pickle-free save/load.  GPU: libcwq cwq_whiten against the same fixture and against
the oracle at the C5 shape (768 -> 256)."""
import os

import numpy as np
import pytest

from conftest import load_golden
from oracle import cobweb_oracle as O

TOL = 1e-5   # relative to the row's max |value|: fp32 summation order only


def row_rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.ndim == 1:
        a, b = a[None], b[None]
    return float(np.max(np.abs(a - b).max(1) / np.maximum(np.abs(b).max(1), 1e-30)))


def params(g):
    return g["mean"], g["pca_components"], g["pca_explained_var"], g["ica_unmixing"], float(g["eps"][0])


def test_oracle_matches_reference_outputs():
    g = load_golden("g6_pcaica")
    m, c, v, u, eps = params(g)
    assert row_rel(O.whiten_transform(g["X"], m, c, v, u, eps), g["X_ica"]) < TOL
    assert row_rel(O.whiten_transform(g["X"], m, c, v, u, eps, is_ica=False), g["X_pca"]) < TOL
    assert row_rel(O.whiten_transform(g["Q"], m, c, v, u, eps), g["Q_ica"]) < TOL
    q0 = O.whiten_transform(g["Q"][0], m, c, v, u, eps)
    assert q0.shape == g["q0_ica"].shape and row_rel(q0, g["q0_ica"]) < TOL
    # whitened: unit variance, decorrelated on the fitting data
    cov = np.cov(g["X_pca"].astype(np.float64).T)
    assert np.allclose(np.diag(cov), 1.0, atol=1e-3)


def test_save_load_round_trip(pkg, tmp_path):
    W = pkg.whitening.PCAICAWhiteningModel
    g = load_golden("g6_pcaica")
    m, c, v, u, eps = params(g)
    w = W(m, c, u, v, eps, device="cpu")
    p = os.path.join(tmp_path, "w.npz")
    w.save(p)
    w2 = W.load(p, device="cpu")
    for a in ("mean", "pca_components", "pca_explained_var", "ica_unmixing"):
        assert np.array_equal(getattr(w, a), getattr(w2, a))
    assert w2.eps == eps


@pytest.mark.gpu
def test_gpu_whiten_matches_reference(pkg):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = load_golden("g6_pcaica")
    m, c, v, u, eps = params(g)
    w = pkg.whitening.PCAICAWhiteningModel(m, c, u, v, eps, device="cuda:0")
    assert row_rel(w.transform(g["X"]), g["X_ica"]) < TOL
    assert row_rel(w.transform(g["X"], is_ica=False), g["X_pca"]) < TOL
    assert row_rel(w.transform(g["Q"]), g["Q_ica"]) < TOL
    q0 = w.transform(g["Q"][0])
    assert q0.shape == (32,) and row_rel(q0, g["q0_ica"]) < TOL
    xt = torch.from_numpy(g["Q"]).cuda()
    out = w.transform(xt)
    assert isinstance(out, torch.Tensor) and out.is_cuda
    assert row_rel(out.cpu().numpy(), g["Q_ica"]) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,p", [(20000, 768, 256), (1000, 384, 100), (777, 100, 37), (5, 1024, 256)])
def test_gpu_whiten_shapes(pkg, n, d, p):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(n + d)
    X = (rng.standard_normal((n, d)) * rng.uniform(0.1, 3, d) + 1.0).astype(np.float32)
    mean = X.mean(0)
    comps = np.linalg.qr(rng.standard_normal((d, p)))[0].T.astype(np.float32)
    var = rng.uniform(0.5, 4.0, p).astype(np.float32)
    unmix = np.linalg.qr(rng.standard_normal((p, p)))[0].astype(np.float32)
    w = pkg.whitening.PCAICAWhiteningModel(mean, comps, unmix, var, 1e-8, device="cuda:0")
    ref = O.whiten_transform(X, mean, comps, var, unmix, 1e-8)
    assert row_rel(w.transform(X), ref) < TOL
    assert row_rel(w.transform(X, is_ica=False), O.whiten_transform(X, mean, comps, var, unmix, 1e-8, False)) < TOL
