"""Golden vectors for the PCA + ICA whitening transform (F4), made by running the REAL
reference's PCAICAWhiteningModel (src/whitening/pca_ica.py, /root/reference, read-only)
in the build container: its own fit (scikit-learn PCA + FastICA) and its own transform.

Run:  python tests/golden/gen_whiten.py        (seconds)

Only data leaves this script (tests/golden/g6_pcaica.npz): the inputs, the fitted
model parameters and the reference's outputs.  Bytecode writing is disabled; the GPU
box never runs this script.
"""
import os
import sys
import warnings

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
sys.path.insert(0, "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))

import numpy as np  # noqa: E402

from src.whitening.pca_ica import PCAICAWhiteningModel   # noqa: E402


def main():
    warnings.filterwarnings("ignore")
    rng = np.random.default_rng(7)
    N, D, P = 3000, 96, 32
    # anisotropic, offset, correlated embeddings (whitening has something to undo)
    Z = rng.standard_normal((N, D)).astype(np.float32)
    A = (rng.standard_normal((D, D)) / np.sqrt(D)).astype(np.float32)
    X = (Z @ A * np.linspace(0.2, 3.0, D, dtype=np.float32) + 0.5).astype(np.float32)
    Q = (X[:200] + 0.05 * rng.standard_normal((200, D)).astype(np.float32)).astype(np.float32)
    np.random.seed(0)   # FastICA's default random_state draws from numpy's global RNG
    m = PCAICAWhiteningModel.fit(X, pca_dim=P, ica_max_iter=2000)
    out = dict(X=X, Q=Q, mean=m.mean, pca_components=m.pca_components, ica_unmixing=m.ica_unmixing,
               pca_explained_var=m.pca_explained_var, eps=np.asarray([m.eps], np.float64),
               X_ica=m.transform(X), X_pca=m.transform(X, is_ica=False), Q_ica=m.transform(Q),
               q0_ica=m.transform(Q[0]))
    for k, v in out.items():
        print(k, np.asarray(v).dtype, np.asarray(v).shape)
    np.savez_compressed(os.path.join(OUT, "g6_pcaica.npz"), **out)


if __name__ == "__main__":
    main()
