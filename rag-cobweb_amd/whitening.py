"""PCA + ICA whitening (F4), drop-in for src/whitening/pca_ica.py:PCAICAWhiteningModel.

Same constructor, attributes, `transform(x, is_ica=True)` semantics (single vector ->
1-D result, batch -> 2-D; numpy in -> numpy out) and `fit(X, pca_dim, eps,
ica_max_iter, ica_tol)` classmethod.  `transform` runs on the GPU through libcwq
`cwq_whiten` (fp32 MFMA GEMMs with the centring and the PCA scaling fused); torch
supplies the device buffers.  `fit` is offline training and, like the reference
(:55-76), delegates to scikit-learn's PCA and FastICA on the host.  `save`/`load` use a
pickle-free .npz (the reference pickles, :78-99).
"""
import ctypes

import numpy as np
import torch

from ._lib import check, lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class PCAICAWhiteningModel:
    def __init__(self, mean, pca_components, ica_unmixing, pca_explained_var, eps=1e-8, device=None):
        self.mean = np.asarray(mean, np.float32)
        self.pca_components = np.asarray(pca_components, np.float32)
        self.pca_explained_var = np.asarray(pca_explained_var, np.float32)
        self.ica_unmixing = None if ica_unmixing is None else np.asarray(ica_unmixing, np.float32)
        self.eps = eps
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._dev = None

    def __repr__(self):
        return (f"{self.__class__.__name__}(\n  mean.shape={self.mean.shape},\n"
                f"  pca_components.shape={self.pca_components.shape},\n"
                f"  pca_explained_var.shape={self.pca_explained_var.shape},\n"
                f"  ica_unmixing.shape={None if self.ica_unmixing is None else self.ica_unmixing.shape},\n"
                f"  eps={self.eps}\n)")

    def _device_params(self):
        if self._dev is None:
            # the divisor exactly as the reference computes it (fp32 add, fp32 sqrt), pca_ica.py:44
            denom = np.sqrt(self.pca_explained_var + np.float32(self.eps)).astype(np.float32)
            to = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
            self._dev = (to(self.mean), to(self.pca_components), to(denom), to(self.ica_unmixing))
        return self._dev

    def transform(self, x, is_ica=True, batch=1 << 20):
        """PCAICAWhiteningModel.transform (pca_ica.py:30-51) on the GPU."""
        as_numpy = not isinstance(x, torch.Tensor)
        xt = torch.as_tensor(np.asarray(x, np.float32) if as_numpy else x, dtype=torch.float32)
        single = xt.dim() == 1
        if single:
            xt = xt[None, :]
        xt = xt.to(self.device).contiguous()
        n, d_in = xt.shape
        mean, comps, denom, unmix = self._device_params()
        if d_in != comps.shape[1]:
            raise ValueError(f"expected inputs of dimension {comps.shape[1]}, got {d_in}")
        d_pca = comps.shape[0]
        use_ica = is_ica and unmix is not None
        d_out = unmix.shape[0] if use_ica else d_pca
        out = torch.empty((n, d_out), dtype=torch.float32, device=self.device)
        work = torch.empty((min(n, batch), d_pca), dtype=torch.float32, device=self.device) if use_ica else None
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        with torch.cuda.device(self.device):
            for i in range(0, n, batch):
                j = min(n, i + batch)
                check(lib().cwq_whiten(ctypes.c_void_p(xt[i:j].data_ptr()), j - i, d_in, _ptr(mean), _ptr(comps),
                                       d_pca, _ptr(denom), _ptr(unmix) if use_ica else None, d_out,
                                       ctypes.c_void_p(out[i:j].data_ptr()), _ptr(work), stream))
        if single:
            out = out[0]
        return out.cpu().numpy() if as_numpy else out

    @classmethod
    def fit(cls, X, pca_dim=256, eps=1e-8, ica_max_iter=5000, ica_tol=1e-3, device=None):
        """pca_ica.py:55-76: PCA -> normalise -> FastICA (host, scikit-learn)."""
        from sklearn.decomposition import PCA, FastICA
        X = np.asarray(X, np.float32)
        mean = X.mean(axis=0)
        X_centered = X - mean
        pca = PCA(n_components=pca_dim)
        X_pca = pca.fit_transform(X_centered)
        components = pca.components_
        explained_var = pca.explained_variance_
        X_pca_normalized = X_pca / np.sqrt(explained_var + eps)
        ica = FastICA(n_components=components.shape[0], whiten="unit-variance", max_iter=ica_max_iter, tol=ica_tol)
        ica.fit_transform(X_pca_normalized)
        return cls(mean, components, ica.components_, explained_var, eps, device=device)

    def save(self, filepath):
        with open(filepath, "wb") as f:
            np.savez(f, mean=self.mean, pca_components=self.pca_components, pca_explained_var=self.pca_explained_var,
                     ica_unmixing=self.ica_unmixing if self.ica_unmixing is not None else np.zeros((0, 0), np.float32),
                     eps=np.asarray([self.eps], np.float64))

    @classmethod
    def load(cls, filepath, device=None):
        with np.load(filepath, allow_pickle=False) as z:
            unmix = z["ica_unmixing"]
            return cls(z["mean"], z["pca_components"], None if unmix.size == 0 else unmix, z["pca_explained_var"],
                       float(z["eps"][0]), device=device)


def encode_and_whiten_pcaica(sentences, st_model, whitening_model):
    """pca_ica.py:103-122: encode (if given strings) then whiten."""
    if isinstance(sentences[0], str):
        embeddings = st_model.encode(sentences, convert_to_numpy=True, batch_size=64, show_progress_bar=False)
    else:
        embeddings = sentences
    return whitening_model.transform(embeddings)
