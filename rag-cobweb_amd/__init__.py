"""rag_cobweb_amd -- MI355X-native Cobweb retrieval path (Teachable-AI-Lab/RAG-Cobweb).

Package layout (directory ``rag-cobweb_amd/``, imported as ``rag_cobweb_amd`` via
``cobweb_pkg.load()``):
  csrc/      HIP kernels for gfx950 + the C-ABI runtime -> libcwq.so
  _lib.py    ctypes binding of include/cobweb_query.h
  index.py   CobwebIndex: the device-resident flattened tree + query calls
  tree.py    host concept tree, reference JSON format, BFS flattening
  fit.py     incremental fit (ifit) with GPU category-utility scoring
  synth.py   synthetic flat / two-level trees for the 1M-10M configurations
  wrapper.py CobwebWrapper drop-in (same API as src/cobweb/CobwebWrapper.py)
  dist.py    multi-GPU: RCCL broadcast of the index + query sharding
  harness.py batched evaluate_retrieval metrics + brute-force ground truth
  whitening.py PCA + ICA whitening transform (fp32 MFMA)
"""
from . import build  # noqa: F401
from ._lib import CwqError, lib  # noqa: F401
from .tree import PRIOR_VAR, CobwebTree, Node  # noqa: F401


def __getattr__(name):
    # torch-dependent modules load lazily so that `build()` works without touching the GPU
    import importlib
    if name in ("index", "synth", "wrapper", "fit", "dist", "harness", "whitening"):
        return importlib.import_module(f".{name}", __name__)
    if name == "CobwebWrapper":
        return importlib.import_module(".wrapper", __name__).CobwebWrapper
    if name == "CobwebIndex":
        return importlib.import_module(".index", __name__).CobwebIndex
    raise AttributeError(name)
