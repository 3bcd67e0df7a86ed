"""Generate the F3 harness fixture (tests/golden/g7_harness.npz) by running the REAL
reference metric code (Teachable-AI-Lab/RAG-Cobweb @ 2025-09-26, read-only at
/root/reference): `evaluate_retrieval` (src/utils/benchmark_utils.py:710-833, with its
get_eval_ks :619-622 and sklearn ndcg_score) on canned retrieval lists, and
`retrieve_torch_dot` (:602-614, the reference's "Torch Dot" / FAISS-flat-IP
equivalent) on a small corpus.

Run:  python tests/golden/gen_harness.py

Only data leaves this script (inputs and the reference's outputs).  No reference source
or bytecode is copied (bytecode writing is off).  The GPU box never runs it.

Import shim: benchmark_utils imports faiss / annoy / hnswlib / sentence_transformers at
module level (used only by the FAISS / Annoy / HNSW baselines and by the encoders,
none of which this script calls) and graphviz (visualisation, CobwebWrapper.py:9);
none is installed here, so empty in-memory stand-ins take their names.  The functions
called below use numpy, torch, time and sklearn only.
"""
import os
import sys
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

import numpy as np  # noqa: E402
import torch  # noqa: E402
# the real transformers names benchmark_utils imports, resolved before the stand-ins
# below exist (transformers probes optional packages by module spec)
from transformers import (AutoModel, AutoTokenizer, DPRContextEncoder, DPRContextEncoderTokenizer,  # noqa: E402,F401
                          DPRQuestionEncoder, DPRQuestionEncoderTokenizer, T5EncoderModel)

class _Absent(types.ModuleType):
    """Stand-in for a missing module: every attribute (only ever used in type
    annotations and in functions this script does not call) is `object`."""

    def __getattr__(self, attr):
        return object


for name in ("graphviz", "faiss", "annoy", "hnswlib", "sentence_transformers"):
    sys.modules[name] = _Absent(name)
sys.path.insert(0, REF)
from src.utils import benchmark_utils as BU  # noqa: E402


def canned_lists(rng, n_queries, n_docs, list_len):
    """Retrieval lists of doc ids with the situations the metric loop has to handle:
    target at any rank or absent, lists shorter than top_k (Cobweb Basic can return
    fewer), and duplicate TEXTS (two ids with one string: the reference matches by
    string, so both count as relevant)."""
    ids = np.full((n_queries, list_len), -1, np.int64)
    lengths = np.zeros(n_queries, np.int64)
    targets = rng.integers(0, n_docs, n_queries)
    for q in range(n_queries):
        L = list_len if q % 5 else int(rng.integers(0, list_len + 1))
        row = rng.choice(n_docs, size=L, replace=False)
        mode = q % 4
        if mode in (0, 1) and L > 0:                   # target somewhere in the list
            row[int(rng.integers(0, L))] = targets[q]
        elif mode == 2 and L > 0:                      # target at rank 1
            row[0] = targets[q]
        ids[q, :L] = row
        lengths[q] = L
    return ids, lengths, targets


def main():
    rng = np.random.default_rng(2025)
    n_docs = 300
    # doc id -> text; ids 2j and 2j+1 share one text for j < 20 (duplicate sentences)
    text_of = np.array([(i // 2 if i < 40 else i) for i in range(n_docs)], np.int64)
    texts = [f"doc-{t}" for t in text_of]
    out = {"text_of": text_of}
    for top_k, nq, list_len in [(10, 400, 12), (50, 300, 60), (5, 100, 5)]:
        ids, lengths, targets = canned_lists(rng, nq, n_docs, list_len)
        lists = [[texts[j] for j in ids[q, :lengths[q]]] for q in range(nq)]
        tstr = [texts[t] for t in targets]

        def retrieve(query, k, _lists=lists):
            return _lists[query]

        m = BU.evaluate_retrieval(f"canned@{top_k}", list(range(nq)), tstr, retrieve, top_k=top_k)
        keys = [k for k in m if k.split("@")[0] in ("recall", "mrr", "ndcg")]
        out[f"k{top_k}_ids"] = ids
        out[f"k{top_k}_lengths"] = lengths
        out[f"k{top_k}_targets"] = targets
        out[f"k{top_k}_metric_names"] = np.array(keys)
        out[f"k{top_k}_metric_values"] = np.array([m[k] for k in keys], np.float64)
    # Torch Dot ground truth (the reference's exact flat inner-product search)
    X = rng.standard_normal((5000, 64)).astype(np.float32)
    Q = rng.standard_normal((64, 64)).astype(np.float32)
    corpus = [f"row-{i}" for i in range(X.shape[0])]
    Xt = torch.from_numpy(X)
    gt = np.array([[int(s[4:]) for s in BU.retrieve_torch_dot(q, 10, Xt, corpus)] for q in Q], np.int64)
    out.update(dot_X=X, dot_Q=Q, dot_ids=gt)
    np.savez_compressed(os.path.join(OUT, "g7_harness.npz"), **out)
    print("wrote g7_harness.npz", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
