"""Drop-in `CobwebWrapper` for src/cobweb/CobwebWrapper.py, backed by libcwq on MI355X.

Same constructor, method names, argument meanings, return types and error
behaviour as the reference class (file:line per method), so harness code such as
src/utils/benchmark_utils.py:576-581 (`retrieve_cobweb_basic`) runs unchanged:

    cobweb.cobweb_predict_fast(query_emb, k)   -> list of sentences   (A6)
    cobweb.cobweb_predict(query_emb, k)        -> list of sentences   (A4/A5)

Differences (documented in DESIGN.md §6):
  * scoring runs on the GPU through libcwq; there is no CPU path;
  * exact score ties are broken deterministically (lower node / sentence id)
    instead of by randn*1e-6 noise (CobwebWrapper.py:246-256) or the heap's random()
    key (CobwebTorchTree.py:243,285); the global random() stream is still advanced by
    the draws the reference makes and the retrieved leaves' lists are shuffled with it
    (CobwebWrapper.py:456), so add -> Basic query -> add builds the reference's tree;
  * `cobweb_rank_scores` returns a tensor without autograd history (training
    through the scores, src/training/cobweb_query_train.py, is out of scope);
  * batched entry points `cobweb_predict_batch` / `cobweb_categorize_batch` take a
    [Q, D] query block and return id tensors.
"""
import json
import math
import os
import random

import numpy as np
import torch

from .index import CobwebIndex
from .tree import CobwebTree

MAX_INIT_SEARCH = 100000   # CobwebWrapper.py:24


_NATIVE_SKIP_MIN = 4096   # below this many draws getrandbits is cheaper than a state round trip


def advance_random(n, rng=random):
    """Advance `rng` (the global `random` module by default) past `n` random() draws:
    random() takes two 32-bit MT19937 outputs (CobwebTorchTree.py:243,268,285).  Small n:
    getrandbits(64*n), which takes exactly 2*n; large n (a flat 1M tree: ~1M draws per
    Basic query, 4.5 ms through an 8 MB integer): the state is twisted forward natively
    (libcwq cwq_mt19937_skip) and set back -- the same state bit for bit."""
    if n <= 0:
        return
    if n < _NATIVE_SKIP_MIN:
        rng.getrandbits(64 * n)
        return
    from . import _lib
    ver, words, gauss = rng.getstate()
    st = np.array(words, dtype=np.uint32)
    _lib.check(_lib.lib().cwq_mt19937_skip(st.ctypes.data, 2 * int(n)))
    rng.setstate((ver, tuple(st.tolist()), gauss))


class CobwebWrapper:
    def __init__(self, corpus=None, corpus_embeddings=None, encode_func=lambda x: x, device=None):
        """CobwebWrapper.py:13-50."""
        self.encode_func = encode_func
        self.sentences = []
        self.sentence_to_node = {}
        if device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("rag_cobweb_amd.CobwebWrapper needs a ROCm GPU (libcwq has no CPU path)")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.max_init_search = MAX_INIT_SEARCH
        self._prediction_index_valid = False
        self._index = None
        self._nodes = None
        self._node_to_index = {}
        self._leaf_to_path_indices = None
        self._level_weights = None
        self._weight_schedule = None
        self._schedule_params = {}
        self.max_depth = 0

        embedding_shape = None
        if corpus_embeddings is not None:
            corpus_embeddings = np.asarray(corpus_embeddings, dtype=np.float32) if isinstance(
                corpus_embeddings, list) else corpus_embeddings
            embedding_shape = tuple(corpus_embeddings.shape[1:])
        elif corpus and len(corpus) > 0:
            embedding_shape = tuple(np.asarray(self.encode_func([corpus[0]])).shape[1:])
        self.tree = CobwebTree(embedding_shape) if embedding_shape is not None else None

        if corpus_embeddings is not None:
            if corpus is None:
                corpus = [None] * len(corpus_embeddings)
            self.add_sentences(corpus, corpus_embeddings)
        elif corpus is not None and len(corpus) > 0:
            self.add_sentences(corpus)

    # ------------------------------------------------------------------ add path
    def add_sentences(self, new_sentences, new_vectors=None):
        """CobwebWrapper.py:52-80: incremental fit of each embedding, then the
        prediction index is invalidated."""
        if new_vectors is None:
            new_embeddings = np.asarray(self.encode_func(new_sentences), dtype=np.float32)
        else:
            new_embeddings = new_vectors
            if isinstance(new_embeddings, list):
                new_embeddings = np.asarray(new_embeddings, dtype=np.float32)
            if self.tree is not None and new_embeddings.shape[1] != self.tree.shape[0]:
                print(f"[Warning] Provided vector dim {new_embeddings.shape[1]} != tree dim "
                      f"{self.tree.shape[0]}, re-encoding...")
                new_embeddings = np.asarray(self.encode_func(new_sentences), dtype=np.float32)
        from .fit import _MAX_DEVICE_DIM, DeviceTreeFitter, TreeFitter
        X = np.asarray(new_embeddings.detach().cpu().numpy() if torch.is_tensor(new_embeddings)
                       else new_embeddings, dtype=np.float32)
        if self.tree is None:
            self.tree = CobwebTree(X.shape[1:])
        start = len(self.sentences)
        n = len(new_sentences)
        # the device-resident insert loop (one kernel for the whole batch) unless disabled
        # (CWQ_FIT_DEVICE=0) or the dimension is past its LDS budget: then the host-driven
        # fitter (per level one KL launch) -- both build the same tree
        use_dev = os.environ.get("CWQ_FIT_DEVICE", "1") != "0" and self.tree.dim <= _MAX_DEVICE_DIM
        if use_dev:
            fitter = DeviceTreeFitter(self.tree, device=self.device)
            leaves = fitter.fit_batch(X[:n])
            self.last_fit_stats = dict(fitter.stats)   # rows, kernel seconds, draws, ... (diagnostics)
        else:
            fitter = TreeFitter(self.tree, device=self.device)
            leaves = [fitter.ifit(X[i]) for i in range(n)]
            fitter.sync_to_host()
        for i, sent in enumerate(new_sentences):
            self.sentences.append(sent)
            leaf = leaves[i]
            if leaf.sentence_id is None:
                leaf.sentence_id = []
            leaf.sentence_id.append(start + i)
            self.sentence_to_node[start + i] = leaf
        self._invalidate_prediction_index()

    # --------------------------------------------------------------- index build
    def _invalidate_prediction_index(self):
        """CobwebWrapper.py:82-89."""
        self._prediction_index_valid = False
        if self._index is not None:
            self._index.close()
        self._index = None
        self._nodes = None
        self._node_to_index = {}
        self._leaf_to_path_indices = None

    def build_prediction_index(self):
        """CobwebWrapper.py:91-208: BFS flatten (O(Nn), not the reference's O(Nn^2)),
        then the device index (dim-major stats, path structure, level weights)."""
        if self._prediction_index_valid:
            return
        if set(self.sentence_to_node.keys()) != set(range(len(self.sentences))):
            raise ValueError("sentence_to_node mapping is inconsistent with sentence indices.")
        nodes, parent, mean, var, nos, max_depth = self.tree.flatten(len(self.sentences))
        for i, node in enumerate(nos):
            if node < 0:
                print(f"[Warning] Leaf path index for sentence ID {i} is None. "
                      f"This may indicate missing sentences in the tree.")
        weights = list(self._level_weights) if self._level_weights is not None else [1.0] * 6
        self._index = CobwebIndex(mean, var, parent, nos, weights, device=self.device)
        self._nodes = nodes
        self._node_to_index = {id(n): i for i, n in enumerate(nodes)}
        par = parent
        paths = []
        for s in nos:
            path, j = [], int(s)
            while j >= 0:
                path.append(j)
                j = int(par[j])
            paths.append(path[::-1] if s >= 0 else None)
        self._leaf_to_path_indices = paths
        self.max_depth = max(self.max_depth, max_depth)
        self._prediction_index_valid = True

    def force_rebuild_index(self):
        self._invalidate_prediction_index()
        self.build_prediction_index()

    def get_prediction_index_info(self):
        """CobwebWrapper.py:315-333 (the reference crashes here once the index is
        valid -- `_node_to_index` is never set; this one reports)."""
        info = {"index_valid": self._prediction_index_valid,
                "total_nodes": len(self._node_to_index) if self._prediction_index_valid else 0,
                "leaf_paths_cached": len(self._leaf_to_path_indices) if self._prediction_index_valid else 0,
                "means_cached": self._prediction_index_valid, "vars_cached": self._prediction_index_valid}
        if self._prediction_index_valid:
            info["means_shape"] = (self._index.n_nodes, self._index.dim)
            info["vars_shape"] = (self._index.n_nodes, self._index.dim)
            info["device"] = str(self.device)
            info.update(self._index.info)
        return info

    def get_node_path_stats(self, sentence_id):
        """CobwebWrapper.py:297-313."""
        self.build_prediction_index()
        if not (0 <= sentence_id < len(self._leaf_to_path_indices)) or self._leaf_to_path_indices[sentence_id] is None:
            return None, None
        path = self._leaf_to_path_indices[sentence_id]
        ns = [self._nodes[i] for i in path]
        means = torch.tensor(np.stack([n.mean for n in ns]), device=self.device)
        vars_ = torch.tensor(np.stack([self.tree.compute_var(n.meanSq, n.count) if n.count > 0
                                       else np.full(self.tree.dim, self.tree.prior_var, np.float32)
                                       for n in ns]), device=self.device)
        return means, vars_

    # ------------------------------------------------------------- level weights
    def set_level_weights(self, weights):
        """CobwebWrapper.py:335-346."""
        self._level_weights = weights
        self._weight_schedule = None
        self._invalidate_prediction_index()

    def set_weight_schedule(self, schedule_type, max_depth=10, **kwargs):
        """CobwebWrapper.py:348-366."""
        if self._prediction_index_valid:
            max_depth = self.max_depth
        self._weight_schedule = schedule_type
        self._schedule_params = kwargs
        self._level_weights = self._generate_weight_schedule(schedule_type, max_depth, **kwargs)
        self._invalidate_prediction_index()

    def _generate_weight_schedule(self, schedule_type, max_depth, **kwargs):
        """CobwebWrapper.py:368-408."""
        weights = []
        if schedule_type == "constant":
            weights = [kwargs.get("value", 1.0)] * max_depth
        elif schedule_type == "linear":
            start, end = kwargs.get("start", 1.0), kwargs.get("end", 1.0)
            if kwargs.get("direction", "increase") == "decrease":
                start, end = end, start
            if max_depth == 1:
                weights = [start]
            else:
                step = (end - start) / (max_depth - 1)
                weights = [start + i * step for i in range(max_depth)]
        elif schedule_type == "quadratic":
            start_n = kwargs.get("start_n", 1)
            for i in range(max_depth):
                n = start_n + i
                if n == 0:
                    n = 1
                weights.append(1 / (n ** 2))
        elif schedule_type == "exponential":
            base = kwargs.get("base", 0.5)
            weights = [base ** i for i in range(max_depth)]
        else:
            raise ValueError(f"Unknown schedule type: {schedule_type}")
        return weights

    def get_level_weights(self):
        return self._level_weights if self._level_weights is not None else [1.0, 1.0, 1.0, 1.0]

    def get_weight_schedule_info(self):
        return {"schedule_type": self._weight_schedule, "schedule_params": self._schedule_params,
                "current_weights": self.get_level_weights()}

    # ------------------------------------------------------------------ queries
    def _embed(self, input, is_embedding):
        emb = input if is_embedding else self.encode_func([input])[0]
        if torch.is_tensor(emb):
            return emb.detach().to(self.device, torch.float32).reshape(-1)
        return torch.as_tensor(np.asarray(emb, dtype=np.float32), device=self.device).reshape(-1)

    def cobweb_predict_indexed(self, input, k=5, return_ids=False, is_embedding=False):
        """CobwebWrapper.py:210-265 ("Cobweb Fast")."""
        self.build_prediction_index()
        n = self._index.n_sent if self._leaf_to_path_indices is None else len(self._leaf_to_path_indices)
        if n == 0:
            return []
        emb = input if is_embedding else self.encode_func([input])[0]
        if not torch.is_tensor(emb):
            # a host embedding (the harness's numpy query): host memory in and out
            ids, _ = self._index.score_topk_host(np.asarray(emb, dtype=np.float32).reshape(1, -1), min(k, n))
        else:
            ids, _ = self._index.score_topk(self._embed(emb, True)[None, :], min(k, n))
        row = ids[0].tolist()
        out = []
        for s in row:
            if 0 <= s < len(self.sentences):
                out.append(s if return_ids else self.sentences[s])
        return out

    def cobweb_predict_fast(self, input, k=5, return_ids=False, is_embedding=False):
        """CobwebWrapper.py:428-433 (alias)."""
        return self.cobweb_predict_indexed(input, k, return_ids, is_embedding)

    def cobweb_rank_scores(self, input, is_embedding=False):
        """CobwebWrapper.py:267-294: [n_sentences] leaf scores (no autograd)."""
        self.build_prediction_index()
        x = input.to(self.device) if is_embedding else self._embed(input, False)
        if len(self._leaf_to_path_indices) == 0:
            return torch.empty(0, device=self.device)
        return self._index.rank_scores(x.reshape(1, -1))[0]

    def cobweb_predict(self, input, k=5, return_ids=False, is_embedding=False):
        """CobwebWrapper.py:435-461 ("Cobweb Basic"): best-first categorize with
        retrieve_k=k and max_nodes=max_init_search; IndexError when fewer than k
        nodes with sentences are retrieved (CobwebTorchTree.py:289)."""
        self.build_prediction_index()
        emb = input if is_embedding else self.encode_func([input])[0]
        if torch.is_tensor(emb):
            x = emb.detach().to(self._index.device, torch.float32).reshape(1, -1)
            nodes, found, calls = self._index.categorize(x, k, self.max_init_search)
            nodes, found, calls = nodes.cpu().numpy(), found.cpu().numpy(), calls.cpu().numpy()
        else:   # a host embedding (the harness's numpy query): host memory in and out, one call
            nodes, found, calls = self._index.categorize_host(np.asarray(emb, np.float32).reshape(1, -1), k,
                                                              self.max_init_search)
        nf = int(found[0])
        # the reference's search draws one random() per heap push (one per log_prob call)
        # and one per retrieval (CobwebTorchTree.py:243,268,285) from the global stream
        # that ifit also draws from; advance it by as many, before the IndexError too
        advance_random(int(calls[0]) + nf)
        if nf < k:
            raise IndexError("list index out of range")
        results = []
        for nid in nodes[0].tolist():
            sid_lst = self._nodes[nid].sentence_id
            random.shuffle(sid_lst)      # CobwebWrapper.py:456, mutating the leaf's list
            for sid in sid_lst:
                if sid is None or sid >= len(self.sentences):
                    continue
                results.append(sid if return_ids else self.sentences[sid])
        return results

    # batched extensions (the benchmark's unit of work)
    def cobweb_predict_batch(self, queries, k=5):
        """[Q, D] queries -> (ids [Q, k] int64 tensor, scores [Q, k] float32), Fast path."""
        self.build_prediction_index()
        return self._index.score_topk(queries, k)

    def cobweb_categorize_batch(self, queries, k=5, max_nodes=None):
        """[Q, D] queries -> (node ids [Q, k] BFS order, n_found [Q], log_prob calls [Q])."""
        self.build_prediction_index()
        return self._index.categorize(queries, k, self.max_init_search if max_nodes is None else max_nodes)

    # -------------------------------------------------------------- persistence
    def dump_json(self, save_path=None):
        """CobwebWrapper.py:484-497."""
        state = {"tree": json.loads(self.tree.dump_json()), "sentences": self.sentences,
                 "embedding_dim": self.tree.shape[0]}
        if save_path:
            with open(save_path, "w") as f:
                json.dump(state, f, indent=2)
        return json.dumps(state, indent=2)

    @staticmethod
    def load_json(json_data, encode_func=lambda x: x, device=None):
        """CobwebWrapper.py:500-555, without its two bugs (identity encoder has no
        .shape; list sentence ids are unhashable): the tree shape comes from the
        JSON and every sentence id of a node maps to that node."""
        data = json.loads(json_data) if isinstance(json_data, str) else json_data
        w = CobwebWrapper.__new__(CobwebWrapper)
        CobwebWrapper.__init__(w, encode_func=encode_func, device=device)
        w.tree = CobwebTree.from_json(data["tree"])
        w.sentences = data.get("sentences", [])
        w.max_init_search = data.get("max_init_search", MAX_INIT_SEARCH)
        stack = [w.tree.root]
        while stack:
            n = stack.pop()
            for s in n.sentence_id or []:
                w.sentence_to_node[s] = n
            stack.extend(n.children)
        return w

    def save_binary(self, path):
        """Binary counterpart of dump_json (F2): the tree's BFS arrays plus the
        sentences (UTF-8 JSON bytes) in one .npz, readable with allow_pickle=False."""
        sent = np.frombuffer(json.dumps(list(self.sentences)).encode(), np.uint8)
        self.tree.save_binary(path, extra={"sentences": sent,
                                           "max_init_search": np.asarray([self.max_init_search], np.int64)})

    @staticmethod
    def load_binary(path, encode_func=lambda x: x, device=None):
        head, a = CobwebTree.read_binary(path)
        sentences = json.loads(bytes(a.pop("sentences")).decode()) if "sentences" in a else []
        mis = int(a.pop("max_init_search")[0]) if "max_init_search" in a else MAX_INIT_SEARCH
        t = CobwebTree.from_arrays(a["parent"], a["count"], a["mean"], a["meanSq"], a["sid_ptr"], a["sid_list"],
                                   prior_var=head["prior_var"])
        t.use_info, t.acuity_cutoff, t.use_kl, t.alpha = (head["use_info"], head["acuity_cutoff"], head["use_kl"],
                                                          head["alpha"])
        w = CobwebWrapper.from_tree(t, sentences, device=device)
        w.encode_func = encode_func
        w.max_init_search = mis
        return w

    @classmethod
    def from_tree(cls, tree, sentences, device=None):
        """Wrap an existing CobwebTree (e.g. CobwebTree.from_arrays / from_json)."""
        w = cls(device=device)
        w.tree = tree
        w.sentences = list(sentences)
        stack = [tree.root]
        while stack:
            n = stack.pop()
            for s in n.sentence_id or []:
                w.sentence_to_node[s] = n
            stack.extend(n.children)
        return w

    @classmethod
    def from_index(cls, index, sentences, encode_func=lambda x: x, node_of_sentence=None):
        """A query-only wrapper over a prebuilt CobwebIndex (e.g. a flat-synth tree at C3/C4
        scale, where the host keeps no node objects): the Fast / rank-score / batch entry
        points work; the add path needs the node tree.  With node_of_sentence (the BFS node
        of every sentence, as given to the index) Basic (cobweb_predict) works too: its id
        expansion reads per-node sentence lists made on first use (_NodeSentences)."""
        w = cls(device=index.device, encode_func=encode_func)
        w.sentences = sentences          # any sequence (len + indexing); not copied
        w._index = index
        w._prediction_index_valid = True
        if node_of_sentence is not None:
            w._nodes = _NodeSentences(node_of_sentence, index.n_nodes)
        return w

    def __len__(self):
        return len(self.sentences)


class _NodeSentences:
    """nodes[i].sentence_id for a wrapper without host Node objects: the sentence ids of
    BFS node i (ascending), made on first access and kept, so the in-place random.shuffle
    of Basic's id expansion (CobwebWrapper.py:456) persists across calls as on the
    reference's node lists."""

    class _Ref:
        __slots__ = ("sentence_id",)

        def __init__(self, ids):
            self.sentence_id = ids

    def __init__(self, node_of_sentence, n_nodes):
        nos = np.asarray(node_of_sentence, np.int64)
        order = np.argsort(nos, kind="stable")
        self._ids = order
        self._ptr = np.searchsorted(nos[order], np.arange(n_nodes + 1))
        self._made = {}

    def __len__(self):
        return len(self._ptr) - 1

    def __getitem__(self, i):
        r = self._made.get(i)
        if r is None:
            r = self._Ref([int(v) for v in self._ids[self._ptr[i]:self._ptr[i + 1]]])
            self._made[i] = r
        return r
