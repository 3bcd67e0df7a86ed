"""Device-resident Cobweb query index: a thin Python handle over libcwq.

`CobwebIndex` owns one `cwq_index*` (include/cobweb_query.h).  It is the MI355X
replacement of the flattened prediction index the reference caches in
CobwebWrapper.build_prediction_index (CobwebWrapper.py:91-208) and of the query
op sequences that read it (:210-294, CobwebTorchTree.py:235-310).

Inputs/outputs are torch tensors on the index device; torch only supplies device
memory and the current HIP stream -- every computation runs in libcwq.
"""
import ctypes

import numpy as np
import torch

from ._lib import check, lib

DEFAULT_LEVEL_WEIGHTS = (1.0, 1.0, 1.0, 1.0, 1.0, 1.0)   # CobwebWrapper.py:155


def _dev(device):
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise ValueError(f"CobwebIndex lives on a GPU, got device {device}")
    return device if device.index is not None else torch.device("cuda", torch.cuda.current_device())


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream_raw(index):
    """torch's current HIP stream on device `index` as an int (the per-call path: no
    Stream object, no device switch -- libcwq sets its device itself)."""
    if _raw_stream is not None:
        return _raw_stream(index)
    return torch.cuda.current_stream(index).cuda_stream


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class CompactVar:
    """Node variances in compact form (cwq_index_create_cv): `row[i]` is node i's variance
    in every dimension -- every count-1 leaf has var = prior_var exactly
    (CobwebTorchTree.py:336-342) -- except for the nodes `an_nodes` (int64, ascending),
    whose full rows are `an_var` [n_an, D].  A flat 10M x 1024 tree's variances are 40 MB
    this way instead of 41 GB."""

    def __init__(self, row, an_nodes, an_var):
        self.row = row
        self.an_nodes = an_nodes
        self.an_var = an_var

    @property
    def shape(self):
        return (int(self.row.shape[0]), int(self.an_var.shape[1]))

    @classmethod
    def from_full(cls, var):
        """Compress a full [Nn, D] variance tensor (bitwise: a row counts as one value
        only when all D values have the same bits)."""
        var = torch.as_tensor(var, dtype=torch.float32)
        bits = var.view(torch.int32)
        iso = (bits == bits[:, :1]).all(1)
        an = torch.nonzero(~iso).squeeze(1).to(torch.int64)
        return cls(var[:, 0].contiguous(), an, var[an].contiguous())

    def full(self):
        """The [Nn, D] array it stands for (tests / small trees)."""
        n, d = self.shape
        out = self.row[:, None].expand(n, d).clone()
        if self.an_nodes.numel():
            out[self.an_nodes.to(out.device)] = self.an_var.to(out.device)
        return out

    def __getitem__(self, i):   # one node's variance row (bench's root var, small reads)
        i = int(i)
        hit = (self.an_nodes == i).nonzero()
        if hit.numel():
            return self.an_var[int(hit[0, 0])]
        return self.row[i].expand(self.shape[1])


class CobwebIndex:
    """Immutable flattened tree on one GPU.

    mean               [Nn, D] float32 (torch on any device, or numpy), BFS order
    var                [Nn, D] float32, or a CompactVar (one scalar per node with full rows
                       only where the D variances differ)
    parent             [Nn] int64, parent[0] = -1, non-decreasing (BFS)
    node_of_sentence   [n_sent] int64, node holding each sentence id (-1: none)
    level_weights      per-depth weights (CobwebWrapper.py:153-168)
    """

    def __init__(self, mean, var, parent, node_of_sentence, level_weights=None, device=None):
        self.device = _dev(device)
        L = self._L = lib()   # the handle belongs to the library that created it
        mean = torch.as_tensor(mean, dtype=torch.float32).to(self.device).contiguous()
        compact = isinstance(var, CompactVar)
        if compact:
            vrow = torch.as_tensor(var.row, dtype=torch.float32).to(self.device).contiguous()
            an_nodes = np.ascontiguousarray(np.asarray(torch.as_tensor(var.an_nodes).cpu(), dtype=np.int64))
            an_var = torch.as_tensor(var.an_var, dtype=torch.float32).to(self.device).contiguous()
            if (mean.dim() != 2 or vrow.shape != (mean.shape[0],) or an_var.dim() != 2
                    or an_var.shape != (an_nodes.size, mean.shape[1])):
                raise ValueError("compact var: row [n_nodes], an_var [n_an, dim] for mean [n_nodes, dim]")
        else:
            var = torch.as_tensor(var, dtype=torch.float32).to(self.device).contiguous()
            if mean.shape != var.shape or mean.dim() != 2:
                raise ValueError("mean and var must both be [n_nodes, dim]")
        parent = np.ascontiguousarray(np.asarray(parent, dtype=np.int64))
        nos = np.ascontiguousarray(np.asarray(node_of_sentence, dtype=np.int64))
        w = np.ascontiguousarray(np.asarray(
            DEFAULT_LEVEL_WEIGHTS if level_weights is None else level_weights, dtype=np.float64))
        self.n_nodes, self.dim = mean.shape
        self.n_sent = int(nos.size)
        self.level_weights = [float(x) for x in w]
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            if compact:
                check(L.cwq_index_create_cv(self.device.index, self.n_nodes, self.dim, _ptr(mean), _ptr(vrow),
                                            an_nodes.ctypes.data_as(ctypes.c_void_p), an_nodes.size, _ptr(an_var),
                                            parent.ctypes.data_as(ctypes.c_void_p),
                                            nos.ctypes.data_as(ctypes.c_void_p), self.n_sent,
                                            w.ctypes.data_as(ctypes.c_void_p), w.size, _stream(self.device),
                                            ctypes.byref(h)))
            else:
                check(L.cwq_index_create(self.device.index, self.n_nodes, self.dim, _ptr(mean), _ptr(var),
                                         parent.ctypes.data_as(ctypes.c_void_p), nos.ctypes.data_as(ctypes.c_void_p),
                                         self.n_sent, w.ctypes.data_as(ctypes.c_void_p), w.size,
                                         _stream(self.device), ctypes.byref(h)))
        self._h = h
        self.info = self._info()

    def _info(self):
        out = np.zeros(8, np.int64)
        check(self._L.cwq_index_info(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        keys = ["n_nodes", "dim", "n_sent", "internal_nodes", "leaf_rows", "isotropic_rows", "max_depth",
                "device_bytes"]
        return dict(zip(keys, (int(v) for v in out)))

    def filter_info(self):
        """How the filters centre their rows (cwq_index_filter_info): group-centred rows on
        clustered trees, the number of groups / group-centred rows, the int8 panel."""
        out = np.zeros(4, np.int64)
        check(self._L.cwq_index_filter_info(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        return {"group_centred": bool(out[0]), "groups": int(out[1]), "group_rows": int(out[2]),
                "int8_panel": bool(out[3])}

    def cut_info(self):
        """The tree-adaptive cut (cwq_index_cut_info): groups, top nodes (computed exactly by
        every pruned query), the deepest centre, groups whose rows are centred."""
        out = np.zeros(4, np.int64)
        check(self._L.cwq_index_cut_info(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        return {"groups": int(out[0]), "top_nodes": int(out[1]), "max_centre_depth": int(out[2]),
                "centred_groups": int(out[3])}

    def set_timing(self, enable=True):
        check(self._L.cwq_set_timing(self._h, int(bool(enable))))

    def last_timing(self):
        """Phase times (ms) of the last score_topk call, from HIP events on its stream."""
        out = np.zeros(8, np.float32)
        check(self._L.cwq_last_timing(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        return {"leaf_scan_ms": float(out[0]), "internal_ms": float(out[1]), "merge_ms": float(out[2]),
                "call_ms": float(out[3]), "leaf_scan_launches": int(out[4]), "sample_ms": float(out[5]),
                "fgemm_ms": float(out[6]), "rerank_ms": float(out[7])}

    def set_filter(self, mode):
        """Isotropic-row strategy of score_topk: -1 automatic, 0 exact fp32 scan,
        1 bf16-MFMA candidate filter + exact rerank (k <= 64).  Results are identical."""
        check(self._L.cwq_set_filter(self._h, int(mode)))

    def last_stats(self):
        out = np.zeros(6, np.int64)
        check(self._L.cwq_last_stats(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        return {"filter_queries": int(out[0]), "fallback_queries": int(out[1]), "filter_used": bool(out[2]),
                "path": {0: "scan", 1: "fgemm", 2: "stream"}.get(int(out[2]) & 255, "?"),
                "int8_pass": bool(int(out[2]) & 256),
                "candidates": int(out[3]), "exact_reranks": int(out[4]), "sample_rows": int(out[5])}

    def last_prune_stats(self):
        """Group pruning of the last Fast call (cwq_last_prune_stats): whether the
        index has it, the queries of the pruned chunk (0: not pruned), the (query, group)
        pairs its stage B computed beyond each query's best group, and the group count."""
        out = np.zeros(4, np.int64)
        check(self._L.cwq_last_prune_stats(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        return {"available": bool(out[0]), "queries": int(out[1]), "extra_pairs": int(out[2]), "groups": int(out[3])}

    def last_categorize_stats(self):
        """How the last categorize call resolved its queries (cwq_last_stats after
        cwq_categorize): counting over the bottleneck order, heap replay, the two-level
        replay of lists that end inside a bottleneck tie, DENSE re-runs."""
        out = np.zeros(6, np.int64)
        check(self._L.cwq_last_stats(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        return {"queries": int(out[0]), "dense_reruns": int(out[1]), "filter_reruns": int(out[2]),
                "by_count": int(out[3]), "by_replay": int(out[4]), "two_level": int(out[5])}

    def last_lazy_stats(self):
        """The last categorize call's exact lazy replays (cwq_last_lazy_stats): queries replayed
        straight away (the list paths skipped), and DENSE re-runs done by the lazy replay."""
        out = np.zeros(2, np.int64)
        check(self._L.cwq_last_lazy_stats(self._h, out.ctypes.data_as(ctypes.c_void_p)))
        return {"direct": int(out[0]), "dense_lazy": int(out[1])}

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._L.cwq_index_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- queries ----
    def _queries(self, q):
        q = torch.as_tensor(q, dtype=torch.float32)
        if q.dim() == 1:
            q = q[None, :]
        if q.dim() != 2 or q.shape[1] != self.dim:
            raise ValueError(f"queries must be [nq, {self.dim}]")
        return q.to(self.device).contiguous()

    def score_topk(self, q, k):
        """Top-k sentence ids/scores per query ("Cobweb Fast", A6).  One call per query is
        the reference harness's mode (benchmark_utils.py:801-805), so a float32 [nq, dim]
        tensor already on the index device goes straight through: no conversion, no device
        switch (the library selects its device itself), the raw current stream."""
        if not (type(q) is torch.Tensor and q.dtype == torch.float32 and q.device == self.device and q.dim() == 2
                and q.shape[1] == self.dim and q.is_contiguous()):
            q = self._queries(q)
        nq = q.shape[0]
        k = int(k)
        ids = torch.empty((nq, k), dtype=torch.int64, device=self.device)
        scores = torch.empty((nq, k), dtype=torch.float32, device=self.device)
        check(self._L.cwq_score_topk(self._h, q.data_ptr(), nq, k, ids.data_ptr(), scores.data_ptr(),
                                     _stream_raw(self.device.index)))
        return ids, scores

    def score_topk_host(self, q, k):
        """score_topk for a host (numpy) query batch -> numpy (ids [nq, k] int64, scores [nq, k]
        float32), the reference harness's call shape (cwq_score_topk_host: pinned staging in,
        the kernels write the results into mapped host memory; no torch tensors per call)."""
        q = np.ascontiguousarray(np.asarray(q, dtype=np.float32))
        if q.ndim == 1:
            q = q[None, :]
        if q.ndim != 2 or q.shape[1] != self.dim:
            raise ValueError(f"queries must be [nq, {self.dim}]")
        nq, k = q.shape[0], int(k)
        ids = np.empty((nq, k), np.int64)
        scores = np.empty((nq, k), np.float32)
        check(self._L.cwq_score_topk_host(self._h, q.ctypes.data, nq, k, ids.ctypes.data, scores.ctypes.data,
                                          _stream_raw(self.device.index)))
        return ids, scores

    def categorize_host(self, q, k, max_nodes=100000):
        """categorize for a host (numpy) query batch -> numpy (nodes [nq, k] int64, found [nq]
        int32, calls [nq] int64): cwq_categorize_host, the harness's Basic call shape (pinned
        staging in, the kernels write the results into mapped host memory)."""
        q = np.ascontiguousarray(np.asarray(q, dtype=np.float32))
        if q.ndim == 1:
            q = q[None, :]
        if q.ndim != 2 or q.shape[1] != self.dim:
            raise ValueError(f"queries must be [nq, {self.dim}]")
        nq, k = q.shape[0], int(k)
        nodes = np.empty((nq, k), np.int64)
        found = np.empty(nq, np.int32)
        calls = np.empty(nq, np.int64)
        mx = int(min(max_nodes, 2 ** 62)) if max_nodes != float("inf") else 2 ** 62
        check(self._L.cwq_categorize_host(self._h, q.ctypes.data, nq, k, mx, nodes.ctypes.data, found.ctypes.data,
                                          calls.ctypes.data, _stream_raw(self.device.index)))
        return nodes, found, calls

    def rank_scores(self, q):
        """All sentence scores (A8), [nq, n_sent]."""
        q = self._queries(q)
        out = torch.empty((q.shape[0], self.n_sent), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(self._L.cwq_rank_scores(self._h, _ptr(q), q.shape[0], _ptr(out), _stream(self.device)))
        return out

    def node_logprob(self, q, full=False):
        """Per-node log-likelihood in BFS order: lp' (full=False) or log_prob (full=True)."""
        q = self._queries(q)
        out = torch.empty((q.shape[0], self.n_nodes), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(self._L.cwq_node_logprob(self._h, _ptr(q), q.shape[0], int(bool(full)), _ptr(out),
                                         _stream(self.device)))
        return out

    def prefix_bounds(self, q):
        """Diagnostic: (lo, hi, exact) [nq, n_internal] -- the Fast path prefixes of the
        internal nodes (BFS order) by the exact pass, and the bf16-MFMA bounds the filter
        uses on hierarchical trees (NaN where the filter reads none)."""
        q = self._queries(q)
        shape = (q.shape[0], int(self.info["internal_nodes"]))
        lo, hi, ex = (torch.empty(shape, dtype=torch.float32, device=self.device) for _ in range(3))
        with torch.cuda.device(self.device):
            check(self._L.cwq_prefix_bounds(self._h, _ptr(q), q.shape[0], _ptr(lo), _ptr(hi), _ptr(ex),
                                          _stream(self.device)))
        return lo, hi, ex

    def categorize(self, q, k, max_nodes=100000):
        """Best-first categorize ("Cobweb Basic", A4): retrieved BFS node ids in pop
        order [nq, k], number found [nq], log_prob call count [nq]."""
        q = self._queries(q)
        nq = q.shape[0]
        nodes = torch.full((nq, k), -1, dtype=torch.int64, device=self.device)
        found = torch.empty(nq, dtype=torch.int32, device=self.device)
        calls = torch.empty(nq, dtype=torch.int64, device=self.device)
        mx = int(min(max_nodes, 2 ** 62)) if max_nodes != float("inf") else 2 ** 62
        with torch.cuda.device(self.device):
            check(self._L.cwq_categorize(self._h, _ptr(q), nq, int(k), mx, _ptr(nodes), _ptr(found), _ptr(calls),
                                       _stream(self.device)))
        return nodes, found, calls


def welford_groups(X, order, group_ptr):
    """Sequential-Welford stats per row group on the GPU (libcwq cwq_welford_groups).
    X [n, D] float32 cuda; order, group_ptr int64 cuda.  Returns (count, mean, meanSq)."""
    n, D = X.shape
    G = group_ptr.numel() - 1
    count = torch.empty(G, dtype=torch.float32, device=X.device)
    mean = torch.empty((G, D), dtype=torch.float32, device=X.device)
    meanSq = torch.empty((G, D), dtype=torch.float32, device=X.device)
    for g0 in range(0, G, 65535):
        g1 = min(G, g0 + 65535)
        with torch.cuda.device(X.device):
            check(lib().cwq_welford_groups(_ptr(X), n, D, _ptr(order), ctypes.c_void_p(group_ptr[g0:].data_ptr()),
                                           g1 - g0, ctypes.c_void_p(count[g0:].data_ptr()),
                                           ctypes.c_void_p(mean[g0:].data_ptr()),
                                           ctypes.c_void_p(meanSq[g0:].data_ptr()), _stream(X.device)))
    return count, mean, meanSq
