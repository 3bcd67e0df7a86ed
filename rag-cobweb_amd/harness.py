"""Batched counterpart of the reference harness metrics.

Same definitions as src/utils/benchmark_utils.py:619-833 (`get_eval_ks`,
`evaluate_retrieval`), computed over a whole [Q, top_k] block of retrieved ids
instead of one Python loop iteration per query:

* recall@k = 1 if the target appears in the first k results (:651-653)
* mrr@k    = 1 / (first position of the target) (:654-655)
* ndcg@k   = sklearn.metrics.ndcg_score([ideal], [relevance]) with relevance the
  0/1 match vector of the first k results and ideal = sorted(relevance) (:657-661).
  sklearn averages over score ties; with binary relevance that is closed-form:
  with m relevant positions of which `a` are among the first m,
  DCG = (a/m)*sum_{r<=m} disc(r) + ((m-a)/(n-m))*sum_{m<r<=n} disc(r),
  IDCG = sum_{r<=m} disc(r), disc(r) = 1/log2(r+1).
Matching is by key: pass integer keys (e.g. a dict from sentence text to id) so
that duplicate sentences count like the reference's string comparison.

Also: exact brute-force flat-IP / flat-L2 top-k (the reference's FAISS and
"Torch Dot" baselines, :536-614) for ground truth.
"""
import time

import torch


def get_eval_ks(top_k):
    """benchmark_utils.py:619-622."""
    return sorted(k for k in [2, 3, 5, 10, 20, 50, 100] if k <= top_k)


def _disc(n, device):
    r = torch.arange(1, n + 1, device=device, dtype=torch.float64)
    return 1.0 / torch.log2(r + 1.0)


def retrieval_metrics(retrieved, targets, top_k, lengths=None):
    """retrieved: [Q, >=top_k] int keys (-1 = no result); targets: [Q] int keys.
    lengths: optional [Q] number of valid results per query (default: count of
    non-negative entries).  Returns the reference's metric dict (rounded to 4)."""
    retrieved = torch.as_tensor(retrieved)
    targets = torch.as_tensor(targets, device=retrieved.device)
    Q = retrieved.shape[0]
    if lengths is None:
        lengths = (retrieved >= 0).sum(1)
    lengths = torch.as_tensor(lengths, device=retrieved.device)
    # The reference's loop aborts a query whose result list holds ONE entry that is the
    # target: ndcg_score raises on a single document ("only meaningful when there is
    # more than 1 document"), the exception ends the k loop after recall/mrr of the
    # first k were added (benchmark_utils.py:807-820), so that query counts for
    # recall@k0 and mrr@k0 only and for no ndcg.
    single_hit = (lengths == 1) & (retrieved[:, 0] == targets)
    out = {}
    for ki, k in enumerate(get_eval_ks(top_k)):
        top = retrieved[:, :k]
        n = torch.clamp(lengths, max=k)                                    # len(top_k_results)
        pos = torch.arange(k, device=top.device)[None, :]
        valid = pos < n[:, None]
        rel = (top == targets[:, None]) & valid
        hit = rel.any(1)
        first = torch.where(hit, rel.float().argmax(1), torch.zeros_like(n))
        recall = hit.double()
        mrr = torch.where(hit, 1.0 / (first.double() + 1.0), torch.zeros(Q, dtype=torch.float64,
                                                                            device=top.device))
        m = rel.sum(1).double()
        a = (rel & (pos < m[:, None])).sum(1).double()
        disc = _disc(k, top.device)
        cum = torch.cat([torch.zeros(1, dtype=torch.float64, device=top.device), torch.cumsum(disc, 0)])
        mi = m.long()
        s_head = cum[mi]                                                     # sum_{r<=m}
        s_tail = cum[n.long()] - cum[mi]                                     # sum_{m<r<=n}
        nm = n.double() - m
        dcg = torch.where(m > 0, a / m.clamp(min=1) * s_head, torch.zeros_like(m)) + \
            torch.where(nm > 0, (m - a) / nm.clamp(min=1) * s_tail, torch.zeros_like(m))
        ndcg = torch.where(m > 0, dcg / s_head.clamp(min=1e-300), torch.zeros_like(m))
        ndcg = torch.where(single_hit, torch.zeros_like(ndcg), ndcg)
        if ki > 0:
            recall = torch.where(single_hit, torch.zeros_like(recall), recall)
            mrr = torch.where(single_hit, torch.zeros_like(mrr), mrr)
        out[f"recall@{k}"] = round(float(recall.mean()), 4)
        out[f"mrr@{k}"] = round(float(mrr.mean()), 4)
        out[f"ndcg@{k}"] = round(float(ndcg.mean()), 4)
    # reference key order: all recalls, then mrr, then ndcg
    ks = get_eval_ks(top_k)
    return {**{f"recall@{k}": out[f"recall@{k}"] for k in ks}, **{f"mrr@{k}": out[f"mrr@{k}"] for k in ks},
            **{f"ndcg@{k}": out[f"ndcg@{k}"] for k in ks}}


def evaluate_retrieval_batch(name, queries, target_keys, retrieve_batch, top_k=10, batch_size=10000,
                             key_of_id=None):
    """Batched `evaluate_retrieval` (benchmark_utils.py:710-833): retrieve_batch(Q_block,
    top_k) -> [q, top_k] ids; key_of_id maps ids to match keys (default identity).
    Latency = wall time per batch / batch size (the reference times one query per call)."""
    ids_all, t_total = [], 0.0
    for i in range(0, len(queries), batch_size):
        qb = queries[i:i + batch_size]
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t = time.time()
        ids = retrieve_batch(qb, top_k)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t_total += time.time() - t
        ids_all.append(torch.as_tensor(ids))
    ids = torch.cat(ids_all)
    keys = ids if key_of_id is None else torch.where(ids >= 0, torch.as_tensor(key_of_id, device=ids.device)[
        ids.clamp(min=0)], ids)
    m = retrieval_metrics(keys, torch.as_tensor(target_keys, device=keys.device), top_k)
    m["time_taken"] = round(t_total, 2)
    m["method"] = name
    m["avg_latency_ms"] = round(1000 * t_total / max(1, len(queries)), 4)
    return m


def brute_force_topk(corpus, queries, k, metric="ip", chunk=1024, exact=False, row_chunk=1 << 20):
    """Exact top-k by inner product (FAISS IndexFlatIP / Torch Dot) or L2.
    exact=True scores in float64 over row chunks with a running top-k (the fp32 GEMM
    of a library may reorder or split the sums; at 10M x 1024 the fp32 ranking of the
    GEMM kernel torch picks drifted from the exact one)."""
    corpus = torch.as_tensor(corpus, dtype=torch.float32)
    queries = torch.as_tensor(queries, dtype=torch.float32, device=corpus.device)
    if not exact:
        cn = (corpus * corpus).sum(1) if metric == "l2" else None
        out = []
        for i in range(0, queries.shape[0], chunk):
            ip = queries[i:i + chunk] @ corpus.T
            s = ip if metric == "ip" else 2 * ip - cn[None, :]
            out.append(torch.topk(s, k, dim=1).indices)
        return torch.cat(out)
    qd = queries.double()
    best_s = best_i = None
    for r0 in range(0, corpus.shape[0], row_chunk):
        c = corpus[r0:r0 + row_chunk].double()
        s = qd @ c.T
        if metric == "l2":
            s = 2 * s - (c * c).sum(1)[None, :]
        kk = min(k, s.shape[1])
        ts, ti = torch.topk(s, kk, dim=1)
        ti = ti + r0
        if best_s is None:
            best_s, best_i = ts, ti
        else:
            cs, ci = torch.cat([best_s, ts], 1), torch.cat([best_i, ti], 1)
            best_s, pos = torch.topk(cs, k, dim=1)
            best_i = torch.gather(ci, 1, pos)
    return best_i
