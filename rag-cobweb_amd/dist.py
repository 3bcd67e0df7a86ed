"""Multi-GPU serving: one process per GPU, torch.distributed over RCCL/xGMI.

The path shards embarrassingly: the flattened tree is frozen, so
rank 0 broadcasts its node statistics once (one collective per array over xGMI;
~6.2 GB for the 1M x 768 tree) and every rank builds its own device index.
Queries are split into contiguous per-rank slices; the query phase has no
collective.  An optional all-gather returns every rank's (ids, scores) to all
ranks (Q/P x k x 12 B per rank -- negligible next to the scan).

Backend-agnostic: "nccl" (RCCL) on GPUs; the same code runs on "gloo" with CPU
tensors, which is how tests/test_dist.py covers it without a GPU.
"""
import numpy as np
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _default_device():
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")


def broadcast_tree(mean, var, parent, node_of_sentence, src=0, device=None, stats=None, compact=False):
    """Broadcast a BFS-flattened tree from `src`.  Non-src ranks pass None for the
    arrays; every rank returns (mean, var, parent, node_of_sentence) with mean/var
    on `device` (the RCCL buffers) and the small structure arrays as numpy.

    `var` travels compressed: a row whose D values are one value repeated (every
    count-1 leaf: var = prior_var exactly, CobwebTorchTree.py:336-342) is sent as that
    scalar, and only the other rows are sent in full.  For a flat-synth tree that is
    N+1 scalars + one row instead of (N+1) x D floats (3.07 GB at C3).  `var` may be
    given as an index.CompactVar already.  compact=False: every rank returns the full
    [Nn, D] var, rebuilt bit for bit; compact=True: every rank returns the CompactVar
    (cwq_index_create_cv builds from it directly: no [Nn, D] array on any rank -- 41 GB
    at C4).  `stats` (dict) receives the bytes sent."""
    from .index import CompactVar
    rank, ws = world()
    dev = torch.device(device) if device is not None else _default_device()
    if rank == src:
        mean = torch.as_tensor(mean, dtype=torch.float32).to(dev).contiguous()
        cv = var if isinstance(var, CompactVar) else CompactVar.from_full(torch.as_tensor(var).to(dev))
        v0 = torch.as_tensor(cv.row, dtype=torch.float32).to(dev).contiguous()
        an_idx = torch.as_tensor(cv.an_nodes, dtype=torch.int64).to(dev).contiguous()
        an_rows = torch.as_tensor(cv.an_var, dtype=torch.float32).to(dev).contiguous()
        meta = torch.tensor([mean.shape[0], mean.shape[1], len(node_of_sentence), an_idx.numel()], dtype=torch.int64)
    else:
        meta = torch.zeros(4, dtype=torch.int64)
    meta = meta.to(dev)
    dist.broadcast(meta, src)
    n_nodes, dim, n_sent, n_an = (int(v) for v in meta.tolist())
    if rank == src:
        par = torch.as_tensor(np.asarray(parent, np.int64)).to(dev)
        nos = torch.as_tensor(np.asarray(node_of_sentence, np.int64)).to(dev)
    else:
        mean = torch.empty((n_nodes, dim), dtype=torch.float32, device=dev)
        v0 = torch.empty(n_nodes, dtype=torch.float32, device=dev)
        an_idx = torch.empty(n_an, dtype=torch.int64, device=dev)
        an_rows = torch.empty((n_an, dim), dtype=torch.float32, device=dev)
        par = torch.empty(n_nodes, dtype=torch.int64, device=dev)
        nos = torch.empty(n_sent, dtype=torch.int64, device=dev)
    sent = 0
    for t in (mean, v0, an_idx, an_rows, par, nos):
        if t.numel():
            dist.broadcast(t, src)
            sent += t.numel() * t.element_size()
    cv = CompactVar(v0, an_idx.cpu(), an_rows)
    if compact:
        var = cv
    elif rank != src or isinstance(var, CompactVar):
        var = cv.full()
    else:
        var = torch.as_tensor(var, dtype=torch.float32).to(dev).contiguous()
    if stats is not None:
        stats["bytes"] = sent
        stats["var_rows_sent"] = n_an
    return mean, var, par.cpu().numpy(), nos.cpu().numpy()


def timed_steps(step, steps, warmup, sync=None):
    """The bench's timed region: `warmup` untimed calls of step(), then exactly `steps`
    calls bracketed by a barrier + device sync on both sides; returns the MAX over ranks
    of the elapsed seconds (every rank gets the same value)."""
    import time
    rank, ws = world()
    sync = sync or (lambda: None)
    for _ in range(warmup):
        step()
    sync()
    if ws > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if ws > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=_default_device())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def shard_bounds(n, rank, ws):
    """Contiguous, balanced [lo, hi) slice of n items for `rank` (sizes differ by <= 1)."""
    base, rem = divmod(n, ws)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def sharded_query(fn, queries, k, gather=True):
    """Run `fn(local_queries, k) -> (ids [q,k] int64, scores [q,k] f32)` on this
    rank's slice and (gather=True) all-gather the results in global query order;
    gather=False returns this rank's slice only (the serving loop, no collective)."""
    rank, ws = world()
    n = queries.shape[0]
    lo, hi = shard_bounds(n, rank, ws)
    ids, scores = fn(queries[lo:hi], k)
    if ws == 1 or not gather:
        return ids, scores
    sizes = [shard_bounds(n, r, ws) for r in range(ws)]
    mx = max(h - l for l, h in sizes)
    pad_ids = torch.full((mx, k), -1, dtype=torch.int64, device=ids.device)
    pad_sc = torch.full((mx, k), float("-inf"), dtype=torch.float32, device=scores.device)
    pad_ids[:hi - lo] = ids
    pad_sc[:hi - lo] = scores
    all_ids = [torch.empty_like(pad_ids) for _ in range(ws)]
    all_sc = [torch.empty_like(pad_sc) for _ in range(ws)]
    dist.all_gather(all_ids, pad_ids)
    dist.all_gather(all_sc, pad_sc)
    out_ids = torch.cat([a[:h - l] for a, (l, h) in zip(all_ids, sizes)])
    out_sc = torch.cat([a[:h - l] for a, (l, h) in zip(all_sc, sizes)])
    return out_ids, out_sc


class ShardedCobwebIndex:
    """A CobwebIndex replicated on every rank from rank 0's tree."""

    def __init__(self, mean=None, var=None, parent=None, node_of_sentence=None, level_weights=None, src=0):
        from .index import CobwebIndex
        mean, var, parent, nos = broadcast_tree(mean, var, parent, node_of_sentence, src=src, compact=True)
        self.index = CobwebIndex(mean, var, parent, nos, level_weights, device=mean.device)

    def score_topk(self, queries, k):
        return sharded_query(self.index.score_topk, queries, k)
