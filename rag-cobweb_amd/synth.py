"""Synthetic trees for the 1M-10M configurations.

The reference cannot build trees at these sizes (ifit is O(N^2 D) on Gaussian
data), so the benchmark trees are synthesised on the GPU with the statistics the
reference's own inserts would accumulate:

* flat-synth: root + N singleton leaves -- what the reference ifit builds for
  isotropic N(0, I) data (root fan-out = N).  Leaf: count 1,
  mean = x, meanSq = 0 (var == prior_var exactly).  Root: sequential Welford over
  X in index order (CobwebTorchNode.increment_counts, :57-68) -- computed by the
  libcwq `cwq_welford_groups` kernel in the same fp32 op order.
* two-level synth: root -> clusters -> leaves (cluster stats by the same Welford
  over each cluster's members in index order); exercises paths of length 3.

Outputs are the BFS-ordered arrays `CobwebIndex` takes.
"""
import torch

from .index import CompactVar, welford_groups
from .tree import PRIOR_VAR


def synthetic_corpus(n, dim, seed=0, device="cuda"):
    """X ~ N(0, I) float32, generated on the device with a seeded generator."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.randn((n, dim), generator=g, device=device, dtype=torch.float32)


def synthetic_queries(X, nq, seed=1, frac_perturbed=0.5, sigma=0.1):
    """Half fresh N(0, I), half corpus points + sigma*N(0, I) (targets = their ids)."""
    g = torch.Generator(device=X.device)
    g.manual_seed(seed)
    n_pert = int(nq * frac_perturbed)
    targets = torch.randint(0, X.shape[0], (n_pert,), generator=g, device=X.device)
    pert = X[targets] + sigma * torch.randn((n_pert, X.shape[1]), generator=g, device=X.device)
    fresh = torch.randn((nq - n_pert, X.shape[1]), generator=g, device=X.device)
    return torch.cat([pert, fresh]).contiguous(), targets


def clustered_corpus(n, dim, n_clusters, nq, seed=2):
    """Config C2's stand-in corpus (numpy, host): n rows in n_clusters Gaussian clusters
    (centres N(0, 4I), spread 0.3) and nq queries, half perturbed corpus rows (+0.1 N(0, I);
    `pick` = their rows), half fresh draws around the cluster centres.  The corpus of
    tests/test_gpu_c2.py, scripts/c2_probe.py and bench.py's hierarchical leg; the tree over
    it is built by the drop-in's own device ifit (a real Cobweb hierarchy, not synthesised)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    C = rng.standard_normal((n_clusters, dim)).astype(np.float32) * 2.0
    X = (C[rng.integers(0, n_clusters, n)] + 0.3 * rng.standard_normal((n, dim))).astype(np.float32)
    pick = rng.choice(n, nq // 2, replace=False)
    Qp = X[pick] + 0.1 * rng.standard_normal((nq // 2, dim))
    Qf = C[rng.integers(0, n_clusters, nq - nq // 2)] + 0.3 * rng.standard_normal((nq - nq // 2, dim))
    return X, np.concatenate([Qp, Qf]).astype(np.float32), pick


def _var_of(count, meanSq):
    # CobwebTorchTree.compute_var: meanSq / count + prior_var (fp32 division then add)
    return meanSq / count[:, None] + float(PRIOR_VAR)


def flat_synth(X, compact=False):
    """root + N leaves.  Returns dict(mean, var, parent, node_of_sentence) with the
    BFS order [root, leaf 0, ..., leaf N-1].  compact=True: var as a CompactVar (the
    leaves' prior_var as one scalar each, the root's row in full) -- the same index,
    without the [N+1, D] variance array."""
    N, D = X.shape
    order = torch.arange(N, device=X.device, dtype=torch.int64)
    gptr = torch.tensor([0, N], device=X.device, dtype=torch.int64)
    cnt, mu, m2 = welford_groups(X, order, gptr)
    mean = torch.cat([mu, X])
    if compact:
        var = CompactVar(torch.full((N + 1,), float(PRIOR_VAR), device=X.device),
                         torch.zeros(1, dtype=torch.int64), _var_of(cnt, m2))
    else:
        var = torch.cat([_var_of(cnt, m2), torch.full((N, D), float(PRIOR_VAR), device=X.device)])
    parent = torch.zeros(N + 1, dtype=torch.int64)
    parent[0] = -1
    nos = torch.arange(1, N + 1, dtype=torch.int64)
    count = torch.cat([cnt, torch.ones(N, device=X.device)])
    return dict(mean=mean, var=var, parent=parent.numpy(), node_of_sentence=nos.numpy(),
                root=(cnt, mu, m2), count=count, meanSq_root=m2)


def two_level_synth(X, labels):
    """root -> one node per non-empty cluster (ascending label) -> its members
    (ascending index).  BFS: [root, clusters..., leaves of cluster 0, ...]."""
    N, D = X.shape
    dev = X.device
    labels = labels.to(dev)
    uniq, inv, counts = torch.unique(labels, sorted=True, return_inverse=True, return_counts=True)
    G = uniq.numel()
    order = torch.argsort(inv * N + torch.arange(N, device=dev))          # by cluster, then index
    gptr = torch.zeros(G + 1, dtype=torch.int64, device=dev)
    gptr[1:] = torch.cumsum(counts, 0)
    c_cnt, c_mu, c_m2 = welford_groups(X, order, gptr)
    r_cnt, r_mu, r_m2 = welford_groups(X, torch.arange(N, device=dev), torch.tensor([0, N], device=dev))
    mean = torch.cat([r_mu, c_mu, X[order]])
    var = torch.cat([_var_of(r_cnt, r_m2), _var_of(c_cnt, c_m2),
                     torch.full((N, D), float(PRIOR_VAR), device=dev)])
    parent = torch.cat([torch.tensor([-1]), torch.zeros(G, dtype=torch.int64),
                        1 + torch.repeat_interleave(torch.arange(G), counts.cpu())])
    node_of_sentence = torch.empty(N, dtype=torch.int64)
    node_of_sentence[order.cpu()] = torch.arange(1 + G, 1 + G + N)
    count = torch.cat([r_cnt, c_cnt, torch.ones(N, device=dev)])
    meanSq = torch.cat([r_m2, c_m2, torch.zeros((N, D), device=dev)])   # leaves: count 1, meanSq 0
    return dict(mean=mean, var=var, parent=parent.numpy(), node_of_sentence=node_of_sentence.numpy(),
                n_clusters=G, count=count, meanSq=meanSq)


def balanced_synth(X, branching, depth, seed=0):
    """A deep tree shaped like a Cobweb hierarchy: the rows are split recursively
    `depth` times into `branching` groups of (nearly) equal size along a random direction
    per group (so that siblings are spatially coherent, as Cobweb's concepts are), the
    last level's groups holding the rows as count-1 leaves.  Node stats by sequential
    Welford over each node's rows (ascending row index).  BFS order: root, level 1, ...,
    level `depth`, then the leaves (by parent, then row index).  Empty groups are dropped."""
    N, D = X.shape
    dev = X.device
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    rows = torch.arange(N, device=dev)
    r_cnt, r_mu, r_m2 = welford_groups(X, rows, torch.tensor([0, N], device=dev))
    means, vars_, parent = [r_mu], [_var_of(r_cnt, r_m2)], [torch.tensor([-1])]
    off_prev, off = 0, 1                      # BFS offset of the previous / current level
    gl = torch.zeros(N, dtype=torch.int64, device=dev)
    for _ in range(depth):
        ng = int(gl.max()) + 1
        dirs = torch.randn((ng, D), generator=gen, device=dev)
        proj = (X * dirs[gl]).sum(1)
        order = torch.argsort(proj)
        order = order[torch.argsort(gl[order], stable=True)]    # by group, then projection
        cnt = torch.bincount(gl, minlength=ng)
        start = torch.cumsum(cnt, 0) - cnt
        rank = torch.empty(N, dtype=torch.int64, device=dev)
        rank[order] = rows - start[gl[order]]
        chunk = torch.clamp(rank * branching // cnt[gl].clamp(min=1), max=branching - 1)
        uniq, gl = torch.unique(gl * branching + chunk, sorted=True, return_inverse=True)
        G = uniq.numel()
        parent.append((uniq // branching).cpu() + off_prev)    # previous level's group -> its BFS index
        ordr = torch.argsort(gl * N + rows)                      # by group, then row index
        gptr = torch.zeros(G + 1, dtype=torch.int64, device=dev)
        gptr[1:] = torch.cumsum(torch.bincount(gl, minlength=G), 0)
        cc, mu, m2 = welford_groups(X, ordr, gptr)
        means.append(mu)
        vars_.append(_var_of(cc, m2))
        off_prev, off = off, off + G
    leaf_order = torch.argsort(gl * N + rows)
    G = int(gl.max()) + 1
    parent.append(off_prev + torch.repeat_interleave(torch.arange(G), torch.bincount(gl, minlength=G).cpu()))
    mean = torch.cat(means + [X[leaf_order]])
    var = torch.cat(vars_ + [torch.full((N, D), float(PRIOR_VAR), device=dev)])
    node_of_sentence = torch.empty(N, dtype=torch.int64)
    node_of_sentence[leaf_order.cpu()] = torch.arange(off, off + N)
    return dict(mean=mean, var=var, parent=torch.cat(parent).to(torch.int64).numpy(),
                node_of_sentence=node_of_sentence.numpy(), n_internal=off)


def tree_synth(X, parent, node_of_sentence):
    """The statistics of a given tree STRUCTURE over the rows X: every node's count, mean
    and meanSq by sequential Welford over the rows of its subtree (ascending row index),
    var = compute_var (prior_var for a node without rows).  parent: BFS-ordered parent
    array (-1 at the root); node_of_sentence: the node each row sits in.  Used to rebuild a
    device-ifit tree's shape (e.g. config C2's) from its saved structure without re-running
    ifit: the shape is ifit's, the statistics are batch Welford's (bit-different from the
    incremental ones, so not a reference tree -- a workload for the query kernels)."""
    N, D = X.shape
    dev = X.device
    par = torch.as_tensor(parent, dtype=torch.int64, device=dev)
    nos = torch.as_tensor(node_of_sentence, dtype=torch.int64, device=dev)
    Nn = par.numel()
    rows = torch.arange(N, device=dev)
    cur, nodes, rws = nos.clone(), [], []
    while True:
        live = cur >= 0
        if not bool(live.any()):
            break
        nodes.append(cur[live])
        rws.append(rows[live])
        cur = torch.where(live, par[cur.clamp(min=0)], cur)
    node_ids = torch.cat(nodes)
    row_ids = torch.cat(rws)
    order_key = torch.argsort(node_ids * N + row_ids)
    order = row_ids[order_key]
    cnt_per = torch.bincount(node_ids, minlength=Nn)
    gptr = torch.zeros(Nn + 1, dtype=torch.int64, device=dev)
    gptr[1:] = torch.cumsum(cnt_per, 0)
    cnt, mu, m2 = welford_groups(X, order, gptr)
    empty = cnt_per == 0
    var = torch.where(empty[:, None], torch.full_like(m2, float(PRIOR_VAR)), _var_of(cnt.clamp(min=1), m2))
    mu = torch.where(empty[:, None], torch.zeros_like(mu), mu)
    return dict(mean=mu, var=var, parent=par.cpu().numpy(), node_of_sentence=nos.cpu().numpy(), count=cnt)
