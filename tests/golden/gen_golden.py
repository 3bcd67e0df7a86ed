"""Generate golden vectors by running the REAL reference (Teachable-AI-Lab/RAG-Cobweb
@ 2025-09-26, mounted read-only at /root/reference) in the build container.

Run:  python tests/golden/gen_golden.py            (takes a few minutes on CPU)

Only data leaves this script: inputs, the reference's tree statistics and the
reference's outputs, written as tests/golden/*.npz (+ one gzipped tree JSON that
the reference's own CobwebTorchTree.dump_json produced).  No reference source
or bytecode is copied (bytecode writing is disabled).  The GPU box never runs
this script and never reads /root/reference.

Import shim: graphviz is only used for visualisation
(CobwebWrapper.py:9,644) and is absent here, so an in-memory stub stands in.
"""
import gzip
import os
import random
import sys
import time
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

import numpy as np
import torch

_g = types.ModuleType("graphviz")
_g.Digraph = object
sys.modules["graphviz"] = _g
sys.path.insert(0, REF)
from src.cobweb.CobwebWrapper import CobwebWrapper          # noqa: E402
from src.cobweb.CobwebTorchTree import CobwebTorchTree      # noqa: E402
from src.cobweb.CobwebTorchNode import CobwebTorchNode      # noqa: E402

torch.set_num_threads(8)
K = 10


class _Quiet:
    def __enter__(self):
        self._o = sys.stdout
        sys.stdout = open(os.devnull, "w")

    def __exit__(self, *a):
        sys.stdout.close()
        sys.stdout = self._o


def bfs(root):
    out, q, h = [], [root], 0
    while h < len(q):
        n = q[h]
        h += 1
        out.append(n)
        q.extend(n.children)
    return out


def export_tree(root, n_sent):
    nodes = bfs(root)
    pos = {id(n): i for i, n in enumerate(nodes)}
    parent = np.array([-1 if n.parent is None else pos[id(n.parent)] for n in nodes], np.int64)
    # children must appear contiguously and in list order in BFS; record it
    count = np.array([float(n.count) for n in nodes], np.float32)
    mean = np.stack([n.mean.numpy() for n in nodes]).astype(np.float32)
    meanSq = np.stack([n.meanSq.numpy() for n in nodes]).astype(np.float32)
    sid_ptr, sid_list = [0], []
    for n in nodes:
        sid_list += list(n.sentence_id or [])
        sid_ptr.append(len(sid_list))
    return nodes, pos, dict(parent=parent, count=count, mean=mean, meanSq=meanSq,
                            sid_ptr=np.array(sid_ptr, np.int64), sid_list=np.array(sid_list, np.int64),
                            n_sent=np.int64(n_sent))


def ref_node_lp(w, Xq):
    """lp' per node with the reference's own expression on the reference's own
    flattened tensors (CobwebWrapper.py:230-236)."""
    M, V = w._node_means, w._node_vars
    out = []
    for x in Xq:
        x = torch.tensor(x)
        diff_sq = (x.unsqueeze(0) - M) ** 2
        out.append((-0.5 * (torch.log(V).sum(dim=1) + (diff_sq / V).sum(dim=1))).numpy())
    return np.stack(out).astype(np.float32)


def count_log_prob_calls():
    orig = CobwebTorchNode.log_prob
    box = {"n": 0}

    def wrapped(self, inst):
        box["n"] += 1
        return orig(self, inst)
    return orig, wrapped, box


def query_outputs(w, Xq, pos, cat=True, k=K, tag="", n_dense=None):
    """All reference outputs for a batch of query embeddings (the dense per-node /
    per-sentence score arrays only for the first `n_dense` queries when given)."""
    res = {}
    with _Quiet():
        w.build_prediction_index()
    Xd = Xq if n_dense is None else Xq[:n_dense]
    res["node_lp"] = ref_node_lp(w, Xd)
    res["rank_scores"] = np.stack([w.cobweb_rank_scores(x).detach().numpy() for x in Xd]).astype(np.float32)
    torch.manual_seed(1234)
    res["fast_ids"] = np.array([w.cobweb_predict_fast(x, k, return_ids=True) for x in Xq], np.int64)
    if cat:
        orig, wrapped, box = count_log_prob_calls()
        CobwebTorchNode.log_prob = wrapped
        try:
            leaves, calls = [], []
            for x in Xq:
                box["n"] = 0
                r = w.tree.categorize(torch.tensor(x), use_best=True, max_nodes=w.max_init_search, retrieve_k=k)
                leaves.append([pos[id(n)] for n in r])
                calls.append(box["n"])
        finally:
            CobwebTorchNode.log_prob = orig
        res["cat_nodes"] = np.array(leaves, np.int64)
        res["cat_calls"] = np.array(calls, np.int64)
        random.seed(99)
        res["basic_ids_first"] = np.array([w.cobweb_predict(x, k, return_ids=True)[0] for x in Xq], np.int64)
        # full log_prob (with 2*pi) of every node, reference CobwebTorchNode.log_prob :100-104
        nodes = bfs(w.tree.root)
        res["node_log_prob"] = np.array([[float(n.log_prob(torch.tensor(x))) for n in nodes] for x in Xq[:4]],
                                        np.float32)
    return res


def clusters(n, d, n_clusters, seed, spread=3.0, noise=1.0):
    rng = np.random.default_rng(seed)
    centers = rng.normal(0, spread, (n_clusters, d)).astype(np.float32)
    lab = rng.integers(0, n_clusters, n)
    X = (centers[lab] + rng.normal(0, noise, (n, d))).astype(np.float32)
    return X, centers


def make_queries(X, n_pert, n_fresh, seed, fresh_fn):
    rng = np.random.default_rng(seed)
    pick = rng.choice(len(X), n_pert, replace=False)
    Xp = (X[pick] + 0.1 * rng.standard_normal((n_pert, X.shape[1]))).astype(np.float32)
    return np.concatenate([Xp, fresh_fn(rng, n_fresh)]).astype(np.float32), pick


def build_by_ifit(X, seed):
    random.seed(seed)
    torch.manual_seed(seed)
    t = time.time()
    with _Quiet():
        w = CobwebWrapper(corpus=[f"s{i}" for i in range(len(X))], corpus_embeddings=X)
    return w, time.time() - t


def case_ifit(name, X, Xq, pick, extra=None, cat=True, json_dump=False, weights_cases=False, n_dense=None):
    w, secs = build_by_ifit(X, 0)
    nodes, pos, tree = export_tree(w.tree.root, len(X))
    print(f"[{name}] ifit N={len(X)} D={X.shape[1]} nodes={len(nodes)} in {secs:.1f}s", flush=True)
    res = query_outputs(w, Xq, pos, cat=cat, n_dense=n_dense)
    data = dict(X=X, Xq=Xq, pick=pick, prior_var=np.float32(w.tree.prior_var), k=np.int64(K), **tree, **res)
    if cat:
        # edge cases: k larger than the number of retrievable leaves; a tiny max_nodes
        n_leaf_nodes = int(sum(1 for n in nodes if n.sentence_id))
        for kk, mx, key in [(n_leaf_nodes + 1, 100000, "err_k_too_big"), (K, 4, "err_max_nodes")]:
            try:
                w.tree.categorize(torch.tensor(Xq[0]), use_best=True, max_nodes=mx, retrieve_k=kk)
                data[key] = np.int64(0)
            except IndexError:
                data[key] = np.int64(1)
        data["n_leaf_nodes"] = np.int64(n_leaf_nodes)
    if weights_cases:
        with _Quiet():
            w.set_level_weights([1.0, 2.0, 0.5])
            data["rank_scores_w3"] = np.stack([w.cobweb_rank_scores(x).detach().numpy() for x in Xq])
            w.set_weight_schedule("exponential", max_depth=10, base=0.5)
            data["weights_exp"] = np.array(w._level_weights, np.float64)
            data["rank_scores_exp"] = np.stack([w.cobweb_rank_scores(x).detach().numpy() for x in Xq])
            w.set_weight_schedule("linear", max_depth=8, start=0.5, end=2.0, direction="increase")
            data["weights_lin"] = np.array(w._level_weights, np.float64)
            w.set_weight_schedule("quadratic", max_depth=6, start_n=0)
            data["weights_quad"] = np.array(w._level_weights, np.float64)
    if json_dump:
        with gzip.open(os.path.join(OUT, f"{name}_tree.json.gz"), "wt") as f:
            f.write(w.tree.dump_json())
    if extra:
        data.update(extra)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **data)
    return w


def inject_flat(X):
    """Flat-synth tree (root + N leaves) injected into a reference CobwebWrapper:
    root stats accumulated by the reference's own CobwebTorchNode.increment_counts
    in index order (SURVEY.md §8(c) 'Large shapes')."""
    N, D = X.shape
    tree = CobwebTorchTree(shape=(D,), device="cpu")
    root = tree.root
    Xt = torch.from_numpy(X)
    for i in range(N):
        root.increment_counts(Xt[i])
    w = CobwebWrapper.__new__(CobwebWrapper)
    w.encode_func = lambda x: x
    w.device = "cpu"
    w.max_init_search = 100000
    w.tree = tree
    w.sentences = [f"s{i}" for i in range(N)]
    w._leaf_to_path_indices = [[0, 1 + i] for i in range(N)]
    means = torch.cat([root.mean[None, :], Xt], 0)
    vars_ = torch.empty_like(means)
    vars_[0] = tree.compute_var(root.meanSq, root.count)
    vars_[1:] = tree.compute_var(torch.zeros(D), torch.tensor(1.0))
    w._node_means, w._node_vars = means, vars_
    rows = torch.arange(N).repeat_interleave(2)
    cols = torch.stack([torch.zeros(N, dtype=torch.long), torch.arange(1, N + 1)], 1).reshape(-1)
    vals = torch.full((2 * N,), 0.5)
    w._path_matrix = torch.sparse_coo_tensor(torch.stack([rows, cols]), vals, (N, N + 1)).coalesce()
    w._prediction_index_valid = True
    return w, root


def case_injected_flat(name, N, D, nq, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, D)).astype(np.float32)
    Xq, pick = make_queries(X, nq // 2, nq - nq // 2, seed + 1,
                            lambda r, n: r.standard_normal((n, D)).astype(np.float32))
    w, root = inject_flat(X)
    res = {"node_lp": ref_node_lp(w, Xq),
           "rank_scores": np.stack([w.cobweb_rank_scores(x).detach().numpy() for x in Xq]).astype(np.float32)}
    torch.manual_seed(1234)
    res["fast_ids"] = np.array([w.cobweb_predict_fast(x, K, return_ids=True) for x in Xq], np.int64)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), X=X, Xq=Xq, pick=pick, k=np.int64(K),
                        root_count=np.float32(root.count), root_mean=root.mean.numpy(),
                        root_meanSq=root.meanSq.numpy(), prior_var=np.float32(w.tree.prior_var), **res)
    print(f"[{name}] injected flat N={N} D={D}", flush=True)


def case_two_level(name, N, D, n_clusters, seed):
    """root -> clusters -> leaves, built from reference node objects, flattened by the
    reference's own build_prediction_index.  Includes a duplicate-sentence leaf
    (count 2, var == prior_var) and a near-duplicate leaf (count 2, anisotropic)."""
    X, _ = clusters(N, D, n_clusters, seed, spread=2.0)
    X[5] = X[4]                                          # exact duplicate -> one leaf, 2 sentences
    X[7] = X[6] + np.float32(1e-3) * np.arange(D, dtype=np.float32) / D   # near duplicate
    tree = CobwebTorchTree(shape=(D,), device="cpu")
    root = tree.root
    rng = np.random.default_rng(seed + 7)
    lab = rng.integers(0, n_clusters, N)
    lab[5] = lab[4]
    lab[7] = lab[6]
    cl = []
    for c in range(n_clusters):
        node = CobwebTorchNode(shape=(D,), device="cpu")
        node.tree, node.parent = tree, root
        root.children.append(node)
        cl.append(node)
    leaf_of = {}
    Xt = torch.from_numpy(X)
    for i in range(N):
        root.increment_counts(Xt[i])
        cl[lab[i]].increment_counts(Xt[i])
        key = {5: 4, 7: 6}.get(i, i)
        if key in leaf_of:
            leaf = leaf_of[key]
        else:
            leaf = CobwebTorchNode(shape=(D,), device="cpu")
            leaf.tree, leaf.parent = tree, cl[lab[i]]
            cl[lab[i]].children.append(leaf)
            leaf_of[key] = leaf
        leaf.increment_counts(Xt[i])
        leaf.sentence_id.append(i)
    w = CobwebWrapper.__new__(CobwebWrapper)
    w.encode_func = lambda x: x
    w.device = "cpu"
    w.max_init_search = 100000
    w._prediction_index_valid = False
    w._index_to_node = {}
    w._node_means = w._node_vars = w._leaf_to_path_indices = None
    w.max_depth = 0
    w.tree = tree
    w.sentences = [f"s{i}" for i in range(N)]
    w.sentence_to_node = {i: leaf_of[{5: 4, 7: 6}.get(i, i)] for i in range(N)}
    Xq, pick = make_queries(X, 12, 12, seed + 1,
                            lambda r, n: (2.0 * r.standard_normal((n, D))).astype(np.float32))
    nodes, pos, tr = export_tree(root, N)
    res = query_outputs(w, Xq, pos, cat=True)
    with _Quiet():
        w.set_level_weights([0.25, 1.0, 3.0])
        res["rank_scores_w3"] = np.stack([w.cobweb_rank_scores(x).detach().numpy() for x in Xq])
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), X=X, Xq=Xq, pick=pick, k=np.int64(K),
                        prior_var=np.float32(tree.prior_var), **tr, **res)
    print(f"[{name}] two-level N={N} D={D} nodes={len(nodes)}", flush=True)


def case_interleaved(name, seed=9):
    """add -> Basic query -> add -> Basic query -> add, all on ONE global random()
    stream: categorize draws one random() per heap push and one per
    retrieval (CobwebTorchTree.py:243,268,285), cobweb_predict shuffles every retrieved
    leaf's sentence list (CobwebWrapper.py:456), and ifit draws its tie-breaks from the
    same stream (CobwebTorchNode.py:362-368,406).  The corpus holds exact duplicates so
    leaves carry several sentences (the shuffles draw), and one query runs with a tiny
    max_init_search so that it raises IndexError after its draws."""
    D, ncl = 16, 6
    rng = np.random.default_rng(seed)
    C = rng.normal(0, 3.0, (ncl, D)).astype(np.float32)

    def block(n):
        X = (C[rng.integers(0, ncl, n)] + rng.normal(0, 1.0, (n, D))).astype(np.float32)
        dup = rng.choice(n, n // 6, replace=False)
        X[dup] = X[rng.integers(0, n, len(dup))]
        return X

    XA, XB, XC = block(120), block(80), block(60)
    XA = np.concatenate([XA, XA[:12]])               # repeats of earlier rows too
    Q1 = (C[rng.integers(0, ncl, 6)] + rng.normal(0, 1.0, (6, D))).astype(np.float32)
    Q2 = np.concatenate([XA[[0, 3, 5]], XB[[1, 2]], Q1[:1]]).astype(np.float32)
    random.seed(seed)
    torch.manual_seed(seed)
    with _Quiet():
        w = CobwebWrapper(corpus=[f"a{i}" for i in range(len(XA))], corpus_embeddings=XA)
    out1 = [w.cobweb_predict(q, 4, return_ids=True) for q in Q1]
    w.max_init_search = 3
    err = 0
    try:
        w.cobweb_predict(Q1[0], 4, return_ids=True)
    except IndexError:
        err = 1
    w.max_init_search = 100000
    with _Quiet():
        w.add_sentences([f"b{i}" for i in range(len(XB))], XB)
    out2 = [w.cobweb_predict(q, 5, return_ids=True) for q in Q2]
    with _Quiet():
        w.add_sentences([f"c{i}" for i in range(len(XC))], XC)
    after = random.random()
    nodes, pos, tree = export_tree(w.tree.root, len(w.sentences))

    def ragged(lists):
        return (np.array([0] + list(np.cumsum([len(x) for x in lists])), np.int64),
                np.array([s for x in lists for s in x], np.int64))
    p1, l1 = ragged(out1)
    p2, l2 = ragged(out2)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), XA=XA, XB=XB, XC=XC, Q1=Q1, Q2=Q2,
                        seed=np.int64(seed), out1_ptr=p1, out1_ids=l1, out2_ptr=p2, out2_ids=l2,
                        err_small_max=np.int64(err), random_after=np.float64(after),
                        prior_var=np.float32(w.tree.prior_var), **tree)
    print(f"[{name}] interleaved add/query N={len(w.sentences)} nodes={len(nodes)} err={err}", flush=True)


def main():
    which = sys.argv[1:] or ["g1", "g4", "g3", "g5", "g2", "g8", "g9"]
    t0 = time.time()
    if "g1" in which:   # hierarchical, built by the reference ifit
        X, C = clusters(300, 32, 10, 0)
        Xq, pick = make_queries(X, 20, 20, 1, lambda r, n: (C[r.integers(0, 10, n)] +
                                                           r.standard_normal((n, 32))).astype(np.float32))
        case_ifit("g1_hier_d32", X, Xq, pick, json_dump=True, weights_cases=True)
    if "g4" in which:
        case_two_level("g4_twolevel_d48", 3000, 48, 16, 4)
    if "g3" in which:
        case_injected_flat("g3_flat_inject_d32", 20000, 32, 16, 3)
    if "g5" in which:   # C1-dimension hierarchical tree (D=384), built by ifit
        X, C = clusters(400, 384, 8, 5, spread=1.0)
        Xq, pick = make_queries(X, 8, 8, 6, lambda r, n: (C[r.integers(0, 8, n)] +
                                                         r.standard_normal((n, 384))).astype(np.float32))
        case_ifit("g5_hier_d384", X, Xq, pick)
    if "g2" in which:   # isotropic N(0,I) at D=768 -> flat tree
        rng = np.random.default_rng(2)
        X = rng.standard_normal((1000, 768)).astype(np.float32)
        Xq, pick = make_queries(X, 8, 8, 12, lambda r, n: r.standard_normal((n, 768)).astype(np.float32))
        case_ifit("g2_flat_d768", X, Xq, pick)
    if "g9" in which:   # add / Basic query / add on one random() stream
        case_interleaved("g9_interleaved_d16")
    if "g8" in which:   # config C1's own shape: 1,500 x 384 N(0,I) by ifit, 300 queries
        rng = np.random.default_rng(8)
        X = rng.standard_normal((1500, 384)).astype(np.float32)
        Xq, pick = make_queries(X, 150, 150, 18, lambda r, n: r.standard_normal((n, 384)).astype(np.float32))
        case_ifit("g8_c1_d384", X, Xq, pick, n_dense=32)
    print(f"done in {time.time() - t0:.0f}s")


if __name__ == "__main__":
    main()
