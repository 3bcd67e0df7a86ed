"""Pin the CPU oracle (oracle/cobweb_oracle.py) against golden vectors produced by
the real reference (tests/golden/gen_golden.py).  CPU only."""
import gzip
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from oracle import cobweb_oracle as O

RTOL = 1e-5          # north-star tolerance on scores
HIER = ["g1_hier_d32", "g4_twolevel_d48", "g5_hier_d384", "g2_flat_d768", "g8_c1_d384"]


def tree_of(g):
    return O.tree_from_arrays(g["parent"], g["count"], g["mean"], g["meanSq"], g["sid_ptr"], g["sid_list"])


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-30))


def assert_topk_equiv(ids, ref_ids, ref_scores, rtol=RTOL):
    """Top-k identical except where the reference's own gap between the swapped
    candidates is below rtol*|score| (SURVEY §8(c) tie rule)."""
    ids = list(ids)
    ref_ids = list(ref_ids)
    if ids == ref_ids:
        return 0
    swaps = 0
    for pos, (a, b) in enumerate(zip(ids, ref_ids)):
        if a != b:
            sa, sb = ref_scores[a], ref_scores[b]
            assert abs(sa - sb) <= rtol * max(abs(sa), abs(sb)), (pos, a, b, sa, sb)
            swaps += 1
    return swaps


def test_prior_var_bits():
    g = load_golden("g1_hier_d32")
    assert np.float32(g["prior_var"]).tobytes() == O.PRIOR_VAR.tobytes()


@pytest.mark.parametrize("name", HIER)
def test_flatten_and_node_lp(name):
    g = load_golden(name)
    idx = O.flatten_tree(tree_of(g), int(g["n_sent"]))
    assert idx.n_nodes == len(g["parent"])
    np.testing.assert_array_equal(idx.parent, g["parent"])
    # (G8 stores the dense per-node / per-sentence arrays for its first 32 queries only)
    lp = np.stack([O.node_logprob_prime(x, idx.means, idx.vars) for x in g["Xq"][:len(g["node_lp"])]])
    assert rel_err(lp, g["node_lp"]) < RTOL


@pytest.mark.parametrize("name", HIER + ["g3_flat_inject_d32"])
def test_rank_scores_and_fast_topk(name):
    g = load_golden(name)
    if name.startswith("g3"):
        idx = O.flat_synth_index(g["X"])
    else:
        idx = O.flatten_tree(tree_of(g), int(g["n_sent"]))
    k = int(g["k"])
    for qi, x in enumerate(g["Xq"]):
        s = O.rank_scores(x, idx)
        if qi < len(g["rank_scores"]):
            assert rel_err(s, g["rank_scores"][qi]) < RTOL
            s = g["rank_scores"][qi]
        ids = O.predict_indexed(x, idx, k)
        assert_topk_equiv(ids, g["fast_ids"][qi], s.astype(np.float64))


def test_flat_synth_root_welford_bitwise():
    """Root stats of the flat-synth tree = sequential Welford in index order, bit
    for bit the reference's CobwebTorchNode.increment_counts sequence."""
    g = load_golden("g3_flat_inject_d32")
    root = O.welford_rows(g["X"])
    assert root.count == g["root_count"]
    np.testing.assert_array_equal(root.mean, g["root_mean"])
    np.testing.assert_array_equal(root.meanSq, g["root_meanSq"])


@pytest.mark.parametrize("name", HIER)
def test_categorize_pop_order(name):
    g = load_golden(name)
    root = tree_of(g)
    nodes = O.bfs_nodes(root)
    t = O.OTree(g["mean"].shape[1])
    t.root = root
    lpfull = np.array([[O.log_prob(n, x) for n in nodes] for x in g["Xq"][:4]])
    assert rel_err(lpfull, g["node_log_prob"]) < RTOL
    k = int(g["k"])
    for qi, x in enumerate(g["Xq"]):
        got, calls = t.categorize(x, k)
        assert [nodes.index(n) for n in got] == list(g["cat_nodes"][qi])
        assert calls == int(g["cat_calls"][qi])


@pytest.mark.parametrize("name", ["g1_hier_d32", "g5_hier_d384", "g2_flat_d768", "g8_c1_d384"])
def test_categorize_errors(name):
    g = load_golden(name)
    t = O.OTree(g["mean"].shape[1])
    t.root = tree_of(g)
    x = g["Xq"][0]
    for kk, mx, key in [(int(g["n_leaf_nodes"]) + 1, 100000, "err_k_too_big"), (int(g["k"]), 4, "err_max_nodes")]:
        raised = False
        try:
            t.categorize(x, kk, max_nodes=mx)
        except IndexError:
            raised = True
        assert raised == bool(g[key])


def test_level_weights_g1():
    g = load_golden("g1_hier_d32")
    root = tree_of(g)
    idx = O.flatten_tree(root, int(g["n_sent"]), [1.0, 2.0, 0.5])
    for qi, x in enumerate(g["Xq"][:8]):
        assert rel_err(O.rank_scores(x, idx), g["rank_scores_w3"][qi]) < RTOL
    idx = O.flatten_tree(root, int(g["n_sent"]), list(g["weights_exp"]))
    for qi, x in enumerate(g["Xq"][:8]):
        assert rel_err(O.rank_scores(x, idx), g["rank_scores_exp"][qi]) < RTOL


@pytest.mark.parametrize("name", ["g1_hier_d32", "g5_hier_d384"])
def test_ifit_structure(name):
    """The restated ifit reproduces the reference tree: same structure, same
    sentence placement, stats within float32 rounding."""
    g = load_golden(name)
    t = O.OTree(g["X"].shape[1], random.Random(0))
    for i, x in enumerate(g["X"]):
        leaf = t.ifit(x)
        leaf.sentence_id.append(i)
    nodes = O.bfs_nodes(t.root)
    pos = {id(n): i for i, n in enumerate(nodes)}
    parent = np.array([-1 if n.parent is None else pos[id(n.parent)] for n in nodes])
    np.testing.assert_array_equal(parent, g["parent"])
    sids = [s for n in nodes for s in n.sentence_id]
    np.testing.assert_array_equal(sids, g["sid_list"])
    np.testing.assert_array_equal([n.count for n in nodes], g["count"])
    np.testing.assert_allclose(np.stack([n.mean for n in nodes]), g["mean"], rtol=1e-5, atol=1e-5)


def test_tree_json_is_reference_format():
    """The reference tree JSON (CobwebTorchTree.dump_json) carries the same stats."""
    path = os.path.join(GOLDEN, "g1_hier_d32_tree.json.gz")
    if not os.path.exists(path):
        pytest.skip("no json fixture")
    with gzip.open(path, "rt") as f:
        d = json.loads(f.read())
    g = load_golden("g1_hier_d32")
    assert d["root"]["count"] == float(g["count"][0])
    np.testing.assert_array_equal(np.float32(d["root"]["mean"]), g["mean"][0])


@pytest.mark.parametrize("name", HIER + ["g3_flat_inject_d32"])
def test_torch_fast_restatement(name):
    """The torch-CPU op sequence bench.py times as the CPU baseline (TorchFastIndex,
    CobwebWrapper.py:222-257) returns the reference's Fast top-k on the goldens."""
    g = load_golden(name)
    if "parent" in g:
        idx = O.flatten_tree(tree_of(g), int(g["n_sent"]))
        T = O.TorchFastIndex(idx.means, idx.vars, idx.paths, idx.weights)
    else:   # injected flat index: root stats + one leaf per row
        root_var = O.compute_var(g["root_meanSq"], g["root_count"])
        T = O.TorchFastIndex.flat(g["root_mean"], root_var, g["X"])
    k = int(g["k"])
    for qi, x in enumerate(g["Xq"]):
        got = T.predict(x, k)
        ref = g["rank_scores"][qi] if qi < len(g["rank_scores"]) else O.rank_scores(x, idx)
        assert_topk_equiv(got, g["fast_ids"][qi], ref)


def test_interleaved_add_query_add_g9():
    """add -> Basic query -> add on ONE random() stream (golden G9 from the real
    reference): the oracle's predict advances its stream by the draws categorize makes
    (one per heap push and per retrieval, CobwebTorchTree.py:243,268,285, also when it
    raises IndexError) and shuffles each retrieved leaf's list (CobwebWrapper.py:456);
    the later inserts then build the reference's tree and the stream ends where the
    reference's did."""
    g = load_golden("g9_interleaved_d16")
    D = g["XA"].shape[1]
    t = O.OTree(D, random.Random(int(g["seed"])))
    n = 0

    def add(X):
        nonlocal n
        for x in X:
            t.ifit(x).sentence_id.append(n)
            n += 1

    def ragged(ptr, ids):
        return [list(ids[ptr[i]:ptr[i + 1]]) for i in range(len(ptr) - 1)]

    add(g["XA"])
    assert [t.predict(q, 4) for q in g["Q1"]] == ragged(g["out1_ptr"], g["out1_ids"])
    with pytest.raises(IndexError):
        t.predict(g["Q1"][0], 4, max_nodes=3)
    assert int(g["err_small_max"]) == 1
    add(g["XB"])
    assert [t.predict(q, 5) for q in g["Q2"]] == ragged(g["out2_ptr"], g["out2_ids"])
    add(g["XC"])
    assert t.rng.random() == float(g["random_after"])
    nodes = O.bfs_nodes(t.root)
    pos = {id(x): i for i, x in enumerate(nodes)}
    np.testing.assert_array_equal([-1 if x.parent is None else pos[id(x.parent)] for x in nodes], g["parent"])
    np.testing.assert_array_equal([s for x in nodes for s in x.sentence_id], g["sid_list"])
    np.testing.assert_array_equal([x.count for x in nodes], g["count"])
