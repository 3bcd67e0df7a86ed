"""F2: binary tree format (CobwebTree.save_binary / load_binary, CobwebWrapper
save_binary / load_binary) round-trips the reference-built trees exactly, and the
array path to the device index matches the reference-order flatten().  CPU only."""
import gzip
import json
import os

import numpy as np

from conftest import GOLDEN, load_golden


def test_binary_round_trip_golden_trees(pkg, tmp_path):
    T = pkg.tree.CobwebTree
    for name in ("g1_hier_d32", "g5_hier_d384", "g4_twolevel_d48"):
        g = load_golden(name)
        t = T.from_arrays(g["parent"], g["count"], g["mean"], g["meanSq"], g["sid_ptr"], g["sid_list"])
        p = os.path.join(tmp_path, name + ".npz")
        t.save_binary(p)
        t2 = T.load_binary(p)
        a, b = t.to_arrays(), t2.to_arrays()
        for k in a:
            assert a[k].dtype == b[k].dtype and np.array_equal(a[k], b[k]), (name, k)
        assert t.dump_json() == t2.dump_json()
        # the arrays equal the golden BFS arrays the reference produced
        assert np.array_equal(a["parent"], g["parent"]) and np.array_equal(a["mean"], g["mean"])


def test_binary_from_reference_json(pkg, tmp_path):
    """Reference dump_json -> from_json (reversed children, as CobwebTorchTree.load_json)
    -> binary -> back: identical JSON."""
    with gzip.open(os.path.join(GOLDEN, "g1_hier_d32_tree.json.gz"), "rt") as f:
        js = f.read()
    T = pkg.tree.CobwebTree
    t = T.from_json(js)
    p = os.path.join(tmp_path, "t.npz")
    t.save_binary(p)
    assert T.load_binary(p).dump_json() == t.dump_json()
    # binary is much smaller than the JSON text
    assert os.path.getsize(p) < len(js)


def test_index_inputs_match_flatten(pkg, tmp_path):
    T = pkg.tree.CobwebTree
    g = load_golden("g4_twolevel_d48")
    t = T.from_arrays(g["parent"], g["count"], g["mean"], g["meanSq"], g["sid_ptr"], g["sid_list"])
    n_sent = int(g["sid_list"].max()) + 1
    _, parent, mean, var, nos, _ = t.flatten(n_sent)
    p = os.path.join(tmp_path, "t.npz")
    t.save_binary(p)
    head, arrs = T.read_binary(p)
    m2, v2, p2, nos2 = T.arrays_to_index_inputs(head, arrs, n_sent)
    assert np.array_equal(parent, p2) and np.array_equal(mean, m2) and np.array_equal(nos, nos2)
    assert np.array_equal(var.view(np.uint32), v2.view(np.uint32))   # bit-identical compute_var


def test_wrapper_binary_round_trip(pkg, tmp_path):
    g = load_golden("g1_hier_d32")
    T = pkg.tree.CobwebTree
    t = T.from_arrays(g["parent"], g["count"], g["mean"], g["meanSq"], g["sid_ptr"], g["sid_list"])
    n_sent = int(g["sid_list"].max()) + 1
    sents = [f"sentence {i} é中" for i in range(n_sent)]
    w = pkg.wrapper.CobwebWrapper.from_tree(t, sents, device="cpu")
    w.max_init_search = 777
    p = os.path.join(tmp_path, "w.npz")
    w.save_binary(p)
    w2 = pkg.wrapper.CobwebWrapper.load_binary(p, device="cpu")
    assert w2.sentences == sents and w2.max_init_search == 777
    assert json.loads(w2.dump_json())["tree"] == json.loads(w.dump_json())["tree"]
    assert set(w2.sentence_to_node) == set(w.sentence_to_node)
