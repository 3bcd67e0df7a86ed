"""CPU-side checks of the product: the C-ABI library loads and exports every symbol
include/cobweb_query.h declares; host tree / JSON logic.  No GPU compute here."""
import ctypes
import gzip
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, load_golden

HEADER = os.path.join(ROOT, "include", "cobweb_query.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(cwq_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_header_symbol(pkg):
    syms = header_symbols()
    assert len(syms) >= 9
    L = pkg.lib()
    for s in syms:
        assert hasattr(L, s), s
        assert s in pkg._lib.SIGNATURES, f"{s} has no ctypes signature"
    assert L.cwq_version() >= 100


def test_error_path_without_gpu_compute(pkg):
    """Argument validation happens before any device work."""
    L = pkg.lib()
    h = ctypes.c_void_p()
    rc = L.cwq_index_create(0, 0, 4, None, None, None, None, 0, None, 0, None, ctypes.byref(h))
    assert rc == pkg._lib.CWQ_ERR_ARG
    assert b"empty" in L.cwq_last_error()
    assert L.cwq_index_destroy(None) == 0


def test_tree_json_roundtrip(pkg):
    """The reference JSON loads (children reversed, as CobwebTorchTree.load_json does)
    and a second load restores the original BFS order exactly."""
    path = os.path.join(GOLDEN, "g1_hier_d32_tree.json.gz")
    if not os.path.exists(path):
        pytest.skip("fixture missing")
    g = load_golden("g1_hier_d32")
    with gzip.open(path, "rt") as f:
        js = f.read()
    t1 = pkg.CobwebTree.from_json(js)
    t2 = pkg.CobwebTree.from_json(t1.dump_json())
    nodes, parent, mean, var, nos, depth = t2.flatten(int(g["n_sent"]))
    np.testing.assert_array_equal(parent, g["parent"])
    np.testing.assert_array_equal(mean, g["mean"])
    np.testing.assert_array_equal(np.array([n.count for n in nodes], np.float32), g["count"])
    # single load: same nodes, reversed sibling order; every sentence keeps its path statistics
    n1, p1, m1, v1, nos1, _ = t1.flatten(int(g["n_sent"]))
    assert len(n1) == len(nodes)
    np.testing.assert_array_equal(m1[nos1], mean[nos])


def test_flatten_matches_oracle(pkg):
    from oracle import cobweb_oracle as O
    g = load_golden("g4_twolevel_d48")
    t = pkg.CobwebTree.from_arrays(g["parent"], g["count"], g["mean"], g["meanSq"], g["sid_ptr"], g["sid_list"])
    nodes, parent, mean, var, nos, _ = t.flatten(int(g["n_sent"]))
    ref = O.flatten_tree(O.tree_from_arrays(g["parent"], g["count"], g["mean"], g["meanSq"], g["sid_ptr"],
                                            g["sid_list"]), int(g["n_sent"]))
    np.testing.assert_array_equal(var, ref.vars)
    np.testing.assert_array_equal(parent, ref.parent)
    assert [p[-1] for p in ref.paths] == list(nos)


def test_prior_var_matches_reference_bits(pkg):
    g = load_golden("g1_hier_d32")
    assert np.float32(pkg.PRIOR_VAR).tobytes() == np.float32(g["prior_var"]).tobytes()


def test_compact_var_create_error_path(pkg):
    """cwq_index_create_cv validates before any device work."""
    L = pkg.lib()
    h = ctypes.c_void_p()
    rc = L.cwq_index_create_cv(0, 0, 4, None, None, None, 0, None, None, None, 0, None, 0, None, ctypes.byref(h))
    assert rc == pkg._lib.CWQ_ERR_ARG and b"empty" in L.cwq_last_error()
    parent = np.array([-1, 0], np.int64)
    an = np.array([5], np.int64)
    rc = L.cwq_index_create_cv(0, 2, 4, ctypes.c_void_p(16), ctypes.c_void_p(16), an.ctypes.data_as(ctypes.c_void_p),
                               1, ctypes.c_void_p(16), parent.ctypes.data_as(ctypes.c_void_p), None, 0, None, 0, None,
                               ctypes.byref(h))
    assert rc == pkg._lib.CWQ_ERR_ARG and b"an_nodes out of range" in L.cwq_last_error()


def test_compact_var_roundtrip_cpu(pkg):
    """CompactVar.from_full keeps one scalar per row whose D values share their bits and the
    other rows in full; full() rebuilds the array bit for bit (the broadcast / index form)."""
    import torch
    rng = np.random.default_rng(0)
    var = np.full((50, 7), pkg.PRIOR_VAR, np.float32)
    var[0] = rng.random(7).astype(np.float32) + 0.1
    var[13, 2] = np.float32(0.5)
    var[20] = np.float32(-0.0)          # one value repeated (bits), even a signed zero
    cv = pkg.index.CompactVar.from_full(torch.from_numpy(var))
    assert cv.an_nodes.tolist() == [0, 13] and cv.shape == (50, 7)
    assert torch.equal(cv.full().view(torch.int32), torch.from_numpy(var).view(torch.int32))
    np.testing.assert_array_equal(cv[13].numpy(), var[13])
    np.testing.assert_array_equal(cv[7].numpy(), var[7])


def test_device_mt19937_is_pythons_random(pkg):
    """The device fitter's random() (cwq_fitdev.hip, run here on the host) is Python's
    random.random() stream from the same state, and leaves the same state behind."""
    import random
    r = random.Random(2024)
    for _ in range(5):
        r.random()
    st = np.ascontiguousarray(np.asarray(r.getstate()[1], np.uint32))
    out = np.zeros(2000, np.float64)
    assert pkg.lib().cwq_mt19937_draw(st.ctypes.data_as(ctypes.c_void_p), 2000,
                                      out.ctypes.data_as(ctypes.c_void_p)) == 0
    want = np.array([r.random() for _ in range(2000)])
    np.testing.assert_array_equal(out, want)
    assert tuple(int(v) for v in st) == r.getstate()[1]


def test_device_mt19937_chain_twist_is_pythons_stream(pkg):
    """The parallel generator of the chip-wide fit (mt_gen_wave: the twist as 227
    independent chains over a wave's lanes, run here in its host form) gives Python's
    getrandbits(32) outputs from the same state -- across many twists, from a mid-block
    index -- and leaves random()'s state behind."""
    import random
    r = random.Random(77)
    for _ in range(101):
        r.random()
    st = np.ascontiguousarray(np.asarray(r.getstate()[1], np.uint32))
    n = 624 * 9 + 313
    out = np.zeros(n, np.uint32)
    assert pkg.lib().cwq_mt19937_words(st.ctypes.data_as(ctypes.c_void_p), n, out.ctypes.data_as(ctypes.c_void_p)) == 0
    want = np.array([r.getrandbits(32) for _ in range(n)], np.uint32)
    np.testing.assert_array_equal(out, want)
    assert tuple(int(v) for v in st) == r.getstate()[1]


@pytest.mark.parametrize("n", [0, 1, 311, 312, 624, 4095, 4096, 10**6 + 1])
def test_native_random_advance_equals_getrandbits(pkg, n):
    """The Basic query's random() advance (wrapper.advance_random: cwq_mt19937_skip for
    large n, getrandbits below) leaves the state getrandbits(64 n) leaves -- from fresh,
    mid-block and end-of-block indices -- and the stream continues identically."""
    import random
    for warm in (0, 1, 311, 624):
        a, b = random.Random(5 + warm), random.Random(5 + warm)
        for _ in range(warm):
            a.random()
            b.random()
        pkg.wrapper.advance_random(n, a)
        if n:
            b.getrandbits(64 * n)
        assert a.getstate() == b.getstate()
        assert [a.random() for _ in range(700)] == [b.random() for _ in range(700)]
    # the native entry point on its own (also below the wrapper's cut-over)
    r = random.Random(9)
    r.random()
    st = np.ascontiguousarray(np.asarray(r.getstate()[1], np.uint32))
    assert pkg.lib().cwq_mt19937_skip(st.ctypes.data_as(ctypes.c_void_p), 2 * n) == 0
    if n:
        r.getrandbits(64 * n)
    assert tuple(int(v) for v in st) == r.getstate()[1]
