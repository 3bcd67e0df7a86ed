"""World-size-2 gloo tests of the multi-GPU layer (rag-cobweb_amd/dist.py) on CPU:
tree broadcast is bit-exact, shards cover every query once, and the gathered
results equal a single-process run.  The per-rank scorer here is the CPU oracle
(GPU ranks use libcwq; the distributed plumbing is identical)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        import cobweb_pkg
        from oracle import cobweb_oracle as O
        pkg = cobweb_pkg.load()
        D = pkg.dist
        g = load_golden("g4_twolevel_d48")
        if rank == 0:
            var = O.compute_var(g["meanSq"], g["count"][:, None]).astype(np.float32)
            nos = np.full(int(g["n_sent"]), -1, np.int64)
            for i in range(len(g["parent"])):
                for s in g["sid_list"][g["sid_ptr"][i]:g["sid_ptr"][i + 1]]:
                    nos[s] = i
            args = (g["mean"], var, g["parent"], nos)
        else:
            args = (None, None, None, None)
        mean, var, parent, nos = D.broadcast_tree(*args, device="cpu")
        # every rank rebuilds the oracle index from the broadcast arrays
        paths = []
        for s in nos:
            p, j = [], int(s)
            while j >= 0:
                p.append(j)
                j = int(parent[j])
            paths.append(p[::-1])
        idx = O.FlatIndex(mean.numpy(), var.numpy(), parent, paths)

        def scorer(qs, k):
            ids, sc = [], []
            for x in qs.numpy():
                s = O.rank_scores(x, idx)
                o, v = O.topk_ids_scores(s, k)
                ids.append(o)
                sc.append(v)
            return torch.tensor(np.array(ids), dtype=torch.int64), torch.tensor(np.array(sc))

        Xq = torch.from_numpy(g["Xq"][:q])
        ids, scores = D.sharded_query(scorer, Xq, 10)
        if rank == 0:
            np.savez(result_path, ids=ids.numpy(), scores=scores.numpy(), mean=mean.numpy())
    finally:
        dist.destroy_process_group()


def test_shard_bounds_cover_exactly_once():
    import cobweb_pkg
    D = cobweb_pkg.load().dist
    for n in [0, 1, 7, 10000, 10001]:
        for ws in [1, 2, 3, 8]:
            seen = []
            for r in range(ws):
                lo, hi = D.shard_bounds(n, r, ws)
                seen += list(range(lo, hi))
            assert seen == list(range(n))


@pytest.mark.parametrize("q", [7, 12])
def test_gloo_world2_broadcast_and_gather(tmp_path, q):
    g = load_golden("g4_twolevel_d48")
    out = str(tmp_path / "res.npz")
    mp.spawn(_worker, args=(2, _free_port(), q, out), nprocs=2, join=True)
    r = np.load(out)
    np.testing.assert_array_equal(r["mean"], g["mean"])          # bit-exact broadcast
    np.testing.assert_array_equal(r["ids"], g["fast_ids"][:q])   # gathered in global order
    np.testing.assert_allclose(r["scores"], np.take_along_axis(g["rank_scores"][:q], g["fast_ids"][:q], 1),
                               rtol=1e-5)


def _bench_path_worker(rank, ws, port, result_path, strong):
    """The functions bench.py calls on every rank, in bench.py's order: broadcast_tree
    (compressed var), timed_steps (barrier + max over ranks) around sharded_query /
    a per-rank batch, on gloo with the CPU oracle as the per-rank scorer."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        import cobweb_pkg
        from oracle import cobweb_oracle as O
        D = cobweb_pkg.load().dist
        rng = np.random.default_rng(5)
        X = rng.standard_normal((300, 24)).astype(np.float32)
        ref = O.flat_synth_index(X)
        if rank == 0:
            var = ref.vars.copy()
            var[7, 3] *= np.float32(1.5)          # one anisotropic row: sent in full
            args = (ref.means, var, ref.parent, np.arange(1, 301))
        else:
            args = (None, None, None, None)
        st = {}
        # bench.py's form: the variances stay compact on every rank (no [Nn, D] array)
        mean, cvar, parent, nos = D.broadcast_tree(*args, device="cpu", stats=st, compact=True)
        assert isinstance(cvar, cobweb_pkg.load().index.CompactVar)
        assert cvar.row.shape == (301,) and cvar.an_var.shape == (2, 24)   # root + the anisotropic row
        var = cvar.full()
        idx = O.FlatIndex(mean.numpy(), var.numpy(), parent, [[0, int(s)] for s in nos])

        def scorer(qs, k):
            out = [O.topk_ids_scores(O.rank_scores(x, idx), k) for x in qs.numpy()]
            return (torch.tensor(np.array([o[0] for o in out]), dtype=torch.int64),
                    torch.tensor(np.array([o[1] for o in out])))

        Q = torch.from_numpy(np.concatenate([X[:6] + 0.05, rng.standard_normal((5, 24)).astype(np.float32)]))
        calls = []
        if strong:
            step = lambda: calls.append(D.sharded_query(scorer, Q, 5, gather=False))   # noqa: E731
        else:
            step = lambda: calls.append(scorer(Q, 5))                                   # noqa: E731
        dt = D.timed_steps(step, 2, 1)
        lo, hi = D.shard_bounds(Q.shape[0], rank, ws) if strong else (0, Q.shape[0])
        gathered = D.sharded_query(scorer, Q, 5)          # the all-gathered form, for the check
        np.savez(result_path + f".{rank}.npz", var=var.numpy(), ids=calls[-1][0].numpy(), lo=lo, hi=hi, dt=dt,
                 n_calls=len(calls), bytes=st["bytes"], an=st["var_rows_sent"], gathered=gathered[0].numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("strong", [False, True])
def test_gloo_world2_bench_path(tmp_path, strong):
    from oracle import cobweb_oracle as O
    out = str(tmp_path / "bench")
    mp.spawn(_bench_path_worker, args=(2, _free_port(), out, strong), nprocs=2, join=True)
    rng = np.random.default_rng(5)
    X = rng.standard_normal((300, 24)).astype(np.float32)
    ref = O.flat_synth_index(X)
    var = ref.vars.copy()
    var[7, 3] *= np.float32(1.5)
    Q = np.concatenate([X[:6] + 0.05, rng.standard_normal((5, 24)).astype(np.float32)])
    want = np.array([O.topk_ids_scores(O.rank_scores(x, O.FlatIndex(ref.means, var, ref.parent,
                                                                   [[0, 1 + i] for i in range(300)])), 5)[0]
                     for x in Q])
    r = [np.load(out + f".{i}.npz") for i in range(2)]
    for ri in r:
        np.testing.assert_array_equal(ri["var"], var)            # compressed var rebuilt bit for bit
        assert int(ri["an"]) == 2                                  # only the root and the anisotropic leaf in full
        assert int(ri["n_calls"]) == 3                             # warmup 1 + steps 2
        np.testing.assert_array_equal(ri["gathered"], want)
        np.testing.assert_array_equal(ri["ids"], want[int(ri["lo"]):int(ri["hi"])])
    assert float(r[0]["dt"]) == float(r[1]["dt"])                  # max over ranks on both
    if strong:
        assert [int(r[0]["lo"]), int(r[0]["hi"]), int(r[1]["lo"]), int(r[1]["hi"])] == [0, 6, 6, 11]
