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
