"""Incremental fit (ifit) with the category-utility scoring on the GPU.

`TreeFitter.ifit(x)` is CobwebTorchTree.cobweb (CobwebTorchTree.py:143-233): the
host walks the tree and picks the operation (best / new / merge / split, fringe
split at a leaf) exactly as the reference does; every D-length computation runs in
libcwq on a device pool of node statistics:

* per tree level ONE `cwq_fit_kl` launch returns KL(c || P+x), KL(c+x || P+x) for
  every child c and KL(new || P+x) -- the terms of two_best_children,
  pu_for_insert and pu_for_new_child (CobwebTorchNode.py:374-515); a second launch
  returns the merge / split terms (:550-650) when those operations apply;
* node updates (increment_counts, update_counts_from_node, is_exact_match) are
  `cwq_fit_node_op` launches.

The scalar combinations (p(c) weights, sums over children, the descending sort by
(gain, count, random()), the operation choice by (pu, random(), name)) follow the
reference's float32 op order; `random()` is drawn from Python's global `random`
module in the same order as the reference, so a run seeded like the reference makes
the same tie-breaks.  Counts are kept on the host as well (exact small integers).
"""
import ctypes
import os
import random as _random_mod

import numpy as np
import torch

from ._lib import CWQ_ERR_OOM, check, lib
from .tree import Node

F32 = np.float32
_ADD, _COMBINE, _ZERO, _EXACT = 0, 1, 2, 3


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _seqsum(terms):
    """Python `score = 0.0; score += t` over float32 terms: sequential fp32 sum."""
    if len(terms) == 0:
        return F32(0.0)
    return F32(np.add.accumulate(np.asarray(terms, F32), dtype=F32)[-1])


class TreeFitter:
    def __init__(self, tree, device=None, rng=None):
        self.tree = tree
        self.D = tree.dim
        self.pv = F32(tree.prior_var)
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.rng = rng if rng is not None else _random_mod   # the reference draws from the global random()
        self.cap, self.used, self.free = 0, 0, []
        self.count = self.mean = self.meanSq = None
        self._flag = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self._kcap = 0
        # every launch and copy goes to the stream current at construction (looked up once;
        # the fitter's callers -- CobwebWrapper's build and add -- do not switch streams)
        self._s = torch.cuda.current_stream(self.dev)
        self._sp = ctypes.c_void_p(self._s.cuda_stream)
        self._owned = []
        self._grow(max(64, self._n_nodes() * 2))
        stack = [tree.root]
        while stack:       # upload the existing tree
            n = stack.pop()
            self._attach(n)
            stack.extend(n.children)

    # ---- device pool ----
    def _n_nodes(self):
        n, stack = 0, [self.tree.root]
        while stack:
            x = stack.pop()
            n += 1
            stack.extend(x.children)
        return n

    def _grow(self, cap):
        cnt = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        mean = torch.zeros((cap, self.D), dtype=torch.float32, device=self.dev)
        m2 = torch.zeros((cap, self.D), dtype=torch.float32, device=self.dev)
        if self.cap:
            cnt[:self.cap] = self.count
            mean[:self.cap] = self.mean
            m2[:self.cap] = self.meanSq
        self.count, self.mean, self.meanSq, self.cap = cnt, mean, m2, cap

    def _new_slot(self):
        if self.free:
            s = self.free.pop()
        else:
            if self.used == self.cap:
                self._grow(self.cap * 2)
            s = self.used
            self.used += 1
        self._op(_ZERO, s)
        return s

    def _attach(self, n):
        n.slot = self._new_slot()
        self._owned.append(n)
        if n.count != 0:
            self.count[n.slot] = float(n.count)
            self.mean[n.slot] = torch.from_numpy(np.asarray(n.mean, F32)).to(self.dev)
            self.meanSq[n.slot] = torch.from_numpy(np.asarray(n.meanSq, F32)).to(self.dev)

    def _stream(self):
        return self._sp

    def _op(self, op, dst, src=-1, x=None):
        check(lib().cwq_fit_node_op(op, _p(self.count), _p(self.mean), _p(self.meanSq), self.D, dst, src,
                                    _p(x) if x is not None else None, _p(self._flag), self._stream()))

    def _kl(self, p_slot, x, jobs):
        """One cwq_fit_kl launch over `jobs` (4 ints each); the jobs go up and the results
        come back through persistent pinned buffers: one stream sync per call."""
        jobs = np.asarray(jobs, np.int32).reshape(-1)
        n = jobs.size // 4
        if n > self._kcap:
            self._kcap = max(n, 2 * self._kcap)
            self._jobs_h = torch.empty(4 * self._kcap, dtype=torch.int32, pin_memory=True)
            self._jobs_d = torch.empty(4 * self._kcap, dtype=torch.int32, device=self.dev)
            self._out_h = torch.empty(self._kcap, dtype=torch.float32, pin_memory=True)
            self._out_d = torch.empty(self._kcap, dtype=torch.float32, device=self.dev)
            self._jobs_np, self._out_np = self._jobs_h.numpy(), self._out_h.numpy()
        self._jobs_np[:4 * n] = jobs
        with torch.cuda.stream(self._s):   # both copies on the stream the kernel runs on
            self._jobs_d[:4 * n].copy_(self._jobs_h[:4 * n], non_blocking=True)
            check(lib().cwq_fit_kl(_p(self.count), _p(self.mean), _p(self.meanSq), self.D, _p(x), float(self.pv),
                                   int(p_slot), _p(self._jobs_d), n, _p(self._out_d), self._sp))
            self._out_h[:n].copy_(self._out_d[:n], non_blocking=True)
        self._s.synchronize()
        return self._out_np[:n].copy()

    def _new_node(self):
        n = Node(self.D)
        n.slot = self._new_slot()
        self._owned.append(n)
        return n

    def _increment(self, n, x):
        self._op(_ADD, n.slot, x=x)
        n.count = F32(n.count + F32(1))

    def _combine(self, dst, src):
        self._op(_COMBINE, dst.slot, src.slot)
        dst.count = F32(dst.count + src.count)

    def _exact_match(self, n, x):
        self._op(_EXACT, n.slot, x=x)
        return bool(self._flag.item())

    # ---- CobwebTorchTree.cobweb ----
    def ifit(self, x_np):
        x = torch.as_tensor(np.asarray(x_np, F32)).to(self.dev)
        t = self.tree
        cur = t.root
        while cur is not None:
            if not cur.children and (cur.count == 0 or self._exact_match(cur, x)):
                self._increment(cur, x)
                break
            if not cur.children:                                   # fringe split :190-204
                new = self._new_node()
                new.parent = cur.parent
                self._combine(new, cur)                            # copy constructor
                cur.parent = new
                new.children.append(cur)
                if new.parent is not None:
                    new.parent.children.remove(cur)
                    new.parent.children.append(new)
                else:
                    t.root = new
                self._increment(new, x)
                cur = self._create_child(new, x)
                break
            action, b1, b2 = self._best_operation(cur, x)
            if action == "best":
                self._increment(cur, x)
                cur = b1
            elif action == "new":
                self._increment(cur, x)
                cur = self._create_child(cur, x)
                break
            elif action == "merge":                                # CobwebTorchNode.py:517-548
                self._increment(cur, x)
                nc = self._new_node()
                nc.parent = cur
                self._combine(nc, b1)
                self._combine(nc, b2)
                b1.parent = nc
                b2.parent = nc
                nc.children += [b1, b2]
                cur.children.remove(b1)
                cur.children.remove(b2)
                cur.children.append(nc)
                cur = nc
            else:                                                  # split :593-609
                cur.children.remove(b1)
                for c in b1.children:
                    c.parent = cur
                    cur.children.append(c)
                self.free.append(b1.slot)
                b1.slot = -1
        return cur

    def _create_child(self, parent, x):
        ch = self._new_node()
        ch.parent = parent
        self._increment(ch, x)
        parent.children.append(ch)
        return ch

    def _best_operation(self, cur, x):
        """two_best_children + get_best_operation (CobwebTorchNode.py:287-420)."""
        ch = cur.children
        b = len(ch)
        jobs = []
        for c in ch:
            jobs += [1, c.slot, -1, 1, 0, c.slot, -1, 1]
        jobs += [2, -1, -1, 1]
        out = self._kl(cur.slot, x, jobs)
        U, T, knew = out[0:2 * b:2], out[1:2 * b:2], out[2 * b]
        nc = np.array([c.count for c in ch], F32)
        nP1 = F32(cur.count + F32(1))
        p1 = (nc + F32(1)) / nP1
        p2 = nc / nP1
        gain = p1 * U - p2 * T
        rel = [(gain[i], nc[i], self.rng.random(), i) for i in range(b)]
        rel.sort(key=lambda r: (r[0], r[1], r[2]), reverse=True)
        i1 = rel[0][3]
        i2 = rel[1][3] if b > 1 else None
        b1, b2 = ch[i1], (ch[i2] if i2 is not None else None)
        t_all = p2 * T
        t_ins = t_all.copy()
        t_ins[i1] = p1[i1] * U[i1]
        pu_best = F32(_seqsum(t_ins) / F32(b))
        pu_new = F32(F32(_seqsum(t_all) + F32(F32(F32(1.0) / nP1) * knew)) / F32(b + 1))
        ops = [(pu_best, self.rng.random(), "best"), (pu_new, self.rng.random(), "new")]
        extra = []
        do_merge = b > 2 and b2 is not None
        do_split = len(b1.children) > 0
        if do_merge:
            extra += [3, b1.slot, b2.slot, 1]
        split_nodes = []
        if do_split:
            split_nodes = [c for c in ch if c is not b1] + list(b1.children)
            for c in split_nodes:
                extra += [0, c.slot, -1, 0]
        if extra:
            out2 = self._kl(cur.slot, x, extra)
            if do_merge:
                keep = [i for i in range(b) if i != i1 and i != i2]
                pm = F32(F32(F32(b1.count + b2.count) + F32(1)) / nP1)
                pu_merge = F32(F32(_seqsum(t_all[keep]) + F32(pm * out2[0])) / F32(b - 1))
                ops.append((pu_merge, self.rng.random(), "merge"))
            if do_split:
                ks = out2[1:] if do_merge else out2
                terms = np.array([c.count for c in split_nodes], F32) / F32(cur.count) * ks
                pu_split = F32(_seqsum(terms) / F32(b - 1 + len(b1.children)))
                ops.append((pu_split, self.rng.random(), "split"))
        ops.sort(reverse=True)
        return ops[0][2], b1, b2

    # ---- results back to the host tree ----
    def sync_to_host(self):
        cnt = self.count.cpu().numpy()
        mean = self.mean.cpu().numpy()
        m2 = self.meanSq.cpu().numpy()
        for n in self._owned:
            if n.slot >= 0:
                n.count = F32(cnt[n.slot])
                n.mean = mean[n.slot].copy()
                n.meanSq = m2[n.slot].copy()


# ----------------------------------------------------------------------------
# Device-resident ifit (cwq_fitdev.hip): the whole insert loop on the GPU
# ----------------------------------------------------------------------------
_ROOM = 1
_MAX_DEVICE_DIM = 1024


class DeviceTreeFitter:
    """CobwebTorchTree.cobweb (CobwebTorchTree.py:143-233) for a batch of rows with the
    tree resident on the GPU (libcwq cwq_fit_*): one kernel inserts every row in order,
    making every decision of TreeFitter.ifit above on the device -- the same KL
    arithmetic, the same float32 scalar order, and random() drawn from Python's own
    MT19937 stream (the state of `rng` goes to the device and comes back advanced by the
    draws made, exactly as if the reference had drawn them).  No host round trip per
    insert or per level; the host tree is rebuilt once after the batch.  Existing Node
    objects keep their identity (slots are never reused within a batch)."""

    def __init__(self, tree, device=None, rng=None):
        if tree.dim > _MAX_DEVICE_DIM:
            raise ValueError(f"DeviceTreeFitter supports dim <= {_MAX_DEVICE_DIM}")
        self.tree = tree
        self.D = tree.dim
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.rng = rng if rng is not None else _random_mod
        self.stats = {}

    # ---- host tree <-> slot arrays ----
    def _flatten(self):
        """The live host tree as slot arrays (root = slot 0, DFS preorder), children in
        list order as CSR."""
        nodes, stack = [], [self.tree.root]
        while stack:
            n = stack.pop()
            nodes.append(n)
            stack.extend(reversed(n.children))
        slot = {id(n): i for i, n in enumerate(nodes)}
        N = len(nodes)
        parent = np.full(N, -1, np.int32)
        cptr = np.zeros(N + 1, np.int32)
        cidx = []
        for i, n in enumerate(nodes):
            if n.parent is not None:
                parent[i] = slot[id(n.parent)]
            cidx.extend(slot[id(c)] for c in n.children)
            cptr[i + 1] = len(cidx)
        count = np.array([n.count for n in nodes], F32)
        mean = np.ascontiguousarray(np.stack([np.asarray(n.mean, F32) for n in nodes]))
        m2 = np.ascontiguousarray(np.stack([np.asarray(n.meanSq, F32) for n in nodes]))
        return nodes, parent, cptr, np.asarray(cidx if cidx else [0], np.int32), count, mean, m2

    def _pool_cap(self, n_nodes, remaining):
        """Node slots for one load: the existing nodes plus ~3 per remaining row (merges
        and fringe splits add nodes), capped by a device-memory budget -- the kernel
        stops for room (ROOM) and the host reloads into a fresh pool, so a cap only costs
        reloads.  Budget: CWQ_FIT_POOL_MB, else 40% of the free device memory;
        CWQ_FIT_POOL_SLOTS caps the slots beyond the loaded nodes (tests force reloads)."""
        want = n_nodes + 3 * remaining + 1024
        per_slot = 8 * self.D + 128          # mean + meanSq + links, arena, scratch (cwq_fitdev.hip)
        mb = os.environ.get("CWQ_FIT_POOL_MB")
        if mb:
            budget = int(mb) << 20
        else:
            free, _ = torch.cuda.mem_get_info(self.dev)
            budget = int(0.4 * free)
        cap = min(want, max(budget // per_slot, n_nodes + 1024))
        extra = os.environ.get("CWQ_FIT_POOL_SLOTS")
        if extra:
            cap = min(cap, n_nodes + max(int(extra), 80))
        return int(min(cap, 2 ** 31 - 1))

    def fit_batch(self, X):
        """Insert the rows of X in order; returns the node each row ended in (ifit's
        return value, CobwebTorchTree.py:123-141), as host Node objects.  If the device
        pool cannot be allocated or runs out mid-insert (CWQ_ERR_OOM), the remaining rows
        go through the host-driven TreeFitter from the last exported tree and random()
        state (the same tree either way).  Any other failure -- a HIP error, bad
        arguments, or a chip-wide KL pass that did not complete (a protocol fault) --
        raises RuntimeError instead of hiding behind a slower fit."""
        import time
        L = lib()
        X = torch.as_tensor(X if torch.is_tensor(X) else np.asarray(X, F32), dtype=torch.float32)
        X = X.to(self.dev).contiguous()
        n = int(X.shape[0])
        if n == 0:
            return []
        mt = np.ascontiguousarray(np.asarray(self.rng.getstate()[1], np.uint32))   # 624 words + index
        leaf = torch.full((n,), -1, dtype=torch.int32, device=self.dev)
        info = np.zeros(4, np.int64)
        sp = ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        out = [None] * n
        done, t_kernel, draws, loads, fallback = 0, 0.0, 0, 0, None

        def hand_back():   # the advanced random() state: the reference's draws, in its order
            old = self.rng.getstate()
            self.rng.setstate((old[0], tuple(int(v) for v in mt), old[2]))

        def failed(rc, call):
            """The host fallback's reason for a full pool; raise for anything else."""
            msg = L.cwq_fit_last_error().decode()
            if rc == CWQ_ERR_OOM:
                return msg
            raise RuntimeError(f"{call} failed (status {rc}): {msg}")

        while done < n:
            nodes, parent, cptr, cidx, count, mean, m2 = self._flatten()
            cap = self._pool_cap(len(nodes), n - done)
            h = ctypes.c_void_p()
            with torch.cuda.device(self.dev):
                rc = L.cwq_fit_create(self.dev.index, self.D, float(self.tree.prior_var), cap, ctypes.byref(h))
                if rc:
                    fallback = failed(rc, "cwq_fit_create")
                    break
                try:
                    rc = L.cwq_fit_load(h, len(nodes), 0, _np_ptr(parent), _np_ptr(cptr), _np_ptr(cidx),
                                        _np_ptr(count), _np_ptr(mean), _np_ptr(m2), _np_ptr(mt), sp)
                    if rc:
                        fallback = failed(rc, "cwq_fit_load")
                        break
                    loads += 1
                    t0 = time.perf_counter()
                    rc = L.cwq_fit_insert(h, ctypes.c_void_p(X[done:].data_ptr()), n - done,
                                          ctypes.c_void_p(leaf[done:].data_ptr()), _np_ptr(info), sp)
                    if rc:
                        # the pool ran out inside one insert: the device tree is
                        # mid-operation, so nothing of this load is kept
                        fallback = failed(rc, "cwq_fit_insert")
                        break
                    t_kernel += time.perf_counter() - t0
                    used = int(info[3])
                    out2 = np.zeros(2, np.int32)
                    P = np.zeros(used, np.int32)
                    CP = np.zeros(used + 1, np.int32)
                    CI = np.zeros(max(used, 1), np.int32)
                    CNT = np.zeros(used, F32)
                    MEAN = np.zeros((used, self.D), F32)
                    M2 = np.zeros((used, self.D), F32)
                    mt_new = mt.copy()
                    rc = L.cwq_fit_export(h, _np_ptr(out2), _np_ptr(P), _np_ptr(CP), _np_ptr(CI), _np_ptr(CNT),
                                          _np_ptr(MEAN), _np_ptr(M2), _np_ptr(mt_new), sp)
                    if rc:
                        fallback = failed(rc, "cwq_fit_export")
                        break
                finally:
                    L.cwq_fit_destroy(h)
            mt = mt_new
            objs = self._rebuild(nodes, out2, P, CP, CI, CNT, MEAN, M2)
            k = int(info[0])
            draws += int(info[1])
            lv = leaf[done:done + k].cpu().numpy()
            for i in range(k):
                out[done + i] = objs[int(lv[i])]
            done += k
            if int(info[2]) == _ROOM and k == 0:
                raise RuntimeError("device fit made no progress after a reload")
            if int(info[2]) != _ROOM:
                if done != n:
                    raise RuntimeError(f"device fit stopped after {done} of {n} rows (status {int(info[2])})")
                break
        hand_back()
        if fallback is not None:
            # the host tree and `mt` are the last export's: continue there on the host
            fitter = TreeFitter(self.tree, device=self.dev, rng=self.rng)
            for i in range(done, n):
                out[i] = fitter.ifit(X[i].cpu().numpy())
            fitter.sync_to_host()
        self.stats = {"rows": n, "kernel_s": round(t_kernel, 4), "random_draws": draws, "loads": loads,
                      "host_rows": n - done, "fallback": fallback}
        return out

    def _rebuild(self, nodes, out2, P, CP, CI, CNT, MEAN, M2):
        """Host Node objects from the exported slots (loaded slots keep their objects);
        returns the slot -> Node list (None for nodes a split removed)."""
        used, root = int(out2[0]), int(out2[1])
        objs = list(nodes) + [Node(self.D) for _ in range(used - len(nodes))]
        for i in range(used):
            if P[i] == -2:            # removed by a split
                objs[i].children = []
                objs[i].parent = None
                objs[i] = None
        for i in range(used):
            o = objs[i]
            if o is None:
                continue
            o.count = F32(CNT[i])
            o.mean = MEAN[i]
            o.meanSq = M2[i]
            o.parent = objs[P[i]] if P[i] >= 0 else None
            o.children = [objs[c] for c in CI[CP[i]:CP[i + 1]]]
        self.tree.root = objs[root]
        return objs


def _np_ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)
