"""Host-side concept tree: node statistics, the reference JSON format and the
BFS flattening that feeds the device index.

Mirrors the data model of CobwebTorchNode (src/cobweb/CobwebTorchNode.py:31-55)
and CobwebTorchTree (src/cobweb/CobwebTorchTree.py:23-121): each node keeps
count, mean and meanSq (Welford M2) in float32, children in list order and the
sentence ids it holds.  Arrays here are numpy float32; the query path never
touches them after `flatten()` hands them to libcwq.
"""
import json
import math
from collections import deque

import numpy as np

F32 = np.float32
# CobwebTorchTree.py:35-40: prior_var = 1 / (2 * e * pi_tensor), computed in fp32
PRIOR_VAR = F32(1.0) / (F32(2 * math.e) * F32(math.pi))


class Node:
    __slots__ = ("count", "mean", "meanSq", "children", "parent", "sentence_id", "slot")

    def __init__(self, dim):
        self.count = F32(0.0)
        self.mean = np.zeros(dim, F32)
        self.meanSq = np.zeros(dim, F32)
        self.children = []
        self.parent = None
        self.sentence_id = []
        self.slot = -1          # row in the device stats pool while a TreeFitter owns the tree

    def increment_counts(self, x):
        """Welford insert, CobwebTorchNode.py:57-68 (fp32, same op order)."""
        self.count = F32(self.count + F32(1))
        delta = x - self.mean
        self.mean = self.mean + delta / self.count
        self.meanSq = self.meanSq + delta * (x - self.mean)


class CobwebTree:
    """Tree container with the reference's defaults (CobwebTorchTree.py:23-41):
    use_info=True, acuity_cutoff=False, use_kl=True, prior_var=1/(2*e*pi)."""

    def __init__(self, shape, prior_var=None):
        self.shape = tuple(int(s) for s in shape)
        self.dim = self.shape[0]
        self.use_info, self.acuity_cutoff, self.use_kl, self.alpha = True, False, True, 1e-8
        self.prior_var = PRIOR_VAR if prior_var is None else F32(prior_var)
        self.root = Node(self.dim)

    def compute_var(self, meanSq, count):
        """CobwebTorchTree.py:336-342 with acuity_cutoff=False."""
        return meanSq / count + self.prior_var

    # ---- reference JSON (CobwebTorchTree.dump_json / load_json, :67-121) ----
    def dump_json(self):
        head = {"use_info": self.use_info, "acuity_cutoff": self.acuity_cutoff, "use_kl": self.use_kl,
                "shape": list(self.shape), "alpha": self.alpha, "prior_var": float(self.prior_var)}

        def node_dict(n):
            return {"count": float(n.count), "mean": n.mean.tolist(), "meanSq": n.meanSq.tolist(),
                    "sentence_id": list(n.sentence_id), "children": [node_dict(c) for c in n.children]}

        # iterative to survive deep trees
        out = dict(head)
        out["root"] = node_dict(self.root) if self._depth() < 500 else self._iter_dict()
        return json.dumps(out)

    def _depth(self):
        d, q = 0, deque([(self.root, 0)])
        while q:
            n, k = q.popleft()
            d = max(d, k)
            q.extend((c, k + 1) for c in n.children)
        return d

    def _iter_dict(self):
        def shell(n):
            return {"count": float(n.count), "mean": n.mean.tolist(), "meanSq": n.meanSq.tolist(),
                    "sentence_id": list(n.sentence_id), "children": []}
        root = shell(self.root)
        stack = [(self.root, root)]
        while stack:
            n, d = stack.pop()
            for c in n.children:
                cd = shell(c)
                d["children"].append(cd)
                stack.append((c, cd))
        return root

    @classmethod
    def from_json(cls, json_string):
        """Rebuild a tree the way CobwebTorchTree.load_json (:94-121) does, including
        its LIFO traversal: every node's children list comes back reversed."""
        data = json.loads(json_string) if isinstance(json_string, str) else json_string
        shape = data["shape"] if isinstance(data["shape"], (list, tuple)) else [data["shape"]]
        t = cls(shape, prior_var=data.get("prior_var"))
        t.use_info, t.acuity_cutoff, t.use_kl = data["use_info"], data["acuity_cutoff"], data["use_kl"]
        t.alpha = data.get("alpha", 1e-8)

        def mk(d):
            n = Node(t.dim)
            n.count = F32(d["count"])
            n.mean = np.asarray(d["mean"], F32)
            n.meanSq = np.asarray(d["meanSq"], F32)
            n.sentence_id = list(d.get("sentence_id") or [])
            return n

        t.root = mk(data["root"])
        queue = [(t.root, c) for c in data["root"]["children"]]
        while queue:
            parent, cd = queue.pop()
            n = mk(cd)
            n.parent = parent
            parent.children.append(n)
            queue.extend((n, c) for c in cd["children"])
        return t

    @classmethod
    def from_arrays(cls, parent, count, mean, meanSq, sid_ptr, sid_list, prior_var=None):
        """BFS-ordered node arrays -> tree (children in BFS order)."""
        t = cls((mean.shape[1],), prior_var)
        nodes = []
        for i in range(len(parent)):
            n = Node(t.dim)
            n.count = F32(count[i])
            n.mean = np.asarray(mean[i], F32)
            n.meanSq = np.asarray(meanSq[i], F32)
            n.sentence_id = [int(s) for s in sid_list[sid_ptr[i]:sid_ptr[i + 1]]]
            if parent[i] >= 0:
                n.parent = nodes[parent[i]]
                n.parent.children.append(n)
            nodes.append(n)
        t.root = nodes[0]
        return t

    # ---- binary format (F2): BFS node arrays in one .npz, no pickles ----
    BINARY_VERSION = 1

    def to_arrays(self):
        """BFS node arrays (children in list order): parent [Nn] int64, count [Nn] f32,
        mean/meanSq [Nn, D] f32, sid_ptr [Nn+1] int64, sid_list int64."""
        nodes, parent = [], []
        q = deque([(self.root, -1)])
        while q:
            n, p = q.popleft()
            idx = len(nodes)
            nodes.append(n)
            parent.append(p)
            q.extend((c, idx) for c in n.children)
        Nn = len(nodes)
        count = np.empty(Nn, F32)
        mean = np.empty((Nn, self.dim), F32)
        meanSq = np.empty((Nn, self.dim), F32)
        sid_ptr = np.zeros(Nn + 1, np.int64)
        sids = []
        for i, n in enumerate(nodes):
            count[i], mean[i], meanSq[i] = n.count, n.mean, n.meanSq
            sids.extend(int(s) for s in (n.sentence_id or []))
            sid_ptr[i + 1] = len(sids)
        return {"parent": np.asarray(parent, np.int64), "count": count, "mean": mean, "meanSq": meanSq,
                "sid_ptr": sid_ptr, "sid_list": np.asarray(sids, np.int64)}

    def save_binary(self, path, extra=None):
        """Write the tree as BFS arrays + header to an .npz (loadable with
        allow_pickle=False).  The reference's JSON (dump_json) is ~25x larger and
        needs a Python node object per concept to read back."""
        arrs = self.to_arrays()
        head = {"version": self.BINARY_VERSION, "shape": list(self.shape), "prior_var": float(self.prior_var),
                "use_info": self.use_info, "acuity_cutoff": self.acuity_cutoff, "use_kl": self.use_kl,
                "alpha": self.alpha}
        arrs["header"] = np.frombuffer(json.dumps(head).encode(), np.uint8)
        for k, v in (extra or {}).items():
            arrs[k] = v
        with open(path, "wb") as f:
            np.savez(f, **arrs)

    @staticmethod
    def read_binary(path):
        """(header dict, arrays dict) of a save_binary file."""
        with np.load(path, allow_pickle=False) as z:
            arrs = {k: z[k] for k in z.files}
        head = json.loads(bytes(arrs.pop("header")).decode())
        if head.get("version") != CobwebTree.BINARY_VERSION:
            raise ValueError(f"unsupported tree binary version {head.get('version')}")
        return head, arrs

    @classmethod
    def load_binary(cls, path):
        head, a = cls.read_binary(path)
        t = cls.from_arrays(a["parent"], a["count"], a["mean"], a["meanSq"], a["sid_ptr"], a["sid_list"],
                            prior_var=head["prior_var"])
        t.use_info, t.acuity_cutoff, t.use_kl, t.alpha = (head["use_info"], head["acuity_cutoff"], head["use_kl"],
                                                          head["alpha"])
        return t

    @staticmethod
    def arrays_to_index_inputs(head, a, n_sentences=None):
        """Index inputs straight from binary arrays, without node objects (C3+ scale):
        (mean, var, parent, node_of_sentence); var = compute_var, prior_var if empty."""
        pv = F32(head["prior_var"])
        count = a["count"]
        var = np.empty_like(a["meanSq"])
        nz = count > 0
        var[nz] = a["meanSq"][nz] / count[nz, None] + pv
        var[~nz] = pv
        sid_ptr, sid_list = a["sid_ptr"], a["sid_list"]
        n_sent = int(sid_list.max()) + 1 if n_sentences is None and sid_list.size else int(n_sentences or 0)
        node_of_sentence = np.full(n_sent, -1, np.int64)
        owner = np.repeat(np.arange(len(count), dtype=np.int64), np.diff(sid_ptr))
        keep = sid_list < n_sent
        node_of_sentence[sid_list[keep]] = owner[keep]
        return a["mean"], var, a["parent"], node_of_sentence

    # ---- flattening (CobwebWrapper.build_prediction_index :107-203) ----
    def flatten(self, n_sentences):
        """BFS order (children in list order).  Returns (nodes, parent, mean, var,
        node_of_sentence, max_depth); var = compute_var, prior_var for empty nodes."""
        nodes, parent, depth = [], [], []
        q = deque([(self.root, -1, 0)])
        while q:
            n, p, d = q.popleft()
            idx = len(nodes)
            nodes.append(n)
            parent.append(p)
            depth.append(d)
            q.extend((c, idx, d + 1) for c in n.children)
        Nn = len(nodes)
        mean = np.empty((Nn, self.dim), F32)
        var = np.empty((Nn, self.dim), F32)
        node_of_sentence = np.full(n_sentences, -1, np.int64)
        max_depth = 0
        for i, n in enumerate(nodes):
            mean[i] = n.mean
            var[i] = self.compute_var(n.meanSq, n.count) if n.count > 0 else self.prior_var
            for s in n.sentence_id or []:
                if s < n_sentences:
                    node_of_sentence[s] = i
                    max_depth = max(max_depth, depth[i] + 1)
        return nodes, np.asarray(parent, np.int64), mean, var, node_of_sentence, max_depth
