"""A/B the hot scan configurations (CWQ_SCAN_CFG) in ONE process on the C3
workload (1M x 768 flat tree, 10k queries, k=10), interleaved rounds; checks
that every configuration returns identical ids/scores."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import cobweb_pkg  # noqa: E402

pkg = cobweb_pkg.load()
N, D, Q, k = (int(v) for v in (sys.argv[1:5] if len(sys.argv) >= 5 else (1_000_000, 768, 10_000, 10)))
# variants: "scan_cfg[:xcd_map]" (CWQ_SCAN_CFG, CWQ_XCD_MAP)
cfgs = sys.argv[5].split(",") if len(sys.argv) > 5 else ["0:1", "0:0", "1:1", "3:1"]
X = pkg.synth.synthetic_corpus(N, D, seed=0)
t = pkg.synth.flat_synth(X)
ix = pkg.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"])
del t
Qs, _ = pkg.synth.synthetic_queries(X, Q, seed=1)
ix.set_timing(True)
res, ref = {c: [] for c in cfgs}, None
for rnd in range(3):
    for c in cfgs:
        sc_, _, xm = c.partition(":")
        os.environ["CWQ_SCAN_CFG"] = sc_
        os.environ["CWQ_XCD_MAP"] = xm or "1"
        ids, sc = ix.score_topk(Qs, k)
        tm = ix.last_timing()
        res[c].append(tm["leaf_scan_ms"])
        if ref is None:
            ref = (ids.cpu(), sc.cpu())
        else:
            assert torch.equal(ids.cpu(), ref[0]), f"cfg {c} ids differ"
            assert torch.equal(sc.cpu(), ref[1]), f"cfg {c} scores differ"
out = {}
for c in cfgs:
    ms = float(np.median(res[c]))
    out[c] = {"scan_ms_median": round(ms, 2), "scan_ms_min": round(min(res[c]), 2),
              "qps": round(Q / (ms / 1e3), 1), "valu_frac": round(2 * N * D * Q / (ms / 1e3) / 78.64e12, 3)}
print(json.dumps({"workload": [N, D, Q, k], "configs": out}))
