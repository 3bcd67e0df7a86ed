"""Device ifit under short spin bounds (CWQ_FIT_SPIN_MS): builds small trees with the
chip-wide fit and the one-workgroup loop, prints timings, whether they agree, and the
kernel's progress words when a join times out.  GPU only.
    CWQ_FIT_SPIN_MS=3000 python scripts/fit_debug.py
"""
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def arrays(root):
    out, q, h = [], [root], 0
    while h < len(q):
        x = q[h]
        h += 1
        out.append(x)
        q.extend(x.children)
    pos = {id(x): i for i, x in enumerate(out)}
    return [-1 if x.parent is None else pos[id(x.parent)] for x in out], np.stack([x.mean for x in out])


def build(pkg, X, helpers, fork_min):
    if helpers is None:
        os.environ.pop("CWQ_FIT_HELPERS", None)
    else:
        os.environ["CWQ_FIT_HELPERS"] = str(helpers)
    os.environ["CWQ_FIT_FORK_MIN"] = str(fork_min)
    os.environ["CWQ_FIT_DEVICE"] = "1"
    random.seed(3)
    t0 = time.perf_counter()
    import importlib
    fitmod = importlib.import_module(pkg.__name__ + ".fit")
    tree = pkg.CobwebTree((X.shape[1],))
    f = fitmod.DeviceTreeFitter(tree, device=torch.device("cuda", 0))
    f.fit_batch(X)
    torch.cuda.synchronize()
    return tree, time.perf_counter() - t0, f.stats, random.random()


def main():
    pkg = cobweb_pkg.load()
    rng = np.random.default_rng(1)
    cases = [(64, 300, 64, 1), (64, 300, 64, None), (64, 600, 64, None), (384, 400, 256, None)]
    if len(sys.argv) > 1:   # D,n,fork_min,helpers (helpers -1: the default)
        v = [int(t) for t in sys.argv[1].split(",")]
        cases = [(v[0], v[1], v[2], None if v[3] < 0 else v[3])]
    for D, n, fork_min, helpers in cases:
        X = rng.standard_normal((n, D)).astype(np.float32)
        ref = build(pkg, X, 0, fork_min)
        print(f"D={D} n={n} one workgroup: {ref[1]:.3f} s, stats {ref[2]}", flush=True)
        try:
            got = build(pkg, X, helpers, fork_min)
        except Exception as e:   # noqa: BLE001
            print(f"  helpers={helpers} fork_min={fork_min}: FAILED {e}", flush=True)
            continue
        pa, ma = arrays(ref[0].root)
        pb, mb = arrays(got[0].root)
        same = pa == pb and np.array_equal(ma, mb) and ref[3] == got[3]
        print(f"  helpers={helpers} fork_min={fork_min}: {got[1]:.3f} s, stats {got[2]}, same tree {same}", flush=True)


if __name__ == "__main__":
    main()
