"""Config C2 (100k x 768, 1k queries, one MI355X) end to end on a tree built by the
drop-in's own device ifit -- the reference's workflow: CobwebWrapper(corpus, embeddings)
(CobwebWrapper.py:13-80) -> build_prediction_index -> queries (benchmark_utils.py:576-581,
801-805).  Same corpus as tests/test_gpu_c2.py (100 Gaussian clusters).  Reports:
  ifit seconds and tree shape; index build seconds;
  Fast batch q/s (filter and exact scan), phases;
  Fast one query per call: score_topk on a device tensor, and the harness's own call
  cobweb_predict_fast(numpy_query, k) (H2D copy, sync, id -> sentence mapping);
  Basic batch q/s with found-k and how the queries resolved; Basic one query per call.
GPU only.   python scripts/c2_probe.py [--n 100000]
"""
import argparse
import os
import random
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402


def med(f, reps):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--clusters", type=int, default=100)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--calls", type=int, default=300, help="one-query calls timed per leg")
    ap.add_argument("--basic-only", action="store_true", help="only the Basic legs (e.g. under rocprofv3)")
    ap.add_argument("--fast-only", action="store_true", help="only the Fast legs")
    ap.add_argument("--ab-prune", action="store_true",
                    help="run the Fast legs with group pruning off (CWQ_GROUP_PRUNE=0) and on, in one process")
    ap.add_argument("--legs", default="all",
                    help="list (comma or +) of fbatch,fpc1,fpc8,fpc64,fphase,fharness,bbatch,bpc (default all)")
    ap.add_argument("--chunk", type=int, default=0, help="device ifit in add_sentences calls of this many rows")
    ap.add_argument("--env-ab", default=None,
                    help="';'-separated variants of '&'-separated KEY=VAL (read per call): the legs named in --legs "
                         "(fpc: Fast nq = 1, 64; bbatch: Basic batch, checked == the first variant; bpc: "
                         "Basic per call) under each, interleaved over 3 rounds, after the other legs")
    ap.add_argument("--save-struct", default=None,
                    help="write the ifit tree's structure (BFS parent, node of each row) to this .npz")
    ap.add_argument("--load-struct", default=None,
                    help="skip ifit: the tree structure from a --save-struct file, node statistics by batch "
                         "Welford over the same corpus (synth.tree_synth) -- the same shape for the query legs")
    ap.add_argument("--save-load", default=None,
                    help="round-trip the ifit tree (full stats: count / mean / meanSq) through the F2 .npz "
                         "(CobwebWrapper.save_binary / load_binary) at this path, check the loaded stats equal "
                         "the ifit's bit for bit, and run the query legs on the loaded wrapper")
    ap.add_argument("--index-env", default=None,
                    help="';'-separated variants of '&'-separated KEY=VAL set at index creation (e.g. "
                         "'CWQ_GROUP_CUT=1;' = the depth-1 cut, then the default): the index is rebuilt from "
                         "the same fitted tree under each and the query legs rerun")
    ap.add_argument("--stamps", action="store_true",
                    help="diagnostic builds (CWQ_LIB=a -DCWQ_STAMP=1 variant): after the Basic per-call leg, "
                         "final_wide phase stamps and simulate_two cycle counts of a few one-query calls")
    args = ap.parse_args()
    pkg = cobweb_pkg.load()
    X, Qn, pick = pkg.synth.clustered_corpus(args.n, args.dim, args.clusters, args.nq)
    random.seed(2)
    w0 = pkg.CobwebWrapper(corpus=None, corpus_embeddings=X[:8])   # warm up libcwq
    w0.build_prediction_index()
    torch.cuda.synchronize()
    random.seed(2)
    t0 = time.perf_counter()
    if args.load_struct:
        z = np.load(args.load_struct)
        t = pkg.synth.tree_synth(torch.from_numpy(X).cuda(), z["parent"], z["node_of_sentence"])
        t_fit = 0.0
        t0 = time.perf_counter()
        ix = pkg.index.CobwebIndex(t["mean"], t["var"], t["parent"], t["node_of_sentence"], [1.0] * 6, device="cuda:0")
        w = pkg.CobwebWrapper.from_index(ix, [f"p{i}" for i in range(args.n)], node_of_sentence=t["node_of_sentence"])
        del t
    elif args.chunk:
        # the same device ifit in add_sentences calls of --chunk rows, progress per chunk (a
        # long build keeps printing; inserts/s against the tree size)
        w = pkg.CobwebWrapper(corpus=None, corpus_embeddings=None)
        for a0 in range(0, args.n, args.chunk):
            a1 = min(args.n, a0 + args.chunk)
            tc = time.perf_counter()
            w.add_sentences([f"p{i}" for i in range(a0, a1)], X[a0:a1])
            torch.cuda.synchronize()
            dt = time.perf_counter() - tc
            print(f"  ifit rows {a0}..{a1}: {(a1 - a0) / dt:.0f} inserts/s ({dt:.1f} s), total "
                  f"{time.perf_counter() - t0:.1f} s", flush=True)
        t_fit = time.perf_counter() - t0
        t0 = time.perf_counter()
        w.build_prediction_index()
    else:
        w = pkg.CobwebWrapper(corpus=[f"p{i}" for i in range(args.n)], corpus_embeddings=X)
        torch.cuda.synchronize()
        t_fit = time.perf_counter() - t0
        t0 = time.perf_counter()
        w.build_prediction_index()
    torch.cuda.synchronize()
    t_ix = time.perf_counter() - t0
    ix = w._index
    if args.save_load and not args.load_struct:
        t0 = time.perf_counter()
        w.save_binary(args.save_load)
        w2 = pkg.CobwebWrapper.load_binary(args.save_load)
        a1, a2 = w.tree.to_arrays(), w2.tree.to_arrays()
        same = all(np.array_equal(a1[key], a2[key]) for key in ("parent", "count", "mean", "meanSq", "sid_ptr", "sid_list"))
        assert same, "loaded tree differs from the ifit tree"
        w2.build_prediction_index()
        torch.cuda.synchronize()
        print(f"tree round trip through {args.save_load}: {os.path.getsize(args.save_load) / 1e6:.0f} MB, "
              f"stats equal to the ifit's: {same} ({time.perf_counter() - t0:.1f} s); the legs run on the loaded tree",
              flush=True)
        os.remove(args.save_load)
        w._invalidate_prediction_index()
        w = w2
        ix = w._index
    if args.save_struct:
        nodes, parent, _, _, nos, _ = w.tree.flatten(args.n)
        np.savez_compressed(args.save_struct, parent=parent.astype(np.int32), node_of_sentence=nos.astype(np.int32))
        print(f"saved the tree structure to {args.save_struct}", flush=True)
    inf = ix.info
    root_c = int((np.load(args.load_struct)['parent'] == 0).sum()) if args.load_struct else len(w.tree.root.children)
    print(f"filter rows: {ix.filter_info()}; cut: {ix.cut_info()}", flush=True)
    print(f"C2 corpus {args.n}x{args.dim} ({args.clusters} clusters): " +
          ("tree structure loaded, batch-Welford stats " if args.load_struct else "") + f"device ifit {t_fit:.2f} s "
          f"({args.n / max(t_fit, 1e-9):.0f} inserts/s); tree {inf['n_nodes']} nodes, {inf['internal_nodes']} internal, "
          f"max depth {inf['max_depth']}, root children {root_c}; index build {t_ix:.2f} s "
          f"({inf['device_bytes'] / 1e9:.2f} GB)", flush=True)
    Q = torch.from_numpy(Qn).cuda()
    k = args.k
    if not args.basic_only:
        if args.ab_prune:
            for mode in ("0", None, "0", None):
                if mode is None:
                    os.environ.pop("CWQ_GROUP_PRUNE", None)
                else:
                    os.environ["CWQ_GROUP_PRUNE"] = mode
                print(f"-- group pruning {'off' if mode else 'on'}", flush=True)
                fast_legs(args, w, ix, Q, Qn, pick, k)
            os.environ.pop("CWQ_GROUP_PRUNE", None)
        else:
            fast_legs(args, w, ix, Q, Qn, pick, k)
    if not args.fast_only:
        basic_legs(args, w, ix, Q, Qn, k)
    if args.env_ab:
        env_ab(args, w, ix, Q, Qn, k)
    if args.index_env is not None and not args.load_struct:
        for v in args.index_env.split(";"):
            env = dict(kv.split("=", 1) for kv in v.split("&") if kv.strip())
            w._invalidate_prediction_index()
            os.environ.update(env)
            t0 = time.perf_counter()
            w.build_prediction_index()
            torch.cuda.synchronize()
            for key in env:
                os.environ.pop(key, None)
            ix = w._index
            print(f"-- index rebuilt under {env or 'default'} ({time.perf_counter() - t0:.2f} s): filter rows "
                  f"{ix.filter_info()}; cut {ix.cut_info()}", flush=True)
            if not args.basic_only:
                fast_legs(args, w, ix, Q, Qn, pick, k)
            if not args.fast_only:
                basic_legs(args, w, ix, Q, Qn, k)
    print("done", flush=True)


def env_ab(args, w, ix, Q, Qn, k):
    variants = []
    for v in args.env_ab.split(";"):
        variants.append(dict(kv.split("=", 1) for kv in v.split("&") if kv.strip()))
    keys = sorted({key for v in variants for key in v})
    ix.set_filter(0)
    ids0, _ = ix.score_topk(Q, k)
    ix.set_filter(-1)
    legs = args.legs.replace("+", ",").split(",")
    ref = ix.categorize(Q, k, w.max_init_search) if "bbatch" in legs else None
    for r in range(3):
        for v in variants:
            for key in keys:
                os.environ.pop(key, None)
            os.environ.update(v)
            print(f"-- round {r} env {v or 'default'}", flush=True)
            if "fpc" in legs or args.legs == "all":
                for nq in (1, 64):
                    fast_percall(args, ix, Q, k, ids0, nq)
            if "bbatch" in legs:
                got = ix.categorize(Q, k, w.max_init_search)
                same = all(torch.equal(a, b) for a, b in zip(ref, got))
                t_b = med(lambda: ix.categorize(Q, k, w.max_init_search), 5)
                print(f"Basic batch nq={args.nq}: {t_b * 1e3:.3f} ms = {args.nq / t_b:.0f} q/s; == first variant "
                      f"{same}; resolved {ix.last_categorize_stats()}; lazy {ix.last_lazy_stats()}", flush=True)
            if "bpc" in legs:
                ts = []
                for i in range(100):
                    t0 = time.perf_counter()
                    w.cobweb_predict(Qn[i % args.nq], k)
                    ts.append(time.perf_counter() - t0)
                ts.sort()
                print(f"Basic per call cobweb_predict(numpy, {k}): median {ts[50] * 1e6:.1f} us; last call lazy "
                      f"{ix.last_lazy_stats()}", flush=True)
    for key in keys:
        os.environ.pop(key, None)


def want(args, leg):
    return args.legs == "all" or leg in args.legs.replace("+", ",").split(",")


def fast_legs(args, w, ix, Q, Qn, pick, k):
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, k)
    ix.set_filter(-1)
    if want(args, "fbatch"):
        fast_batch(args, ix, Q, pick, k, ids0, s0)
    for nq in (1, 8, 64):
        if want(args, f"fpc{nq}"):
            fast_percall(args, ix, Q, k, ids0, nq)
    if want(args, "fphase"):
        fast_phases(ix, Q, k)
    if want(args, "fharness"):
        fast_harness(args, w, Qn, k)


def fast_batch(args, ix, Q, pick, k, ids0, s0):
    ix.set_filter(0)
    ids0, s0 = ix.score_topk(Q, k)
    t_scan = med(lambda: ix.score_topk(Q, k), 5)
    ix.set_filter(-1)
    ids1, s1 = ix.score_topk(Q, k)
    same = torch.equal(ids0, ids1) and torch.equal(s0, s1)
    ix.set_timing(True)
    t_f = med(lambda: ix.score_topk(Q, k), 11)
    tm = ix.last_timing()
    ix.set_timing(False)
    st = ix.last_stats()
    top1 = float((ids1[:len(pick), 0].cpu().numpy() == pick).mean())
    print(f"Fast batch nq={args.nq}: filter {t_f * 1e3:.3f} ms = {args.nq / t_f:.0f} q/s (exact scan "
          f"{t_scan * 1e3:.3f} ms = {args.nq / t_scan:.0f} q/s); ids/scores == exact scan: {same}; "
          f"candidates/query {st['candidates']}, exact reranks {st['exact_reranks']}, "
          f"fallback queries {st['fallback_queries']}; "
          f"perturbed passage ranked first {top1:.3f}", flush=True)
    print(f"  last call phases (HIP events, ms): " + ", ".join(f"{a} {b:.3f}" for a, b in tm.items()), flush=True)
    print(f"  prune stats: {ix.last_prune_stats()}", flush=True)


def fast_percall(args, ix, Q, k, ids0, nq):
    qs = [Q[i:i + nq].contiguous() for i in range(0, min(args.nq, args.calls * nq), nq)][:args.calls]
    ok = all(torch.equal(ix.score_topk(q, k)[0], ids0[i * nq:i * nq + nq]) for i, q in enumerate(qs[:20]))
    ts = []
    for q in qs:
        t0 = time.perf_counter()
        ix.score_topk(q, k)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    st = ix.last_stats()
    print(f"Fast per call nq={nq} (score_topk, device tensor): median {ts[len(ts) // 2] * 1e6:.1f} us, "
          f"p10 {ts[len(ts) // 10] * 1e6:.1f} us; path {st['path']} int8 {st['int8_pass']}; "
          f"== exact {ok}", flush=True)


def fast_phases(ix, Q, k):
    # one query per call: phase times from HIP events (median over 30 calls)
    ix.set_timing(True)
    ph = []
    for i in range(30):
        ix.score_topk(Q[i:i + 1].contiguous(), k)
        ph.append(ix.last_timing())
    ix.set_timing(False)
    print("  per-call phases (HIP events, median ms): " +
          ", ".join(f"{n} {sorted(p[n] for p in ph)[15]:.4f}" for n in ph[0] if n.endswith("_ms")), flush=True)


def fast_harness(args, w, Qn, k):
    ts = []
    for i in range(args.calls):
        t0 = time.perf_counter()
        w.cobweb_predict_fast(Qn[i % args.nq], k)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"Fast per call, the harness's cobweb_predict_fast(numpy, {k}) -> sentences: median "
          f"{ts[len(ts) // 2] * 1e6:.1f} us, p10 {ts[len(ts) // 10] * 1e6:.1f} us", flush=True)


def basic_legs(args, w, ix, Q, Qn, k):
    nodes, found, calls = ix.categorize(Q, k, w.max_init_search)
    if want(args, "bbatch"):
        t_b = med(lambda: ix.categorize(Q, k, w.max_init_search), 5)
        cst = ix.last_categorize_stats()
        print(f"Basic batch nq={args.nq}: {t_b * 1e3:.3f} ms = {args.nq / t_b:.0f} q/s; found-k "
              f"{float((found == k).float().mean()):.3f}; log_prob calls/query mean "
              f"{float(calls.float().mean()):.0f}; resolved {cst}", flush=True)
    if not want(args, "bpc"):
        return
    ok = True
    for i in range(20):   # one-query calls == the batch's rows
        n1, f1, c1 = ix.categorize(Q[i:i + 1].contiguous(), k, w.max_init_search)
        ok &= torch.equal(n1[0], nodes[i]) and int(f1[0]) == int(found[i]) and int(c1[0]) == int(calls[i])
    print(f"Basic one-query calls == batch rows (20 queries): {ok}", flush=True)
    ts = []
    for i in range(min(args.calls, 200)):
        t0 = time.perf_counter()
        w.cobweb_predict(Qn[i % args.nq], k)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"Basic per call cobweb_predict(numpy, {k}): median {ts[len(ts) // 2] * 1e6:.1f} us", flush=True)
    if args.stamps:
        print_stamps(w, Qn, k)


def print_stamps(w, Qn, k):
    import ctypes
    L = ctypes.CDLL(os.environ["CWQ_LIB"])
    fw = (ctypes.c_ulonglong * 4096)()
    two = (ctypes.c_ulonglong * 16)()
    names = ["pop", "load", "push", "rows", "pops", "int_pops", "child_push", "row_push", "total", "pop_select", "max_live_runs"]
    for i in range(5):
        L.cwq_debug_fw_stamp(fw, 4096)   # clears
        w.cobweb_predict(Qn[i], k)
        torch.cuda.synchronize()
        L.cwq_debug_fw_stamp(fw, 4096)
        L.cwq_debug_two_stamp(two, 16)
        blocks = [[fw[b * 16 + p] for p in range(14)] for b in range(256) if fw[b * 16]]
        t0 = min(r[0] for r in blocks)
        rel = lambda v: (v - t0) * 0.01 if v >= t0 else float("nan")
        lines = []
        for b, r in enumerate(blocks):
            lines.append(" ".join(f"{rel(v):7.2f}" for v in r))
        print(f"-- call {i}: final_wide (last launch) {len(blocks)} workgroups, phase stamps us "
              f"(0 entry,1 cands,2 T2,3 surv,4 rounds,5 kw-merge,6 last-arrival,7 split-merge,8 end | 9 T2 pre-load,10 T2 lists,11 T2 staged,12 round-0 partials,13 round-0 chains)", flush=True)
        for ln in lines[:4] + (["..."] if len(lines) > 8 else []) + lines[-4:] if len(lines) > 8 else lines:
            print("   ", ln)
        print("   simulate_two q0 (cycles):", {n: int(two[j]) for j, n in enumerate(names)}, flush=True)
    if hasattr(L, "cwq_debug_lz_stamp"):   # the lazy replay of the direct path, query 0 of one-query calls
        lz = (ctypes.c_ulonglong * 16)()
        lz_names = ["total_cyc", "total_wall", "pop_loop", "inline_children", "score_phase", "deferred_children",
                    "rank_phase", "pops", "int_pops", "jobs", "rows", "arena", "pop_select", "pop_read"]
        os.environ["CWQ_CAT_DIRECT"] = "1"
        for i in range(5):
            w.cobweb_predict(Qn[i], k)
            torch.cuda.synchronize()
            L.cwq_debug_lz_stamp(lz, 16)
            print(f"   lazy replay call {i} (cycles; wall at 100 MHz):", {n: int(lz[j]) for j, n in enumerate(lz_names)},
                  flush=True)
        os.environ.pop("CWQ_CAT_DIRECT", None)


if __name__ == "__main__":
    main()
