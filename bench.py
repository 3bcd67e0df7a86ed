"""Benchmark: "Cobweb Fast" batched queries/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2]): synthetic flat-synth tree
over X ~ N(0, I), N = 1,000,000 x D = 768 fp32 (seed 0), 10,000 queries per step per
GPU (half corpus points + 0.1*N(0,I), half fresh N(0,I); seed 1 + rank), k = 10.
A step = one libcwq cwq_score_topk call over the batch (scan + path score + top-k
+ merge + sentence ids), inputs resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Multi-GPU: rank 0 synthesises the tree and broadcasts the frozen node statistics
over RCCL (one torch.distributed broadcast per array, timed separately); every rank
then scans its own 10k-query batch (weak scaling, no collective in the timed loop).
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import cobweb_pkg  # noqa: E402

PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA dense peak
PEAK_BF16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA dense peak (no sparsity)
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def config_label(N, D):
    """Which BASELINE.json config a run measures (SURVEY §8 shorthand)."""
    if (N, D) == (1_000_000, 768):
        return "BASELINE configs[2], C3"
    if (N, D) == (10_000_000, 1024):
        return "BASELINE configs[3], C4 per-GPU shard"
    return "custom size"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(X_host, root_mean, root_var, Q_host, k, sample, ids_gpu):
    """The oracle (numpy fp32 restatement of CobwebWrapper.cobweb_predict_indexed,
    oracle/cobweb_oracle.py) timed on this host, one query per call like the
    reference harness (benchmark_utils.py:801-805).  Checker only: its results are
    compared with the GPU ids for the sampled queries."""
    from oracle import cobweb_oracle as O
    N, D = X_host.shape
    means = np.concatenate([root_mean[None, :], X_host])
    vars_ = np.empty_like(means)
    vars_[0] = root_var
    vars_[1:] = O.PRIOR_VAR
    idx = O.FlatIndex(means, vars_, np.r_[-1, np.zeros(N, np.int64)], [], list(O.DEFAULT_LEVEL_WEIGHTS))
    nodes = np.stack([np.zeros(N, np.int64), np.arange(1, N + 1)], 1)
    coef = np.full((N, 2), O.path_weight(0, 2, idx.weights), np.float32)
    times, agree = [], 0
    for i in range(sample):
        t = time.perf_counter()
        got = O.predict_indexed_vec(Q_host[i], idx, k, (nodes, coef))
        times.append(time.perf_counter() - t)
        agree += int(list(got) == list(ids_gpu[i]))
    sec = float(np.mean(times))
    return {"value": round(1.0 / sec, 4), "unit": "queries/s", "cores": 1, "kind": "port",
            "sample": f"{sample} queries x full {N}x{D} flat tree, one query per call "
                      f"({sec:.2f} s/query; numpy fp32 oracle, single thread; CPU: {cpu_model()}); "
                      f"GPU top-{k} identical on {agree}/{sample}",
            "s_per_query": round(sec, 3)}


def recall_at_k(pkg, X, Q, ids, targets, k, n_eval):
    """recall@k of the Fast ranking vs exact brute force (flat-L2 and flat-IP =
    the reference's FAISS / Torch Dot baselines, benchmark_utils.py:536-614), scored in
    float64 (harness.brute_force_topk(exact=True))."""
    Qe = Q[:n_eval]
    gt_l2 = pkg.harness.brute_force_topk(X, Qe, k, "l2", exact=True).cpu().numpy()
    gt_ip = pkg.harness.brute_force_topk(X, Qe, k, "ip", exact=True).cpu().numpy()
    got = ids[:n_eval].cpu().numpy()
    r_l2 = np.mean([len(set(a) & set(b)) / k for a, b in zip(got, gt_l2)])
    r_ip = np.mean([len(set(a) & set(b)) / k for a, b in zip(got, gt_ip)])
    tg = targets.cpu().numpy()
    r_tgt = float(np.mean([t in set(row) for t, row in zip(tg, ids[:len(tg)].cpu().numpy())])) if len(tg) else None
    return round(float(r_l2), 4), round(float(r_ip), 4), r_tgt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--queries", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--cpu-sample", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--recall-queries", type=int, default=512)
    ap.add_argument("--pmc-file", default=os.path.join(ROOT, "profiles", "pmc_r01_fgemm.json"))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    pkg = cobweb_pkg.load()
    pkg.lib()
    N, D, Qn, k = args.n, args.dim, args.queries, args.k

    # ---- tree: synthesised on rank 0, node statistics broadcast over RCCL ----
    t0 = time.perf_counter()
    if rank == 0:
        X = pkg.synth.synthetic_corpus(N, D, seed=0, device=dev)
        tree = pkg.synth.flat_synth(X)
        mean, var = tree["mean"], tree["var"]
        root_cnt, root_mu, root_m2 = tree["root"]
        del tree, X
    else:
        mean = torch.empty((N + 1, D), dtype=torch.float32, device=dev)
        var = torch.empty((N + 1, D), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    t_synth = time.perf_counter() - t0
    t_bcast = 0.0
    if world > 1:
        dist.barrier()
        t1 = time.perf_counter()
        dist.broadcast(mean, 0)
        dist.broadcast(var, 0)
        torch.cuda.synchronize()
        t_bcast = time.perf_counter() - t1
    parent = np.zeros(N + 1, np.int64)
    parent[0] = -1
    nos = np.arange(1, N + 1, dtype=np.int64)
    t1 = time.perf_counter()
    index = pkg.index.CobwebIndex(mean, var, parent, nos, device=dev)
    torch.cuda.synchronize()
    t_index = time.perf_counter() - t1
    X = mean[1:]                          # leaf means are the corpus rows
    Q, targets = pkg.synth.synthetic_queries(X, Qn, seed=1 + rank)
    root_var_host = var[0].cpu().numpy() if rank == 0 else None
    del var
    torch.cuda.empty_cache()

    # ---- timed loop ----
    for _ in range(args.warmup):
        index.score_topk(Q, k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ids, scores = index.score_topk(Q, k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    qps = world * Qn * args.steps / dt

    # ---- dominant kernel timing (HIP events on the launch stream) ----
    st = index.last_stats()
    index.set_timing(True)
    tms = []
    for _ in range(3):
        index.score_topk(Q, k)
        tms.append(index.last_timing())
    index.set_timing(False)
    call_ms = float(np.mean([t["call_ms"] for t in tms]))
    NL = index.info["leaf_rows"]
    if st["filter_used"]:
        # bf16-MFMA candidate filter (cwq_mfma.hip fgemm): 2*D flops per (query, leaf row)
        kern_ms = float(np.mean([t["fgemm_ms"] for t in tms]))
        flops_launch = 2.0 * D * NL * Qn
        peak, kname, pipe = PEAK_BF16_TFLOPS, "fgemm_kernel<0> (bf16 MFMA filter pass)", "bf16 MFMA dense"
        launches = max(1, round(float(np.mean([t["leaf_scan_launches"] for t in tms]))))   # filter phases
        phases = {"sample_ms": round(float(np.mean([t["sample_ms"] for t in tms])), 3),
                  "fgemm_ms": round(kern_ms, 3),
                  "rerank_ms": round(float(np.mean([t["rerank_ms"] for t in tms])), 3)}
    else:
        kern_ms = float(np.mean([t["leaf_scan_ms"] / max(1, t["leaf_scan_launches"]) for t in tms]))
        flops_launch = 4.0 * D * NL * Qn                  # 4*Nn*D per query (leaf rows)
        peak, kname, pipe = PEAK_FP32_TFLOPS, "scan_kernel<ISO,TOPK> (exact fp32 leaf scan)", "fp32 VALU"
        phases = {}
        launches = 1
    achieved_tf = flops_launch / (kern_ms * 1e-3) / 1e12
    bytes_q = 8.0 * (N + 1) * D + 8.0 * 2 * N + 4.0 * D + 12.0 * k   # SURVEY §8(d) bytes per query
    traffic = None
    if os.path.exists(args.pmc_file):
        try:
            pm = json.load(open(args.pmc_file))
            if pm.get("workload") == [N, D, Qn, k] and pm.get("kernel") == kname.split(" ")[0]:
                # per step (the launches of one call), like `achieved`
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    rec_l2 = rec_ip = rec_tgt = None
    if rank == 0 and args.recall_queries > 0:
        rec_l2, rec_ip, rec_tgt = recall_at_k(pkg, X, Q, ids, targets, k, min(args.recall_queries, Qn))

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        Xh = X.cpu().numpy()
        log(f"cpu baseline: {args.cpu_sample} queries on the full tree ...")
        base = cpu_baseline(Xh, root_mu[0].cpu().numpy(), root_var_host, Q[:args.cpu_sample].cpu().numpy(), k,
                            args.cpu_sample, ids[:args.cpu_sample].cpu().numpy())
        del Xh

    if rank == 0:
        out = {
            "metric": "queries/sec + recall@10 vs FAISS-flat, 1M×768 corpus, 1/2/4/8 MI355X",
            "value": round(qps, 1), "unit": "queries/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * dt / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"Cobweb Fast top-{k}: synthetic flat-synth tree (root + {N} leaves), "
                                   f"X~N(0,I) {N}x{D} fp32, {Qn} queries/step/GPU ({config_label(N, D)})",
                       "corpus": N, "dim": D, "queries_per_gpu": Qn, "k": k, "tree": "flat-synth",
                       "parallelism": f"query-shard x{world}, index broadcast over RCCL" if world > 1
                       else "single GPU"},
            "roofline": {"bound": "mfma", "pipe": pipe,
                         "achieved": round(achieved_tf, 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(achieved_tf / peak, 4), "traffic": traffic,
                         "kernel": kname, "kernel_ms": round(kern_ms, 3), "launches_per_step": launches,
                         "avg_launch_ms": round(kern_ms / launches, 3),
                         "call_ms": round(call_ms, 3), "flops_per_step": flops_launch, "phases_ms": phases},
            "filter": {k_: st[k_] for k_ in ("filter_used", "fallback_queries", "candidates", "exact_reranks",
                                              "sample_rows")},
            "hbm_roofline": {"bytes_per_query": bytes_q,
                             "per_query_roof_qps": round(PEAK_HBM_GBS * 1e9 / bytes_q, 1),
                             "frac": round(qps / world * bytes_q / (PEAK_HBM_GBS * 1e9), 3)},
            "recall@10": {"vs_flat_l2": rec_l2, "vs_flat_ip": rec_ip, "target_in_top10": rec_tgt,
                          "n_queries": min(args.recall_queries, Qn)},
            "cpu_baseline": base,
            "setup_s": {"synth": round(t_synth, 3), "rccl_broadcast": round(t_bcast, 3),
                        "index_build": round(t_index, 3)},
        }
        print(json.dumps(out), flush=True)
    index.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
