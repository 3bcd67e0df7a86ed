"""Summarise rocprofv3 output for the hot kernel into profiles/ (JSON).

    python scripts/pmc_summary.py gpurun_out/pmc gpurun_out/prof profiles/pmc_r01.json
Counters are per dispatch of scan_kernel<ISO,TOPK> (the leaf scan).  FETCH_SIZE
is the L2 memory-side read volume (KB; Infinity-Cache hits included, see
MI355X_MICROARCH.md §HBM); GRBM_GUI_ACTIVE / 8 XCDs / duration = effective clock."""
import collections
import csv
import glob
import json
import os
import sys

pmc_dir, prof_dir, out = sys.argv[1:4]
HOT = "scan_kernel<true, 2"
agg, durs = collections.defaultdict(list), []
for d in sorted(glob.glob(os.path.join(pmc_dir, "p*"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if HOT in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for disp in per.values():
        for k, v in disp.items():
            agg[k].append(v)
c = {k: sum(v) / len(v) for k, v in agg.items()}
dur_ms = sorted(durs)[len(durs) // 2] if durs else None
res = {"kernel": "scan_kernel<ISO,TOPK,fast> (leaf scan)", "median_dispatch_ms": dur_ms, "counters": c}
if dur_ms and "GRBM_GUI_ACTIVE" in c:
    clk = c["GRBM_GUI_ACTIVE"] / 8 / (dur_ms / 1e3)
    res["effective_clock_ghz"] = round(clk / 1e9, 3)
    if "SQ_INSTS_VALU" in c:
        res["valu_pipe_busy"] = round(c["SQ_INSTS_VALU"] * 2 / (1024 * clk * dur_ms / 1e3), 3)
if "SQ_WAVE_CYCLES" in c:
    w = c["SQ_WAVE_CYCLES"]
    res["wave_cycle_split"] = {k: round(c.get(n, 0) / w, 3) for k, n in
                               [("waiting_on_data", "SQ_WAIT_ANY"), ("issue_stalled", "SQ_WAIT_INST_ANY"),
                                ("issuing", "SQ_ACTIVE_INST_ANY")]}
if "TCC_HIT_sum" in c:
    res["l2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 3)
if "FETCH_SIZE" in c:
    res["fetch_bytes_per_launch"] = c["FETCH_SIZE"] * 1024
    res["hbm_bytes_per_launch"] = c["FETCH_SIZE"] * 1024   # upper bound: MALL hits are counted too
kstats = os.path.join(prof_dir, "run_kernel_stats.csv")
if os.path.exists(kstats):
    res["kernel_stats_top"] = [{"name": r["Name"][:100], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                "pct": float(r["Percentage"])} for r in list(csv.DictReader(open(kstats)))[:8]]
res["workload"] = [1000000, 768, 10000, 10]   # bench.py defaults the passes ran
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k not in ("counters", "kernel_stats_top")}))
