"""Summarise rocprofv3 PMC passes for one hot kernel into profiles/ (JSON).

    python scripts/pmc_summary.py gpurun_out/pmc profiles/pmc_r01_fgemm.json [kernel-substring]

Counters are summed over the filter launches of one score_topk call (fgemm_kernel<0>
dispatches come in groups of PHASES per call; the threshold-sample pass is the
separate instantiation fgemm_kernel<1>) and averaged over calls.  FETCH_SIZE is the L2 memory-side read
volume in KB; on gfx950 it reports half the bytes of 16-B-per-lane streaming reads
(global_load and global_load_lds alike, MI355X_MICROARCH.md §HBM), so bytes =
2 * 1024 * FETCH_SIZE; Infinity-Cache hits are counted too.  GRBM_GUI_ACTIVE / 8
XCDs / duration = effective clock."""
import collections
import csv
import glob
import json
import os
import sys

pmc_dir, out = sys.argv[1:3]
HOT = sys.argv[3] if len(sys.argv) > 3 else "fgemm_kernel<0>"
PHASES = int(os.environ.get("PMC_PHASES", "3"))
agg, durs = collections.defaultdict(list), []
for d in sorted(glob.glob(os.path.join(pmc_dir, "p*"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    alt = HOT.replace("<0>", "ILi0E").replace("<1>", "ILi1E")   # mangled form in some traces
    rows = [r for r in csv.DictReader(open(f)) if HOT in r["Kernel_Name"] or alt in r["Kernel_Name"]]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in rows:
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    ids = sorted(per)
    G = PHASES
    for c0 in range(0, len(ids) - G + 1, G):
        grp = ids[c0:c0 + G]
        tot = collections.defaultdict(float)
        for did in grp:
            for k, v in per[did].items():
                tot[k] += v
        for k, v in tot.items():
            agg[k].append(v)
        durs.append(sum(dur[did] for did in grp))
c = {k: sum(v) / len(v) for k, v in agg.items()}
dur_ms = sorted(durs)[len(durs) // 2] if durs else None
res = {"kernel": HOT, "filter_launches_per_call": PHASES, "median_call_fgemm_ms_profiled": dur_ms, "counters": c}
if dur_ms and "GRBM_GUI_ACTIVE" in c:
    clk = c["GRBM_GUI_ACTIVE"] / 8 / (dur_ms / 1e3)
    res["effective_clock_ghz"] = round(clk / 1e9, 3)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        # cycles summed over SIMDs (1024 SIMDs)
        res["mfma_pipe_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * clk * dur_ms / 1e3), 3)
if "SQ_WAVE_CYCLES" in c:
    w = c["SQ_WAVE_CYCLES"]
    res["wave_cycle_split"] = {k: round(c.get(n, 0) / w, 3) for k, n in
                               [("waiting_on_data", "SQ_WAIT_ANY"), ("issue_stalled", "SQ_WAIT_INST_ANY"),
                                ("issuing", "SQ_ACTIVE_INST_ANY")]}
if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"]:
    res["lds_bank_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
if "TCC_HIT_sum" in c:
    res["l2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 3)
if "FETCH_SIZE" in c:
    # summed over the PHASES filter launches of one call (one bench step), not one launch
    res["fetch_bytes_per_call"] = 2 * c["FETCH_SIZE"] * 1024          # gfx950 16-B-lane correction
    res["hbm_bytes_per_call"] = res["fetch_bytes_per_call"]           # upper bound: MALL hits counted
    res["hbm_bytes_per_launch"] = res["fetch_bytes_per_call"] / PHASES
if "WRITE_SIZE" in c:
    res["write_bytes_per_call"] = c["WRITE_SIZE"] * 1024
res["workload"] = [1000000, 768, 10000, 10]   # filter_probe defaults the passes ran
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "counters"}))
