"""Host/GPU timeline of the last N per-call iterations from a rocprofv3 csv run with
--hip-runtime-trace --kernel-trace: every HIP API call (host) and kernel (device) on one
clock, so the host gap between calls can be split into its API calls.

    python scripts/api_timeline.py gpurun_out/api/run [--last 3]
"""
import argparse
import csv
import glob


def rows(pattern):
    out = []
    for f in glob.glob(pattern):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--last", type=int, default=3)
    a = ap.parse_args()
    ev = []
    for r in rows(a.prefix + "*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "GPU", r["Kernel_Name"][:60]))
    for r in rows(a.prefix + "*hip_api_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "API", r["Function"][:60]))
    ev.sort()
    starts = [i for i, e in enumerate(ev) if e[2] == "GPU" and ("sb_prep" in e[3] or "stream_kernel<1" in e[3])]
    if len(starts) < a.last + 1:
        print("not enough calls", len(starts))
        return
    i0 = starts[-a.last - 1]
    t0 = ev[i0][0]
    sel = ev[i0:]
    for j, (s, e, kind, name) in enumerate(sel):
        # a polling loop (hipStreamQuery) prints as its first and last call only
        poll = name == "hipStreamQuery"
        if poll and 0 < j < len(sel) - 1 and sel[j - 1][3] == name and sel[j + 1][3] == name:
            continue
        print(f"{(s - t0) / 1e3:10.1f} us  {kind}  dur {(e - s) / 1e3:8.1f}  {name}")


if __name__ == "__main__":
    main()
