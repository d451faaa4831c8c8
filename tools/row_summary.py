"""Summarise tools/row_profile.sh output: per row, the kernels of one call
(from the kernel trace, after the generation gap), their mean durations, and
the PMC counters per call with the HBM traffic (FETCH_SIZE x 2 on gfx950 for
16-byte streaming reads, WRITE_SIZE; KiB -> bytes) against the row's
algorithmic bytes (printed by row_prof.py). Writes <dir>/rows_summary.json.

    python tools/row_summary.py <dir> ROW [ROW ...]
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

CALLS = 7   # tools/row_prof.py: 2 warm-up + 5 timed calls
# algorithmic bytes per candle: printed by tools/row_prof.py (the inputs the
# row reads once + every output it returns written once at its dtype)
SHAPE = re.compile(r"(\d+)x(\d+) ms/call ([0-9.]+)(?: alg_bpc ([0-9.]+))?")


def trace_kernels(d):
    f = glob.glob(f"{d}/trace/**/*kernel_trace.csv", recursive=True)
    if not f:
        return {}, None
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in rows]
    gaps = [(starts[i + 1] - starts[i], i + 1) for i in range(len(starts) - 1)]
    first = max(gaps)[1] if gaps else 0
    k = defaultdict(list)
    for r in rows[first:]:
        k[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {n: {"calls": len(v), "mean_us": sum(v) / len(v) / 1e3, "per_call_us": sum(v) / CALLS / 1e3}
            for n, v in k.items()}, None


def pmc(d):
    agg = defaultdict(float)
    per_kernel = defaultdict(lambda: defaultdict(float))
    for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            v = float(r["Counter_Value"])
            agg[r["Counter_Name"]] += v
            per_kernel[r["Kernel_Name"]][r["Counter_Name"]] += v
    per_call = {c: v / CALLS for c, v in agg.items()}
    return per_call, {k: {c: v / CALLS for c, v in cs.items()} for k, cs in per_kernel.items()}


def main():
    out_dir, rows = sys.argv[1], sys.argv[2:]
    summary = {}
    for row in rows:
        d = f"{out_dir}/{row}"
        m = None
        try:
            m = SHAPE.search(open(f"{d}/trace.log").read())
        except OSError:
            pass
        S, T, ms = (int(m.group(1)), int(m.group(2)), float(m.group(3))) if m else (None, None, None)
        bpc = float(m.group(4)) if m and m.group(4) else 0.0
        kern, _ = trace_kernels(d)
        cnt, cnt_k = pmc(d)
        fetch = cnt.get("FETCH_SIZE", 0.0) * 1024 * 2
        write = cnt.get("WRITE_SIZE", 0.0) * 1024
        alg = bpc * S * T if S else None
        dev_us = sum(k["per_call_us"] for k in kern.values())
        s = {
            "shape": [S, T], "ms_per_call_hip_events": ms, "kernel_us_per_call": dev_us,
            "algorithmic_bytes_per_candle": bpc, "algorithmic_bytes": alg,
            "traffic_bytes": fetch + write, "fetch_bytes_x2": fetch, "write_bytes": write,
            "traffic_over_algorithmic": (fetch + write) / alg if alg else None,
            "achieved_GBps_alg": alg / (ms * 1e-3) / 1e9 if alg and ms else None,
            "frac_of_8TBps": alg / (ms * 1e-3) / 8e12 if alg and ms else None,
            "valu_busy": (cnt.get("SQ_ACTIVE_INST_VALU", 0) / cnt["SQ_WAVE_CYCLES"]) if cnt.get("SQ_WAVE_CYCLES") else None,
            "wait_share": (cnt.get("SQ_WAIT_ANY", 0) / cnt["SQ_WAVE_CYCLES"]) if cnt.get("SQ_WAVE_CYCLES") else None,
            "kernels": kern, "counters_per_call": cnt,
            "counters_per_call_by_kernel": cnt_k,
        }
        summary[row] = s
        print(f"{row:22s} {S}x{T} {ms if ms else float('nan'):8.3f} ms  alg {bpc:6.1f} B/c  "
              f"frac {s['frac_of_8TBps'] or 0:.3f}  traffic/alg {s['traffic_over_algorithmic'] or 0:.2f}  "
              f"valu {s['valu_busy'] or 0:.2f} wait {s['wait_share'] or 0:.2f}")
        for n, k in sorted(kern.items(), key=lambda x: -x[1]["per_call_us"])[:6]:
            print(f"    {k['per_call_us']:9.1f} us/call  {k['calls']:3d}x {k['mean_us']:9.1f} us  {n[:90]}")
    json.dump(summary, open(f"{out_dir}/rows_summary.json", "w"), indent=1)


if __name__ == "__main__":
    main()
