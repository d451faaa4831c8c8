"""Summarise tools/shard_pmc.sh: per case (enrich at the 12.5k shard with the
padded / contiguous output pitch, the 100k headline) the enrich_kernel's mean
duration, fraction of 8 TB/s on 152 B/candle, HBM traffic per launch, L2 hit
rate, DRAM credit stalls per launch and SQ wait share.
    python tools/shard_summary.py <dir>"""
import csv
import glob
import json
import sys
from collections import defaultdict

d = sys.argv[1]
out = {}
for case in sorted(glob.glob(f"{d}/*_*/")):
    name = case.rstrip("/").split("/")[-1]
    S = int(name.split("_")[-1])
    ks = glob.glob(f"{case}trace/**/*kernel_stats.csv", recursive=True)
    dur = None
    for f in ks:
        for r in csv.DictReader(open(f)):
            if "enrich_kernel" in r["Name"]:
                dur = float(r["AverageNs"]) / 1e6
    cnt = defaultdict(list)
    for f in glob.glob(f"{case}p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "enrich_kernel" in r["Kernel_Name"]:
                cnt[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in cnt.items()}
    alg = S * 10_000 * 152
    fetch = m.get("FETCH_SIZE", 0) * 1024 * 2
    write = m.get("WRITE_SIZE", 0) * 1024
    hits, miss = m.get("TCC_HIT_sum", 0), m.get("TCC_MISS_sum", 0)
    s = {"symbols": S, "kernel_ms": dur, "frac": alg / (dur * 1e-3) / 8e12 if dur else None,
         "traffic_over_alg": (fetch + write) / alg, "l2_hit_rate": hits / (hits + miss) if hits + miss else None,
         "wr_credit_stall_per_launch": m.get("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"),
         "rd_credit_stall_per_launch": m.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"),
         "wait_share": m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"] if m.get("SQ_WAVE_CYCLES") else None,
         "clock_ghz": m["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e-3) / 1e9 if dur and m.get("GRBM_GUI_ACTIVE") else None,
         "counters": m}
    out[name] = s
    per = lambda x: x / (S * 10_000) if x is not None else float("nan")  # noqa: E731
    print(f"{name:20s} {dur or 0:8.3f} ms  frac {s['frac'] or 0:.3f}  traffic/alg {s['traffic_over_alg']:.3f}  "
          f"L2 hit {s['l2_hit_rate'] or 0:.3f}  wr stall/candle {per(s['wr_credit_stall_per_launch']):.3f}  "
          f"rd stall/candle {per(s['rd_credit_stall_per_launch']):.3f}  wait {s['wait_share'] or 0:.3f}  "
          f"clk {s['clock_ghz'] or 0:.2f} GHz")
json.dump(out, open(f"{d}/shard_summary.json", "w"), indent=1)
