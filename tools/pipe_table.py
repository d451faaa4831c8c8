"""Summarise gpurun_out/pipe_<name>/run_kernel_stats.csv (tools/pipeline_profile.sh):
ms per pipeline iteration (3 iterations traced) by kernel family."""
import csv
import sys

names = sys.argv[1:] or ["activity_burst", "pump_score", "failed_spike", "top_gainer", "adx", "zscore", "wilder_rsi"]
for p in names:
    rows = list(csv.DictReader(open(f"gpurun_out/pipe_{p}/run_kernel_stats.csv")))
    fam = {}
    for r in rows:
        n = r["Name"]
        k = ("fused(native)" if n.startswith("bq_fk") else "fused(interp)" if "fused_kernel" in n else
             "replay" if "replay" in n else "rank" if "rank" in n else "torch" if "at::native" in n else
             n.split("(")[0].replace("void ", "").replace("bq::", ""))
        fam[k] = fam.get(k, 0.0) + float(r["TotalDurationNs"]) / 3e6
    tot = sum(fam.values())
    print(f"{p:15s} total {tot:7.3f} ms  " + "  ".join(f"{k} {v:.3f}" for k, v in sorted(fam.items(), key=lambda x: -x[1])))
