"""Per-kernel launch-duration summary from a rocprofv3 kernel trace
(run_kernel_trace.csv), split by grid size, for one kernel name substring:
the average duration at the headline grid is what bench.py's roofline
kernel_ms must agree with. Usage: python tools/trace_summary.py <trace_dir> <kernel>"""
import csv
import glob
import sys
from collections import defaultdict

d, kern = sys.argv[1], sys.argv[2]
rows = defaultdict(list)
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        rows[grid].append(dur)
for g, v in sorted(rows.items(), key=lambda kv: -len(kv[1])):
    v.sort()
    print(f"{kern} grid_x={g}: launches={len(v)} mean_ms={sum(v) / len(v) / 1e6:.4f} "
          f"min_ms={v[0] / 1e6:.4f} median_ms={v[len(v) // 2] / 1e6:.4f} max_ms={v[-1] / 1e6:.4f}")
